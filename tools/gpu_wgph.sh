# Per-phase shader clocks of the driver-shaped launch (wgt variant), G1 = 4 and 8
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/wgph; mkdir -p $O
for g in 4 8; do
  SSPP_G1=$g SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_wgt.so timeout -k 10 120 python tools/wg_timing.py 20 $O/wg20_g$g.json > $O/wg20_g$g.log 2>&1 || { echo "WG FAILED"; tail -5 $O/wg20_g$g.log; exit 1; }
  python -c "import json;d=json.load(open('$O/wg20_g$g.json'));print($g, {k:d[k] for k in ['span_us','dur_us_pcts','concurrency_at','phase_clocks_mean']}); print(d['phase_clocks_by_survivors'])"
done
