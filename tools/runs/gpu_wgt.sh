# Per-workgroup timelines of k_sspp_c2f launches (needs the wgt variant: bash tools/build_variant.sh
# wgt "-DSSPP_DEV_ONLY -DSSPP_WG_TIMING"): bash tools/runs/gpu_wgt.sh TAG [steps...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-wgt}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for s in ${@:-20 5 32}; do
  SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_wgt.so timeout -k 10 120 python3 tools/wg_timing.py $s $O/wg$s.json > $O/wg$s.log 2>&1 || { tail -20 $O/wg$s.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/wg$s.json'));print($s, 'span', round(d['span_us'],1), 'dur pcts', {k: round(v,1) for k,v in d['dur_us_pcts'].items()}, 'by surv', {k: [v[0], round(v[1],1)] for k,v in d['dur_us_by_survivors'].items()}); print('  phases', {k: round(v) for k,v in d['phase_clocks_mean'].items()}); print('  end pcts', {k: round(v,1) for k,v in d['end_us_pcts'].items()})"
done
echo DONE
