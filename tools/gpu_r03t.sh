# Where a c2f workgroup's time goes (WG-timing variant: per-phase shader clocks) at the driver's
# 20-step shape and the single-step shape, plus VALU instruction counts per ablation.
#   gpurun --timeout 900 -- bash tools/gpu_r03t.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03t}; O=$R/gpurun_out/$TAG; mkdir -p $O
for st in 20 1; do
  SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_wgt.so timeout -k 10 120 python tools/wg_timing.py $st $O/wg$st.json > $O/wg$st.log 2>&1 || { echo "WG FAILED"; tail -5 $O/wg$st.log; exit 1; }
  python -c "import json;d=json.load(open('$O/wg$st.json'));print($st, {k:d[k] for k in ['span_us','dur_us_pcts','concurrency_at','phase_clocks_mean']}); print(d['phase_clocks_by_survivors'])"
done
cd /tmp && export TMPDIR=/tmp
for m in 0 1 8 2 4; do
  SSPP_ABLATE=$m timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/ab$m -o run --output-format csv -- python3 $R/bench.py --steps 64 --warmup 4 --no-cpu-baseline --roofline-launches 10 > $O/ab$m.log 2>&1 || { echo "PMC $m FAILED"; tail -5 $O/ab$m.log; exit 1; }
  echo "ablate $m: $(tail -c 300 $O/ab$m.log | head -c 300)"
done
echo DONE
