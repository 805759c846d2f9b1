# Single-plan latency: c2f parity tests, drop-in plan() latency + isolated step, WG phase clocks.
#   gpurun -- bash tools/gpu_lat.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-lat}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "robocrane or cylinder or fused or executor or hull or dropin or planner or score_ctrl" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python bench.py --mode dropin --no-cpu-baseline --steps 2000 --warmup 100 > $O/dropin.json 2>>$O/err.log || exit 1
python -c "import json;d=json.load(open('$O/dropin.json'));print('dropin', d['latency_us'], 'isolated', d['isolated_step_kernel_us'])"
for rep in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s20.json 2>>$O/err.log || exit 1
python -c "import json;d=json.load(open('$O/s20.json'));print('short20', round(d['value']/1e6,1))"
done
SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_wgt.so timeout -k 10 120 python tools/wg_timing.py 1 $O/wg1.json > $O/wg1.log 2>&1 || { tail -5 $O/wg1.log; exit 1; }
python -c "import json;d=json.load(open('$O/wg1.json'));print({k:d[k] for k in ['span_us','dur_us_pcts','dur_us_by_survivors']}); print(d['phase_clocks_by_survivors'])"
echo DONE
