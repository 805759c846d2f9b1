# Drop-in latency breakdown: C-ABI plan() per call, the empty-kernel floor, the same with an
# empty scoring kernel (SSPP_ABLATE=64), python plan(), and single-step WG phase clocks.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-lat2}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 120 ./tools/plan_lat.bin | tee $O/plan_lat.txt || exit 1
SSPP_ABLATE=64 timeout -k 10 120 ./tools/plan_lat.bin | tail -1 | sed 's/^/[empty scorer] /' | tee -a $O/plan_lat.txt || exit 1
timeout -k 10 200 python bench.py --mode dropin --no-cpu-baseline --steps 2000 --warmup 100 > $O/dropin.json 2>>$O/err.log || exit 1
python -c "import json;d=json.load(open('$O/dropin.json'));print('dropin', d['latency_us'], 'isolated', d['isolated_step_kernel_us'])"
SSPP_ABLATE=64 timeout -k 10 200 python bench.py --mode dropin --no-cpu-baseline --steps 2000 --warmup 100 > $O/dropin_empty.json 2>>$O/err.log || exit 1
python -c "import json;d=json.load(open('$O/dropin_empty.json'));print('dropin empty scorer', d['latency_us'], 'isolated', d['isolated_step_kernel_us'])"
SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_wgt.so timeout -k 10 120 python tools/wg_timing.py 1 $O/wg1.json > $O/wg1.log 2>&1 || { tail -5 $O/wg1.log; exit 1; }
python -c "import json;d=json.load(open('$O/wg1.json'));print({k:d[k] for k in ['span_us','dur_us_pcts','dur_us_by_survivors']}); print(d['phase_clocks_by_survivors'])"
echo DONE
