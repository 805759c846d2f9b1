# Upright cylinder-box mode: GPU tests (full), multi-goal / stacking benches generic vs upright,
# ICRA anytime latency.   gpurun --timeout 1100 -- bash tools/gpu_cbu.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-cbu}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for e in "SSPP_TSP_GENERIC=1" "SSPP_UP=1"; do
  for cfg in multigoal stacking; do
    timeout -k 10 200 env $e python bench.py --config $cfg --no-cpu-baseline > $O/b_$cfg.json 2>>$O/err.log || { echo "FAIL $e $cfg"; exit 1; }
    echo "$e $cfg $(python -c "import json;d=json.load(open('$O/b_$cfg.json'));print(round(d['value']/1e6,2),'M/s', round(d['roofline']['kernel_us'],1),'us/kernel')")"
  done
  timeout -k 10 300 env $e python bench.py --mode tsp-anytime --steps 5 --warmup 1 --no-cpu-baseline > $O/any.json 2>>$O/err.log || { echo "FAIL $e anytime"; exit 1; }
  echo "$e anytime $(python -c "import json;d=json.load(open('$O/any.json'));print(d['latency_us'], d['iterations_per_budget'])")"
done
timeout -k 10 200 python bench.py --mode dropin --no-cpu-baseline --steps 2000 --warmup 100 > $O/dropin.json 2>>$O/err.log || exit 1
python -c "import json;d=json.load(open('$O/dropin.json'));print('dropin', d['latency_us'], 'isolated', d['isolated_step_kernel_us'])"
echo DONE
