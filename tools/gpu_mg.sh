# TaskSpacePlanner tests + multi-goal / stacking / anytime benches
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-mg}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "tsp or stacking or ces or gripper or icra" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for cfg in multigoal stacking; do
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline > $O/b_$cfg.json 2>>$O/err.log || { echo "FAIL $cfg"; exit 1; }
    echo "$cfg $(python -c "import json;d=json.load(open('$O/b_$cfg.json'));print(round(d['value']/1e6,2),'M/s', round(d['roofline']['kernel_us'],1),'us/kernel')")"
  done
done
timeout -k 10 300 python bench.py --mode tsp-anytime --steps 5 --warmup 1 --no-cpu-baseline > $O/any.json 2>>$O/err.log || { echo "FAIL anytime"; exit 1; }
echo "anytime $(python -c "import json;d=json.load(open('$O/any.json'));print(d['latency_us'], d['iterations_per_budget'])")"
echo DONE
