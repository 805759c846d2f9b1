# Hit-rate pair order (SSPP_PAIR_ORDER=2) A/B: parity tests under it, 20-step and long runs
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-order}; O=$R/gpurun_out/$TAG; mkdir -p $O
SSPP_PAIR_ORDER=2 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "robocrane or executor or fused or cylinder or dropin" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for e in "X=0" "SSPP_PAIR_ORDER=2"; do
  for rep in 1 2 3; do
    timeout -k 10 200 env $e python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s20.json 2>>$O/err.log || { echo "FAIL $e"; exit 1; }
    echo "[$e] short20 $(python -c "import json;d=json.load(open('$O/s20.json'));print(round(d['value']/1e6,1))")"
  done
  timeout -k 10 200 env $e python bench.py --steps 2048 --warmup 64 --no-cpu-baseline > $O/long.json 2>>$O/err.log || { echo "FAIL $e long"; exit 1; }
  echo "[$e] long $(python -c "import json;d=json.load(open('$O/long.json'));print(round(d['value']/1e6,1), round(d['roofline']['kernel_us'],1))")"
  timeout -k 10 200 env $e python bench.py --mode dropin --no-cpu-baseline --steps 1000 --warmup 100 > $O/dropin.json 2>>$O/err.log || exit 1
  echo "[$e] dropin $(python -c "import json;d=json.load(open('$O/dropin.json'));print(round(d['latency_us']['median'],1), round(d['isolated_step_kernel_us'],1))")"
done
echo DONE
