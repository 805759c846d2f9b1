# Phase-1 iteration cap A/B: parity tests, 20-step and long runs for SSPP_P1CAP = 0..3
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-cap}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "phase1_cap or executor or robocrane_sample" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in 0 1 2 3; do
  for rep in 1 2; do
    SSPP_P1CAP=$c timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s20.json 2>>$O/err.log || { echo "FAIL $c"; exit 1; }
    echo "cap $c short20 $(python -c "import json;d=json.load(open('$O/s20.json'));print(round(d['value']/1e6,1))")"
  done
  SSPP_P1CAP=$c timeout -k 10 200 python bench.py --steps 2048 --warmup 64 --no-cpu-baseline > $O/long.json 2>>$O/err.log || { echo "FAIL $c long"; exit 1; }
  echo "cap $c long $(python -c "import json;d=json.load(open('$O/long.json'));print(round(d['value']/1e6,1), round(d['roofline']['kernel_us'],1))")"
done
for c in 0 2; do
  SSPP_P1CAP=$c timeout -k 10 200 python bench.py --mode dropin --no-cpu-baseline --steps 1000 --warmup 100 > $O/dropin.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/dropin.json'));print('cap $c dropin', round(d['latency_us']['median'],1), 'isolated', round(d['isolated_step_kernel_us'],1))"
done
echo DONE
