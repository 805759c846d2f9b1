# k_tsp change check: TSP/CES GPU parity tests, then stacking + multi-goal benches.
#   gpurun --timeout 900 -- bash tools/gpu_tsp_ab.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-tspab}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in stacking multigoal; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/$c.json 2>>$O/err.log || { echo "BENCH $c FAILED"; tail -20 $O/err.log; exit 1; }
  echo "$c $(python -c "import json;d=json.load(open('$O/$c.json'));print(round(d['value']/1e6,2),'M/s k_tsp us',round(d['roofline']['kernel_us'],2))")"
done
