# k_tsp upright specialisation: TSP parity tests, then stacking / multi-goal benches generic vs UP.
#   gpurun -- bash tools/gpu_up.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-up}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "tsp or stacking or ces or gripper" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for e in "SSPP_TSP_GENERIC=1" "SSPP_UP=1"; do
  for cfg in stacking multigoal; do
    timeout -k 10 200 env $e python bench.py --config $cfg --no-cpu-baseline > $O/b.json 2>>$O/err.log || { echo "FAIL $e $cfg"; exit 1; }
    echo "$e $cfg $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,2),'M/s', round(d['roofline']['kernel_us'],1),'us/kernel')")"
  done
done
echo DONE
