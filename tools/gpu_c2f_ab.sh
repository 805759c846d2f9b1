# c2f change check: all GPU parity tests, then the robocrane bench.
#   gpurun --timeout 900 -- bash tools/gpu_c2f_ab.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-c2fab}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/robocrane_$i.json 2>>$O/err.log || { echo "BENCH FAILED"; tail -20 $O/err.log; exit 1; }
  echo "robocrane $(python -c "import json;d=json.load(open('$O/robocrane_$i.json'));print(round(d['value']/1e6,1),'M/s c2f us',round(d['roofline']['kernel_us'],2))")"
done
