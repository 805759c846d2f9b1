# Dev loop: focused GPU tests, then benches of the given configs.
#   gpurun --timeout 900 -- bash tools/gpu_dev.sh TAG "KEXPR" "config1 config2 ..."
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-dev}; O=$R/gpurun_out/$TAG; mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$2" > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
for c in $3; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { echo "BENCH $c FAILED"; tail -20 $O/bench_$c.err; exit 1; }
  cat $O/bench_$c.json; echo
done
