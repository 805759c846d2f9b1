# Iteration check: GPU tests (optionally a -k filter), smoke, the driver-shaped bench, a long
# bench and the drop-in latency bench.   gpurun -- bash tools/gpu_check.sh TAG ["-k expr"]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-chk}; K=${2:-}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $O/gpu_tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_short_$i.json 2> $O/bench_short_$i.err || { echo "BENCH FAILED"; tail -20 $O/bench_short_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_short_$i.json'));print('short', round(d['value']/1e6,1), 'M/s', d['roofline']['kernel_us'], 'us/kernel', 'cpu', round(d['cpu_baseline']['value']/1e6,3), round(d['cpu_baseline']['scoring_only_value']/1e6,3))"
done
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_long.json 2> $O/bench_long.err || { echo "BENCH LONG FAILED"; tail -20 $O/bench_long.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_long.json'));print('long', round(d['value']/1e6,1), 'M/s')"
timeout -k 10 200 python bench.py --mode dropin --steps 2000 --warmup 50 > $O/bench_dropin.json 2> $O/bench_dropin.err || { echo "DROPIN FAILED"; tail -20 $O/bench_dropin.err; exit 1; }
cat $O/bench_dropin.json
timeout -k 10 200 python bench.py --config stacking --no-cpu-baseline > $O/bench_stacking.json 2> $O/bench_stacking.err || { echo "STACKING FAILED"; tail -20 $O/bench_stacking.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_stacking.json'));print('stacking', round(d['value']/1e6,1), 'M/s')"
timeout -k 10 200 python bench.py --config multigoal --no-cpu-baseline > $O/bench_multigoal.json 2> $O/bench_multigoal.err || { echo "MULTIGOAL FAILED"; tail -20 $O/bench_multigoal.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_multigoal.json'));print('multigoal', round(d['value']/1e6,1), 'M/s')"
echo DONE
