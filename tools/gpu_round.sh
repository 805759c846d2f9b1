# Round evidence: gpu tests, smoke, bench (N=1), rocprofv3 kernel-trace stats, PMC HBM passes.
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh [tag]
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
O=$R/gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --config stacking > $O/bench_stacking.json 2> $O/bench_stacking.err || { echo "BENCH2 FAILED"; tail -20 $O/bench_stacking.err; exit 1; }
timeout -k 10 300 python bench.py --config multigoal > $O/bench_multigoal.json 2> $O/bench_multigoal.err || { echo "BENCH3 FAILED"; tail -20 $O/bench_multigoal.err; exit 1; }
timeout -k 10 300 python bench.py --batch 32768 --waypoints 256 --steps 1024 --no-cpu-baseline > $O/bench_config4_shard.json 2> $O/bench_config4.err || { echo "BENCH4 FAILED"; tail -20 $O/bench_config4.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { echo "PROF FAILED"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 64 --warmup 4 --no-cpu-baseline --roofline-launches 20 > $O/pmc_fetch.log 2>&1 || { echo "PMC1 FAILED"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 64 --warmup 4 --no-cpu-baseline --roofline-launches 20 > $O/pmc_write.log 2>&1 || { echo "PMC2 FAILED"; exit 1; }
echo DONE
