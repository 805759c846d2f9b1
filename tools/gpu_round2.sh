# Round evidence, part 1: GPU tests, smoke, benches (driver-shaped and per config), the
# rocprofv3 --kernel-trace --stats summary of the default bench, and a kernel + HIP runtime
# trace of the driver's short run (bench.py --steps 20 --warmup 5).
#   gpurun --timeout 1100 -- bash tools/gpu_round2.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r02}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
b() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/bench_$name.json 2> $O/bench_$name.err \
        || { echo "BENCH $name FAILED"; tail -20 $O/bench_$name.err; exit 1; }; echo "$name $(head -c 300 $O/bench_$name.json)"; }
b robocrane
b robocrane_short --steps 20 --warmup 5
b stacking --config stacking
b multigoal --config multigoal
b config4_shard --batch 32768 --waypoints 256 --steps 256 --no-cpu-baseline
b dropin --mode dropin --steps 2000 --warmup 50
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { echo "PROF FAILED"; tail -5 $O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $O/trace20 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace20.log 2>&1 || { echo "TRACE20 FAILED"; tail -5 $O/trace20.log; exit 1; }
for c in stacking multigoal; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu-baseline > $O/prof_$c.log 2>&1 || { echo "PROF $c FAILED"; tail -5 $O/prof_$c.log; exit 1; }
done
echo DONE
