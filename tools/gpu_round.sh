set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; echo "EXIT $?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench4.json 2> gpurun_out/bench4.err || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof4.log 2>&1
