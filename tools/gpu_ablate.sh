set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; echo "EXIT $?" >> gpurun_out/gpu_tests.log
for m in 0 1 2 4 6; do
  SSPP_ABLATE=$m timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate.jsonl 2>>gpurun_out/ablate.err || exit 1
done
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench5.json 2> gpurun_out/bench5.err || exit 1
