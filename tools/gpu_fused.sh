set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for ins in 0 1; do
  SSPP_INSAMPLE=$ins CONFIG=robocrane timeout -k 10 120 python tools/ablate.py >> gpurun_out/fused.jsonl 2>>gpurun_out/fused.err || exit 1
done
CONFIG=stacking timeout -k 10 120 python tools/ablate.py >> gpurun_out/fused.jsonl 2>>gpurun_out/fused.err || exit 1
cat gpurun_out/fused.jsonl
