# tests (gpu) + per-config timings; usage: bash tools/gpu_quick.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/quick.jsonl
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for cfg in robocrane stacking; do
  CONFIG=$cfg timeout -k 10 120 python tools/ablate.py >> gpurun_out/quick.jsonl 2>>gpurun_out/quick.err || exit 1
done
cat gpurun_out/quick.jsonl
