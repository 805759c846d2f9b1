set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; echo "EXIT $?" >> gpurun_out/gpu_tests.log
for cfg in robocrane stacking; do
  for lib in "" build/variants/libsspp_w4.so build/variants/libsspp_w5.so; do
    CONFIG=$cfg SSPP_LIB_PATH=$lib timeout -k 10 120 python tools/ablate.py >> gpurun_out/variants.jsonl 2>>gpurun_out/variants.err || exit 1
  done
done
