set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/streams.jsonl
for cfg in robocrane stacking; do
  CONFIG=$cfg timeout -k 10 120 python tools/ablate.py >> gpurun_out/streams.jsonl 2>>gpurun_out/streams.err || exit 1
done
cat gpurun_out/streams.jsonl
