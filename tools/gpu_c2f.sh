set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/c2f; mkdir -p $O; rm -f $O/*.jsonl
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for k in 0 1; do for g in 8 16 32; do for ins in 0 1; do
  SSPP_KERNEL=$k SSPP_G1=$g SSPP_INSAMPLE=$ins timeout -k 10 120 python tools/ablate.py >> $O/ablate.jsonl 2>>$O/err.log || exit 1
done; done; done
for m in 2 4 6; do SSPP_ABLATE=$m timeout -k 10 120 python tools/ablate.py >> $O/ablate.jsonl 2>>$O/err.log || exit 1; done
cat $O/ablate.jsonl
