# robocrane parity (64x8 c2f) + the cylinder-box test on a dev variant, then the A/B bench
#   gpurun -- bash tools/gpu_ab_fix.sh TAG VARIANT variant...
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-abf}; V=$2; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_$V.so timeout -k 10 300 python -u -m pytest $(cat tools/dev_ids.txt) -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
shift
bash tools/gpu_ab_quick.sh $TAG "$@"
