# GPU tests only (optionally a -k filter): gpurun --timeout 900 -- bash tools/gpu_tests.sh TAG [KEXPR]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-tests}; O=$R/gpurun_out/$TAG; mkdir -p $O
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1
rc=$?; tail -30 $O/gpu_tests.log; exit $rc
