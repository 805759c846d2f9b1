# Full GPU tests on the current build, A/B bench vs variants, WG timeline of the short run.
#   gpurun -- bash tools/gpu_r2b.sh TAG variant...
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r2b}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/gpu_ab_quick.sh $TAG default "$@" || exit 1
SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_wgt.so timeout -k 10 120 python tools/wg_timing.py 20 $O/wg20.json > $O/wg20.log 2>&1 || { echo "WG FAILED"; tail -5 $O/wg20.log; exit 1; }
python -c "import json;d=json.load(open('$O/wg20.json'));print({k:d[k] for k in ['span_us','dur_us_pcts','start_us_pcts','end_us_pcts','concurrency_at']})"
