# GPU tests, then robocrane long + driver-shaped short benches per library variant.
#   gpurun -- bash tools/gpu_ab_c2f.sh TAG variant...
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-abc}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for v in default "$@"; do
  L=""; [ "$v" != default ] && L="SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_$v.so"
  for a in "" "--steps 20 --warmup 5" "" "--steps 20 --warmup 5"; do
    timeout -k 10 200 env $L python bench.py --no-cpu-baseline $a > $O/b.json 2>>$O/err.log || { echo "FAIL $v"; exit 1; }
    echo "$v [$a] $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s', round(d['roofline']['kernel_us'],1),'us/kernel')")"
  done
done
echo DONE
