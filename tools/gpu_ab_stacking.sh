set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/abs; mkdir -p $O
for v in default bb bb4 default; do
  L=""; [ "$v" != default ] && L="SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_$v.so"
  timeout -k 10 200 env $L python bench.py --config stacking --steps 256 --warmup 8 --no-cpu-baseline > $O/b.json 2>>$O/err.log || { echo "FAIL $v"; tail -5 $O/err.log; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s', round(d['roofline']['kernel_us'],1),'us/kernel')")"
done
SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_bb.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "stacking" --timeout 120 --timeout-method thread 2>&1 | tail -2
