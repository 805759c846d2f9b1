# Round-3 A/B of variant libraries (SSPP_LIB_PATH): driver-shaped 20-step runs, a long run and
# the single-step drop-in latency, interleaved over variants.
#   gpurun -- bash tools/gpu_ab6.sh TAG name1 name2 ...
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    export SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_$v.so
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s_$v.json 2>>$O/err.log || { echo "FAIL $v"; exit 1; }
    s=$(python -c "import json;d=json.load(open('$O/s_$v.json'));print(round(d['value']/1e6,1))")
    timeout -k 10 120 python bench.py --steps 1024 --no-cpu-baseline > $O/l_$v.json 2>>$O/err.log || { echo "FAIL $v"; exit 1; }
    l=$(python -c "import json;d=json.load(open('$O/l_$v.json'));print(round(d['value']/1e6,1), round(d['roofline']['kernel_us'],1))")
    timeout -k 10 120 python bench.py --mode dropin --steps 200 --warmup 20 > $O/d_$v.json 2>>$O/err.log || { echo "FAIL $v"; exit 1; }
    d=$(python -c "import json;d=json.load(open('$O/d_$v.json'));print(round(d['value'],1), round(d['isolated_step_kernel_us'],1))")
    echo "$v short20 $s M/s | long $l | dropin $d"
  done
done
echo DONE
