# k_tsp occupancy variants (SSPP_LIB_PATH) on the stacking and multi-goal benches.
#   gpurun -- bash tools/gpu_tsp_w.sh TAG variant...
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-tspw}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
for v in default "$@"; do
  L=""; [ "$v" != default ] && L="SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_$v.so"
  for cfg in stacking multigoal; do
    timeout -k 10 200 env $L python bench.py --config $cfg --no-cpu-baseline > $O/b.json 2>>$O/err.log || { echo "FAIL $v $cfg"; exit 1; }
    echo "$v $cfg $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,2),'M/s', round(d['roofline']['kernel_us'],1),'us/kernel')")"
  done
done
echo DONE
