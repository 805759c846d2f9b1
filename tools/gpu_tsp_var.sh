# Compare library variants on the TSP benches: bash tools/gpu_tsp_var.sh TAG NAME...
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=$R/sspp_amd/lib/variants/libsspp_$v.so
  for c in stacking multigoal; do
    SSPP_LIB_PATH=$lib timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/b.json 2>>$O/err.log || exit 1
    echo "$v $c $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,2),'M/s k_tsp us',round(d['roofline']['kernel_us'],2))")"
  done
done
