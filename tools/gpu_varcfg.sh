# Compare library variants on one bench config: bash tools/gpu_varcfg.sh TAG CONFIG NAME... (base = main lib)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=$1; CFG=$2; shift 2; O=$R/gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=$R/sspp_amd/lib/variants/libsspp_$v.so
  SSPP_LIB_PATH=$lib timeout -k 10 200 python bench.py --config $CFG --no-cpu-baseline --roofline-launches 50 > $O/b.json 2>>$O/err.log || exit 1
  echo "$v $CFG $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step', round(d['roofline']['kernel_us'],2), 'us/kernel')")"
done; done
