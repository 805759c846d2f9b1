# Compare library variants on the robocrane bench: bash tools/gpu_var.sh TAG NAME... ("" = main lib)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=$R/sspp_amd/lib/variants/libsspp_$v.so
  for spl in 1 8; do
    SSPP_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4096 --warmup 64 --steps-per-launch $spl --roofline-launches 50 > $O/b.json 2>>$O/err.log || exit 1
    echo "$v spl $spl $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step', round(d['roofline']['kernel_us'],2), 'us/kernel')")"
  done
done
