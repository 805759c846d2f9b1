# robocrane throughput (native executor) + ablations; usage: bash tools/gpu_quick.sh TAG [ablate masks...]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-quick}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O; rm -f $O/*.json*
for m in 0 "$@"; do for spl in 8; do
  SSPP_ABLATE=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4096 --warmup 64 --steps-per-launch $spl --roofline-launches 50 > $O/b.json 2>>$O/err.log || exit 1
  echo "ablate $m spl $spl $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step', round(d['roofline']['kernel_us'],2), 'us/kernel')")"
done; done
