# Shape / occupancy sweep of the driver-shaped robocrane run (bench.py --steps 20 --warmup 5)
# and the long run: SHAPES="auto 64x4 ..." bash tools/runs/gpu_shapes.sh TAG [variant libs...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-shapes}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
one() {  # name, extra args...
  local n=$1; shift
  timeout -k 10 120 python3 bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.log || { tail -5 $O/$n.log; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/$n.json'));c=d['config'];print('%-28s %8.1f M/s  %7.2f us/step  kernel %6.1f us  %s %s' % ('$n', d['value']/1e6, d['ms_per_step']*1e3, d['roofline']['kernel_us'], c.get('shape'), c.get('library','')))"
}
for s in ${SHAPES:-auto 64x4 64x3 64x8 64x16}; do
  A=""; [ $s != auto ] && A="--shape $s"
  for r in 1 2; do one short20_${s}_$r --gpus 1 --steps 20 --warmup 5 $A; done
  one long_${s} --steps 2048 --warmup 64 $A
done
for v in "$@"; do
  for r in 1 2; do SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_$v.so one short20_lib${v}_$r --gpus 1 --steps 20 --warmup 5; done
  SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_$v.so one long_lib$v --steps 2048 --warmup 64
done
echo DONE
