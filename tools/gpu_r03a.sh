# Round-3 probe: single-step latency of the current k_sspp_c2f under lane-group shapes
# (candidates per one-wave workgroup = 64 / G1), and the driver-shaped 20-step run.
#   gpurun -- bash tools/gpu_r03a.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03a}; O=$R/gpurun_out/$TAG; mkdir -p $O
for g1 in 4 16 64; do
  SSPP_G1=$g1 timeout -k 10 120 python bench.py --mode dropin --steps 300 --warmup 30 > $O/dropin_g$g1.json 2>>$O/err.log || { echo "FAIL dropin $g1"; exit 1; }
  echo "g1 $g1 $(python -c "import json;d=json.load(open('$O/dropin_g$g1.json'));print('plan us',round(d['value'],1),'kernel us',round(d['isolated_step_kernel_us'],1))")"
done
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/short$rep.json 2>>$O/err.log || { echo "FAIL short"; exit 1; }
  echo "short20 $(python -c "import json;d=json.load(open('$O/short$rep.json'));print(round(d['value']/1e6,1),'M/s', round(d['ms_per_step']*1e3,2),'us/step')")"
done
SSPP_ABLATE=64 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/short_empty.json 2>>$O/err.log || { echo "FAIL empty"; exit 1; }
echo "short20 empty-body $(python -c "import json;d=json.load(open('$O/short_empty.json'));print(round(d['ms_per_step']*1e3*20,1),'us region')")"
echo DONE
