# Round-3: k_sspp_c2f shape sweep with the FP64 sampler and job-level pair culling.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03e}; O=$R/gpurun_out/$TAG; mkdir -p $O
run_dropin() { local lab=$1; shift
  env "$@" timeout -k 10 120 python bench.py --mode dropin --steps 200 --warmup 20 > $O/dropin_$lab.json 2>>$O/err.log || { echo "FAIL dropin $lab"; exit 1; }
  echo "dropin $lab $(python -c "import json;d=json.load(open('$O/dropin_$lab.json'));print('plan us',round(d['value'],1),'kernel us',round(d['isolated_step_kernel_us'],1))")"; }
run_short() { local lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/short_$lab.json 2>>$O/err.log || { echo "FAIL short $lab"; exit 1; }
  echo "short20 $lab $(python -c "import json;d=json.load(open('$O/short_$lab.json'));print(round(d['value']/1e6,1),'M/s', round(d['ms_per_step']*1e3,2),'us/step kernel_us',round(d['roofline']['kernel_us'],1))")"; }
run_dropin empty SSPP_KERNEL=1 SSPP_ABLATE=64
for cfg in "64 4" "64 16" "64 64" "128 32" "128 64" "256 16" "256 32" "256 64"; do set -- $cfg
  run_dropin c2f_nt$1_g$2 SSPP_KERNEL=1 SSPP_NT=$1 SSPP_G1=$2; done
for cfg in "64 4" "64 8" "128 8" "256 16"; do set -- $cfg
  run_short c2f_nt$1_g$2 SSPP_KERNEL=1 SSPP_NT=$1 SSPP_G1=$2; done
run_short empty SSPP_KERNEL=1 SSPP_ABLATE=64
echo DONE
