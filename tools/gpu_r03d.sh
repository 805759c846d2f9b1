# Round-3: k_sspp_wq1/2 shape sweep (single-step latency and driver-shaped 20-step run) + a
# rocprofv3 kernel trace of both.
#   gpurun -- bash tools/gpu_r03d.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03d}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
run_dropin() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 120 python bench.py --mode dropin --steps 200 --warmup 20 > $O/dropin_$lab.json 2>>$O/err.log || { echo "FAIL dropin $lab"; exit 1; }
  echo "dropin $lab $(python -c "import json;d=json.load(open('$O/dropin_$lab.json'));print('plan us',round(d['value'],1),'kernel us',round(d['isolated_step_kernel_us'],1))")"
}
run_short() {
  local lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/short_$lab.json 2>>$O/err.log || { echo "FAIL short $lab"; exit 1; }
  echo "short20 $lab $(python -c "import json;d=json.load(open('$O/short_$lab.json'));print(round(d['value']/1e6,1),'M/s', round(d['ms_per_step']*1e3,2),'us/step kernel_us',round(d['roofline']['kernel_us'],1))")"
}
run_dropin base
run_dropin cpw1_npg1 SSPP_WQ_CPW=1 SSPP_WQ_NPG=1
run_dropin cpw1_npg4 SSPP_WQ_CPW=1 SSPP_WQ_NPG=4
run_dropin cpw2 SSPP_WQ_CPW=2
run_dropin cpw4 SSPP_WQ_CPW=4
run_dropin cpw16 SSPP_WQ_CPW=16
run_dropin fp32 SSPP_SAMPLER=1
run_dropin g2_64 SSPP_WQ_G2=64
run_dropin g2_1024 SSPP_WQ_G2=1024
run_dropin c2f SSPP_KERNEL=1
run_short base
run_short cpw4 SSPP_WQ_CPW=4
run_short cpw16_npg2 SSPP_WQ_CPW=16 SSPP_WQ_NPG=2
run_short fp32 SSPP_SAMPLER=1
run_short c2f SSPP_KERNEL=1
run_short c2f_fp32 SSPP_KERNEL=1 SSPP_SAMPLER=1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_dropin -o run -- python bench.py --mode dropin --steps 50 --warmup 10 > $O/prof_dropin.log 2>&1 || { echo "FAIL prof dropin"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_short -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --roofline-launches 20 > $O/prof_short.log 2>&1 || { echo "FAIL prof short"; exit 1; }
find $O/prof_dropin $O/prof_short -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 $f | head -8; done
echo DONE
