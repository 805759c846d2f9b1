# Launch-shape A/B for the robocrane bench: steps per launch x streams, at the driver's
# --steps 20 --warmup 5 and at a long run; then c2f occupancy variants (SSPP_LIB_PATH).
#   gpurun -- bash tools/gpu_launch_ab.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-lab}; O=$R/gpurun_out/$TAG; mkdir -p $O
one() {  # label, extra env, bench args...
  local lab=$1; shift
  timeout -k 10 120 env $ENVX python bench.py --no-cpu-baseline --roofline-launches 20 $BARGS > $O/b.json 2>>$O/err.log || { echo "FAIL $lab"; exit 1; }
  echo "$lab $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step', round(d['roofline']['kernel_us'],2), 'us/kernel')")"
}
for spl in 8 16 20 32 64; do for ns in 1 2 4; do
  for rep in 1 2; do ENVX="" BARGS="--steps 20 --warmup 5 --steps-per-launch $spl --streams $ns" one "short spl=$spl ns=$ns"; done
  ENVX="" BARGS="--steps 4096 --warmup 64 --steps-per-launch $spl --streams $ns" one "long  spl=$spl ns=$ns"
done; done
for v in w4 w5 w6; do
  for spl in 8 32; do
    ENVX="SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_$v.so" BARGS="--steps 20 --warmup 5 --steps-per-launch $spl --streams 4" one "short $v spl=$spl"
    ENVX="SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_$v.so" BARGS="--steps 4096 --warmup 64 --steps-per-launch $spl --streams 4" one "long  $v spl=$spl"
  done
done
echo DONE
