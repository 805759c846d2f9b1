# PMC evidence, one counter group per run (never combined with a trace domain): HBM FETCH_SIZE /
# WRITE_SIZE, the FP64 instruction mix, occupancy (gfx950 derived MeanOccupancyPerCU plus the
# wave-cycle / VALU counters) for the robocrane scorer (bench default and the config-4 shard)
# and both TaskSpacePlanner configs.  Fold with: python tools/update_latest.py gpurun_out/TAG profiles/PREFIX
#   gpurun --timeout 1100 -- bash tools/runs/gpu_pmc.sh TAG [configs...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-pmc}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
CFGS=${@:-robocrane robocrane_spl20 robocrane_b32768_w256 stacking multigoal}
cd /tmp && export TMPDIR=/tmp
F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
OCC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE"
run() { local d=$1 grp=$2; shift 2; mkdir -p $O/$d
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $O/$d -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/$d.log 2>&1 \
    || { echo "PMC $d FAILED"; tail -5 $O/$d.log; exit 1; }; echo "ok $d"; }
for c in $CFGS; do
  case $c in
    robocrane) A="--steps 80 --warmup 4 --roofline-launches 20";;
    robocrane_spl20) A="--steps 20 --warmup 5 --roofline-launches 20";;
    robocrane_b32768_w256) A="--batch 32768 --waypoints 256 --steps 80 --warmup 4 --roofline-launches 10";;
    *) A="--config $c --steps 4 --warmup 1 --roofline-launches 20";;
  esac
  run $c/pmc_fetch FETCH_SIZE $A
  run $c/pmc_write WRITE_SIZE $A
  run $c/p1 "$F64" $A
  run $c/occ/p1 "$OCC" $A
  run $c/occ/p2 MeanOccupancyPerCU $A
  run $c/util "VALUUtilization SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU" $A
done
echo DONE
