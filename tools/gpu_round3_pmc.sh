# Round-3 PMC evidence, one counter group per run (never combined with a trace domain):
# HBM FETCH_SIZE / WRITE_SIZE, the FP64 instruction mix, and occupancy (the gfx950 derived
# MeanOccupancyPerCU = accumulate(SQ_LEVEL_WAVES, HIGH_RES) / GRBM_GUI_ACTIVE / CU_NUM, plus the
# wave-cycle / VALU counters) for the robocrane scorer and both TaskSpacePlanner configs.
#   gpurun --timeout 1100 -- bash tools/gpu_round3_pmc.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-r03pmc}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
OCC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE"
run() { local d=$1 grp=$2; shift 2; mkdir -p $O/$d
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $O/$d -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/$d.log 2>&1 \
    || { echo "PMC $d FAILED"; tail -5 $O/$d.log; exit 1; }; echo "ok $d"; }
RC="--steps 64 --warmup 4 --roofline-launches 20"
TS="--steps 4 --warmup 1 --roofline-launches 20"
run robocrane/pmc_fetch FETCH_SIZE $RC
run robocrane/pmc_write WRITE_SIZE $RC
run robocrane/p1 "$F64" $RC
run robocrane/occ/p1 "$OCC" $RC
run robocrane/occ/p2 MeanOccupancyPerCU $RC
for c in stacking multigoal; do
  run $c/pmc_fetch FETCH_SIZE --config $c $TS
  run $c/pmc_write WRITE_SIZE --config $c $TS
  run $c/p1 "$F64" --config $c $TS
  run $c/occ/p1 "$OCC" --config $c $TS
  run $c/occ/p2 MeanOccupancyPerCU --config $c $TS
done
echo DONE
