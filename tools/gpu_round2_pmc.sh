# Round evidence, part 2: PMC passes, one counter group per run (never combined with a trace
# domain): HBM FETCH_SIZE / WRITE_SIZE and the FP64 instruction mix for every config, and an
# occupancy / stall pass for the robocrane kernel.
#   gpurun --timeout 1100 -- bash tools/gpu_round2_pmc.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-r02pmc}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
OCC="SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
run() { local d=$1 grp=$2; shift 2; mkdir -p $O/$d
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $O/$d -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/$d.log 2>&1 \
    || { echo "PMC $d FAILED"; tail -5 $O/$d.log; exit 1; }; echo "ok $d"; }
RC="--steps 64 --warmup 4 --roofline-launches 20"
TS="--steps 4 --warmup 1 --roofline-launches 20"
run robocrane/pmc_fetch FETCH_SIZE $RC
run robocrane/pmc_write WRITE_SIZE $RC
run robocrane/p1 "$F64" $RC
for c in stacking multigoal; do
  run $c/pmc_fetch FETCH_SIZE --config $c $TS
  run $c/pmc_write WRITE_SIZE --config $c $TS
  run $c/p1 "$F64" --config $c $TS
done
C4="--batch 32768 --waypoints 256 --steps 64 --warmup 4 --roofline-launches 10"
run robocrane_b32768_w256/pmc_fetch FETCH_SIZE $C4
run robocrane_b32768_w256/pmc_write WRITE_SIZE $C4
run robocrane_b32768_w256/p1 "$F64" $C4
run robocrane/occ/p1 "$OCC" $RC
echo DONE
