# PMC passes (one counter group per run): VALU mix, FP64 op counts, occupancy/stalls.
#   gpurun --timeout 600 -- bash tools/gpu_pmc.sh TAG [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-pmc}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps 64 --warmup 4 --roofline-launches 20 $*"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/p$i.log 2>&1 || { echo "PMC pass $i FAILED"; tail -5 $O/p$i.log; exit 1; }
done
echo PMC DONE
