set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $R/gpurun_out/pmc1 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --roofline-launches 5 > $R/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM -d $R/gpurun_out/pmc2 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --roofline-launches 5 > $R/gpurun_out/pmc2.log 2>&1 || exit 1
