# Exploration: ablations (SSPP_ABLATE mask), occupancy variants, SQ counters.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/explore; mkdir -p $O; rm -f $O/*.jsonl
for m in 0 1 2 4 6; do
  SSPP_ABLATE=$m timeout -k 10 120 python tools/ablate.py >> $O/ablate.jsonl 2>>$O/err.log || exit 1
done
for cfg in robocrane stacking; do
  for lib in "" build/variants/libsspp_w3.so build/variants/libsspp_w2.so; do
    CONFIG=$cfg SSPP_LIB_PATH=$lib timeout -k 10 120 python tools/ablate.py >> $O/variants.jsonl 2>>$O/err.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/sq1 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --roofline-launches 10 > $O/sq1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --roofline-launches 10 > $O/sq2.log 2>&1 || exit 1
cat $O/ablate.jsonl $O/variants.jsonl
