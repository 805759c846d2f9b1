set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcab; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in 0 1 2 4 7; do
SSPP_ABLATE=$m timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d $O/sq$m -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --roofline-launches 10 > $O/sq$m.log 2>&1 || exit 1
done
