# Kernel-trace stats of the default-shape bench + robocrane PMC passes (hit pair order tree)
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-r03o}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/bench.py --steps 2048 --warmup 64 --no-cpu-baseline > $O/stats_bench.json 2>$O/stats.log || { tail -5 $O/stats.log; exit 1; }
cat $O/stats_bench.json
F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
run() { local d=$1 grp=$2; shift 2; mkdir -p $O/$d
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $O/$d -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/$d.log 2>&1 \
    || { echo "PMC $d FAILED"; tail -5 $O/$d.log; exit 1; }; echo "ok $d"; }
RC="--steps 64 --warmup 4 --roofline-launches 20"
run robocrane/pmc_fetch FETCH_SIZE $RC
run robocrane/pmc_write WRITE_SIZE $RC
run robocrane/p1 "$F64" $RC
echo DONE
