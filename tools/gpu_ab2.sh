set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/ab2; mkdir -p $O; rm -f $O/*.json*
for m in 0 8 16 24 32 2 6 7; do
  SSPP_ABLATE=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1000 --warmup 50 --roofline-launches 50 > $O/b$m.json 2>>$O/err.log || exit 1
  echo "ablate $m $(python -c "import json;d=json.load(open('$O/b$m.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step', round(d['roofline']['kernel_us'],1))")"
done
cd /tmp && export TMPDIR=/tmp
for m in 0 8 16 24 32; do
SSPP_ABLATE=$m timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d $O/sq$m -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --roofline-launches 10 > $O/sq$m.log 2>&1 || exit 1
done
