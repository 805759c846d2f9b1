set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/hwq; mkdir -p $O; rm -f $O/*.json*
for q in 4 8 16; do for st in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu-baseline --streams $st --steps 1000 --warmup 50 --roofline-launches 50 > $O/b_${q}_${st}.json 2>>$O/err.log || exit 1
  echo "hwq $q streams $st $(python -c "import json;d=json.load(open('$O/b_${q}_${st}.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step')")"
done; done
