# Multi-goal CES bench vs hardware queue count: gpurun --timeout 600 -- bash tools/gpu_mg_hwq.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/mghwq; mkdir -p $O; rm -f $O/*.json
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --config multigoal --no-cpu-baseline > $O/mg_$q.json 2>>$O/err.log || exit 1
  echo "hwq $q $(python -c "import json;d=json.load(open('$O/mg_$q.json'));print(round(d['value']/1e6,2),'M/s',round(d['ms_per_step']*1e3,1),'us/step k_tsp',round(d['roofline']['kernel_us'],1))")"
done
