# Round-3: latency benches only (drop-in plan(), ICRA anytime).
#   gpurun -- bash tools/gpu_lat.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-lat}; O=$R/gpurun_out/$TAG; mkdir -p $O
for i in 1 2; do
timeout -k 10 120 python bench.py --mode dropin --steps 300 --warmup 30 > $O/dropin_$i.json 2>>$O/err.log || { echo "FAIL dropin"; exit 1; }
python -c "import json;d=json.load(open('$O/dropin_$i.json'));print('dropin', round(d['value'],1),'us/plan', {k:round(v,1) for k,v in d['latency_us'].items()}, 'isolated', round(d['isolated_step_kernel_us'],1))"
done
timeout -k 10 200 python bench.py --mode tsp-anytime --steps 10 --no-cpu-baseline > $O/anytime.json 2>>$O/err.log || { echo "FAIL anytime"; exit 1; }
python -c "import json;d=json.load(open('$O/anytime.json'));print('anytime us/iter', round(d['value'],1), {k:round(v,1) for k,v in d['latency_us'].items()}, d['iterations_per_budget'])"
echo DONE
