# Round-3: SamplingPathPlanner latency/throughput snapshot + kernel traces of the drop-in plan()
# loop and the driver-shaped 20-step run.
#   gpurun -- bash tools/gpu_r03j.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03j}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; echo "FAIL pytest"; exit 1; }
  tail -1 $O/pytest.log
fi
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/short_$i.json 2>>$O/err.log || { echo "FAIL short"; exit 1; }
  python -c "import json;d=json.load(open('$O/short_$i.json'));print('short20', round(d['value']/1e6,1),'M/s', round(d['ms_per_step']*1e3,2),'us/step')"
done
timeout -k 10 200 python bench.py > $O/default.json 2>>$O/err.log || { echo "FAIL default"; exit 1; }
python -c "import json;d=json.load(open('$O/default.json'));print('default', round(d['value']/1e6,1),'M/s kernel_us', round(d['roofline']['kernel_us'],1), 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 120 python bench.py --mode dropin --steps 300 --warmup 30 > $O/dropin.json 2>>$O/err.log || { echo "FAIL dropin"; exit 1; }
python -c "import json;d=json.load(open('$O/dropin.json'));print('dropin', round(d['value'],1),'us/plan', d['latency_us'], 'isolated', round(d['isolated_step_kernel_us'],1))"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dropin -o run -- python bench.py --mode dropin --steps 100 --warmup 10 > $O/prof_dropin.log 2>&1 || { echo "FAIL prof dropin"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_short -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --roofline-launches 20 > $O/prof_short.log 2>&1 || { echo "FAIL prof short"; exit 1; }
find $O/prof_dropin $O/prof_short -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 $f | head -6; done
echo DONE
