# Round-3: k_sspp_wq parity + latency/throughput probe.
#   gpurun -- bash tools/gpu_r03b.sh TAG [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03b}; O=$R/gpurun_out/$TAG; mkdir -p $O
K=${2:-}
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py ${K:+-k "$K"} > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; exit 1; }
timeout -k 10 120 python bench.py --mode dropin --steps 300 --warmup 30 > $O/dropin.json 2>>$O/err.log || { echo "FAIL dropin"; exit 1; }
echo "dropin $(python -c "import json;d=json.load(open('$O/dropin.json'));print('plan us',round(d['value'],1),'kernel us',round(d['isolated_step_kernel_us'],1))")"
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/short$rep.json 2>>$O/err.log || { echo "FAIL short"; exit 1; }
  echo "short20 $(python -c "import json;d=json.load(open('$O/short$rep.json'));print(round(d['value']/1e6,1),'M/s', round(d['ms_per_step']*1e3,2),'us/step kernel_us',round(d['roofline']['kernel_us'],1))")"
done
timeout -k 10 200 python bench.py --steps 2048 --no-cpu-baseline > $O/long.json 2>>$O/err.log || { echo "FAIL long"; exit 1; }
echo "long $(python -c "import json;d=json.load(open('$O/long.json'));print(round(d['value']/1e6,1),'M/s kernel_us',round(d['roofline']['kernel_us'],1))")"
echo DONE
