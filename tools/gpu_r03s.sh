# Session-start check: GPU tests + the driver-shaped bench + drop-in latency.
#   gpurun --timeout 1100 -- bash tools/gpu_r03s.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03s}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/short20_$rep.json 2>>$O/err.log || exit 1
  python -c "import json;d=json.load(open('$O/short20_$rep.json'));print('short20', round(d['value']/1e6,1),'M/s')"
done
timeout -k 10 200 python bench.py --mode dropin --no-cpu-baseline > $O/dropin.json 2>>$O/err.log || exit 1
tail -c 600 $O/dropin.json
echo DONE
