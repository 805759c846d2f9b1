# Round-3: CES / drop-in hygiene checks + the ICRA anytime bench (+ kernel trace).
#   gpurun -- bash tools/gpu_r03h.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03h}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ces.py tests/test_dropin_sspp.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; echo "FAIL pytest"; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python bench.py --mode tsp-anytime --steps 10 --cpu-seconds 4 > $O/anytime.json 2>>$O/err.log || { echo "FAIL anytime"; exit 1; }
python -c "import json;d=json.load(open('$O/anytime.json'));print('anytime us/iter', round(d['value'],1), d['latency_us'], d['iterations_per_budget'], 'cpu us/iter', round(d['cpu_baseline']['value'],1))"
SSPP_CES_UNFUSED=1 timeout -k 10 200 python bench.py --mode tsp-anytime --steps 10 --no-cpu-baseline > $O/anytime_unfused.json 2>>$O/err.log || { echo "FAIL anytime unfused"; exit 1; }
python -c "import json;d=json.load(open('$O/anytime_unfused.json'));print('unfused us/iter', round(d['value'],1), d['latency_us'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_anytime -o run -- python bench.py --mode tsp-anytime --steps 3 --no-cpu-baseline --budgets-ms 20 > $O/prof_anytime.log 2>&1 || { echo "FAIL prof"; exit 1; }
find $O/prof_anytime -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 $f | head -12; done
echo DONE
