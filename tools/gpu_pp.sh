# k_tsp_pp (pair-split TaskSpacePlanner kernel): parity tests + anytime latency, pp on/off.
#   gpurun -- bash tools/gpu_pp.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-pp}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ces.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; echo "FAIL pytest"; exit 1; }
tail -1 $O/pytest.log
SSPP_TSP_PP=1 timeout -k 10 400 python -u -m pytest tests/test_ces.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tsp or ces or stacking or icra" > $O/pytest_pp1.log 2>&1 || { tail -40 $O/pytest_pp1.log; echo "FAIL pytest pp1"; exit 1; }
tail -1 $O/pytest_pp1.log
for v in 2 1 0; do
  SSPP_TSP_PP=$v timeout -k 10 200 python bench.py --mode tsp-anytime --steps 10 --no-cpu-baseline > $O/anytime_pp$v.json 2>>$O/err.log || { echo "FAIL anytime"; exit 1; }
  python -c "import json;d=json.load(open('$O/anytime_pp$v.json'));print('pp=$v anytime us/iter', round(d['value'],1), {k:round(v,1) for k,v in d['latency_us'].items()}, d['iterations_per_budget'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --mode tsp-anytime --steps 3 --no-cpu-baseline --budgets-ms 20 > $O/prof.log 2>&1 || { echo "FAIL prof"; exit 1; }
cut -d, -f1-4 $O/prof/run_kernel_stats.csv | head -8
echo DONE
