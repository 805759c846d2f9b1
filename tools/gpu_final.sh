# Last check of the committed tree: full GPU tests, smoke(), the driver's default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-final}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; echo "FAIL pytest"; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; echo "FAIL smoke"; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2>>$O/err.log || { echo "FAIL bench"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_default.json'));print('default bench', round(d['value']/1e6,1), 'M/s', d['steps'], 'steps', 'frac', round(d['roofline']['frac'],4), 'traffic', d['roofline'].get('traffic'), 'cpu', d['cpu_baseline']['value'])"
echo DONE
