# Default hit-rate pair order: full GPU tests, smoke, job-create host cost, bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-order2}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 120 python tools/job_create_time.py > $O/create.log 2>&1 || { tail $O/create.log; exit 1; }
cat $O/create.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s20.json 2>>$O/err.log || exit 1
  echo "short20 $(python -c "import json;d=json.load(open('$O/s20.json'));print(round(d['value']/1e6,1))")"
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2>>$O/err.log || exit 1
cat $O/bench_default.json
echo DONE
