# Round-3: full GPU suite + TaskSpacePlanner benches (stacking, multi-goal) with kernel traces.
#   gpurun -- bash tools/gpu_r03i.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03i}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; echo "FAIL pytest"; exit 1; }
tail -2 $O/pytest.log
for c in stacking multigoal; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>>$O/err.log || { echo "FAIL bench $c"; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', round(d['value']/1e6,2),'M/s kernel_us',round(d['roofline']['kernel_us'],1))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stacking -o run -- python bench.py --config stacking --steps 128 --no-cpu-baseline --roofline-launches 20 > $O/prof_stacking.log 2>&1 || { echo "FAIL prof stacking"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_multigoal -o run -- python bench.py --config multigoal --steps 16 --no-cpu-baseline --roofline-launches 5 > $O/prof_multigoal.log 2>&1 || { echo "FAIL prof multigoal"; exit 1; }
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 $f | head -6; done
echo DONE
