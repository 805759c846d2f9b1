# Round-3 final evidence on the final tree: GPU tests, every bench line, rocprofv3 kernel stats.
#   gpurun --timeout 1100 -- bash tools/gpu_r03f.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03f}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; echo "FAIL pytest"; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_short20.json 2>>$O/err.log || { echo "FAIL short20"; exit 1; }
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_short20_rep$rep.json 2>>$O/err.log || { echo "FAIL short20 rep"; exit 1; }
done
timeout -k 10 300 python bench.py --steps 4096 --warmup 64 --no-cpu-baseline > $O/bench_robocrane.json 2>>$O/err.log || { echo "FAIL long"; exit 1; }
timeout -k 10 200 python bench.py --mode dropin --no-cpu-baseline --steps 2000 --warmup 100 > $O/bench_dropin.json 2>>$O/err.log || { echo "FAIL dropin"; exit 1; }
for c in stacking multigoal; do
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2>>$O/err.log || { echo "FAIL $c"; exit 1; }
done
timeout -k 10 300 python bench.py --mode tsp-anytime --steps 10 --cpu-seconds 4 > $O/bench_anytime.json 2>>$O/err.log || { echo "FAIL anytime"; exit 1; }
python - <<PY
import json
for f in ["short20", "short20_rep1", "short20_rep2", "robocrane", "stacking", "multigoal"]:
    d = json.load(open("$O/bench_%s.json" % f)); r = d.get("roofline", {})
    print(f, round(d["value"] / 1e6, 1), "M/s", "kernel_us", round(r.get("kernel_us", 0), 1), "frac", round(r.get("frac", 0), 4))
d = json.load(open("$O/bench_dropin.json")); print("dropin", d["latency_us"], "isolated", d["isolated_step_kernel_us"])
d = json.load(open("$O/bench_anytime.json")); print("anytime", d["latency_us"], d["iterations_per_budget"])
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_short20 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_short20.log 2>&1 || { echo "FAIL prof short20"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_robocrane -o run -- python3 bench.py --steps 256 --warmup 16 --no-cpu-baseline > $O/prof_robocrane.log 2>&1 || { echo "FAIL prof long"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dropin -o run -- python3 bench.py --mode dropin --steps 300 --warmup 30 --no-cpu-baseline > $O/prof_dropin.log 2>&1 || { echo "FAIL prof dropin"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stacking -o run -- python3 bench.py --config stacking --steps 128 --no-cpu-baseline --roofline-launches 20 > $O/prof_stacking.log 2>&1 || { echo "FAIL prof stacking"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_multigoal -o run -- python3 bench.py --config multigoal --steps 16 --no-cpu-baseline --roofline-launches 5 > $O/prof_multigoal.log 2>&1 || { echo "FAIL prof multigoal"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_anytime -o run -- python3 bench.py --mode tsp-anytime --steps 3 --no-cpu-baseline --budgets-ms 20 > $O/prof_anytime.log 2>&1 || { echo "FAIL prof anytime"; exit 1; }
find $O -name "*kernel_stats.csv" | sort | while read f; do echo "== $f"; cut -d, -f1-4 $f | head -5 | cut -c1-150; done
echo DONE
