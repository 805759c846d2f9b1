# One GPU evidence pass (run on the box via gpurun from the repo root):
#   bash tools/runs/gpu_check.sh TAG [tests|bench|configs|all]
# tests: pytest -m gpu + smoke(); bench: the driver's command (3 repeats), the default long run,
# the drop-in latency, and a rocprofv3 kernel trace of the driver-shaped run; configs: the
# stacking / multi-goal / config-4 / anytime lines and kernel statistics of the other runs.  Outputs under
# gpurun_out/TAG.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-run}; WHAT=${2:-all}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
    || { tail -30 $O/gpu_tests.txt; exit 1; }
  tail -3 $O/gpu_tests.txt
  timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
  cat $O/smoke.txt
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  for i in 1 2 3; do
    timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_short20_$i.json 2> $O/bench_short20_$i.log \
      || { tail -20 $O/bench_short20_$i.log; exit 1; }
  done
  python3 - "$O" <<'PY'
import json, sys
for i in (1, 2, 3):
    d = json.load(open("%s/bench_short20_%d.json" % (sys.argv[1], i)))
    print("short20 rep %d: %.1f M cand/s, %.2f us/step, kernel_us %.1f, cfg %s" % (
        i, d["value"] / 1e6, d["ms_per_step"] * 1e3, d["roofline"]["kernel_us"],
        {k: d["config"].get(k) for k in ("shape", "pair_order", "waypoint_order", "prepass_ms")}))
PY
  timeout -k 10 240 python3 bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.log || { tail -20 $O/bench_default.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default: %.1f M cand/s kernel_us %.1f frac %.4f' % (d['value']/1e6, d['roofline']['kernel_us'], d['roofline']['frac']))"
  timeout -k 10 180 python3 bench.py --mode dropin --steps 400 --warmup 50 > $O/bench_dropin.json 2> $O/bench_dropin.log || { tail -20 $O/bench_dropin.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_dropin.json'));print('dropin: %.1f us/plan isolated %.1f' % (d['value'], d['isolated_step_kernel_us']))"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/short20_trace -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/short20_trace.json 2> $O/short20_trace.log \
    || { tail -20 $O/short20_trace.log; exit 1; }
  cd $R
fi
if [ "$WHAT" = configs ] || [ "$WHAT" = all ]; then
  # the other bench lines: TaskSpacePlanner configs 3 and 5, the config-4 shard, the ICRA
  # anytime size; each with its rocprofv3 kernel statistics
  for c in stacking multigoal; do
    timeout -k 10 300 python3 bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.log || { tail -20 $O/bench_$c.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c: %.2f M cand/s kernel_us %.1f cpu %.3f M/s' % (d['value']/1e6, d['roofline']['kernel_us'], (d['cpu_baseline'] or {}).get('value', 0)/1e6))"
  done
  timeout -k 10 240 python3 bench.py --batch 32768 --waypoints 256 --no-cpu-baseline > $O/bench_config4.json 2> $O/bench_config4.log || { tail -20 $O/bench_config4.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_config4.json'));print('config4 shard: %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
  timeout -k 10 240 python3 bench.py --mode tsp-anytime > $O/bench_anytime.json 2> $O/bench_anytime.log || { tail -20 $O/bench_anytime.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_anytime.json'));print('anytime: %.1f us per plan' % d['value'])"
  cd /tmp && export TMPDIR=/tmp
  for c in stacking multigoal; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/${c}_trace -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu-baseline > $O/${c}_trace.json 2> $O/${c}_trace.log \
      || { tail -20 $O/${c}_trace.log; exit 1; }
  done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/default_trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/default_trace.json 2> $O/default_trace.log \
    || { tail -20 $O/default_trace.log; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/dropin_trace -o run --output-format csv -- python3 $R/bench.py --mode dropin --steps 400 --warmup 50 > $O/dropin_trace.json 2> $O/dropin_trace.log \
    || { tail -20 $O/dropin_trace.log; exit 1; }
  cd $R
fi
echo DONE
