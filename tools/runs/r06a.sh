# round 6: split-queue hand-over / lost-work tests, timed-instance parity, short bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06a; mkdir -p $O; cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "split or multistep or step_executor" > $O/tests_split.txt 2>&1 || { tail -40 $O/tests_split.txt; exit 1; }
tail -3 $O/tests_split.txt
for i in 1 2 3; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_short20_$i.json 2> $O/bench_short20_$i.log \
    || { tail -20 $O/bench_short20_$i.log; exit 1; }
done
python3 - "$O" <<'PY'
import json, sys
for i in (1, 2, 3):
    d = json.load(open("%s/bench_short20_%d.json" % (sys.argv[1], i)))
    print("short20 rep %d: %.1f M cand/s, %.2f us/step, kernel_us %.1f, split_handoffs %s parity %s" % (
        i, d["value"] / 1e6, d["ms_per_step"] * 1e3, d["roofline"]["kernel_us"], d["config"].get("split_handoffs"),
        (d["cpu_baseline"] or {}).get("parity")))
PY
timeout -k 10 400 python3 -u -m pytest tests/test_ces.py -x -v --timeout 300 --timeout-method thread \
  -k "group_matches_oracle" > $O/tests_group.txt 2>&1 || { tail -40 $O/tests_group.txt; exit 1; }
tail -3 $O/tests_group.txt
echo DONE
