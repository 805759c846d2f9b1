# round 6: waypoint height from the recorded pose (stacking 15 -> 12 spilled VGPRs): GPU tests, TSP lines, WRITE_SIZE
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06p; mkdir -p $O; cd $R
timeout -k 10 300 python3 -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for c in stacking multigoal stacking multigoal; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.log || { tail -20 $O/bench_$c.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c: %.2f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
cd /tmp && export TMPDIR=/tmp
for c in stacking multigoal; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w_$c -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --config $c --steps 4 --warmup 1 --roofline-launches 20 > $O/w_$c.log 2>&1 || { tail -5 $O/w_$c.log; exit 1; }
done
echo DONE
