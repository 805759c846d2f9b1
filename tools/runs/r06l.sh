# round 6: kDeep through scalar registers (multi-goal 11 -> 9 spilled VGPRs): TSP/CES parity, stacking and multi-goal lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06l; mkdir -p $O; cd $R
timeout -k 10 300 python3 -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for c in stacking multigoal stacking multigoal; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.log || { tail -20 $O/bench_$c.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c: %.2f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
