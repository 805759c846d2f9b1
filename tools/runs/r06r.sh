# round 6: hull pad through scalar registers, lane indices laundered at the split tail (split instance scratch 0): tests and lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06r; mkdir -p $O; cd $R
timeout -k 10 300 python3 -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for i in 1 2 3; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/short20_$i.json 2> $O/short20_$i.log || { tail -20 $O/short20_$i.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/short20_$i.json'));print('short20: %.1f M cand/s kernel_us %.1f parity %s' % (d['value']/1e6, d['roofline']['kernel_us'], (d['cpu_baseline'] or {}).get('parity', {}).get('record_identical')))"
done
timeout -k 10 240 python3 bench.py --no-cpu-baseline > $O/default.json 2> $O/default.log || { tail -20 $O/default.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/default.json'));print('default: %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
timeout -k 10 180 python3 bench.py --mode dropin --steps 400 --warmup 50 > $O/dropin.json 2> $O/dropin.log || { tail -20 $O/dropin.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/dropin.json'));print('dropin: %.1f us/plan isolated %.1f max cold %.0f' % (d['value'], d['isolated_step_kernel_us'], d['first_call_us_max']))"
for c in stacking multigoal; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/$c.json 2> $O/$c.log || { tail -20 $O/$c.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$c.json'));print('$c: %.2f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
