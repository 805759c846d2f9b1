# round 6: the default long run at 20 steps per launch (split, one resident round) against 40 (unsplit, two rounds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06zb; mkdir -p $O; cd $R
timeout -k 10 300 python3 -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
for spl in 40 20 40 20; do
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps-per-launch $spl > $O/default_spl$spl.json 2> $O/default_spl$spl.log || { tail -20 $O/default_spl$spl.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/default_spl$spl.json'));print('spl $spl: %.1f M cand/s kernel_us %.1f split %s' % (d['value']/1e6, d['roofline']['kernel_us'], d['config'].get('split')))"
done
