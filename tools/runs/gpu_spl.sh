# Steps per launch and steps per executor call of the long robocrane run:
#   bash tools/runs/gpu_spl.sh TAG "chunk:spl ..."
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
TAG=${1:-spl}; O=gpurun_out/$TAG; mkdir -p $O
for cs in ${2:-64:32 128:32 80:40 160:40 120:40}; do
  c=${cs%%:*}; s=${cs##*:}
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --chunk $c --steps-per-launch $s > $O/c${c}_s$s.json 2> $O/c${c}_s$s.log || exit 1
  python3 -c "import json;d=json.load(open('$O/c${c}_s$s.json'));print('chunk $c spl $s: %.1f M cand/s kernel_us %.1f (%d cand/launch) frac_fp64 %s' % (d['value']/1e6, d['roofline']['kernel_us'], d['roofline']['candidates_per_launch'], d['roofline_fp64']['frac']))"
done
