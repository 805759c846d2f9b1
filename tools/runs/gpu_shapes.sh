# Launch-shape sweep on the driver's command (the --shape tuning option):
#   bash tools/runs/gpu_shapes.sh TAG REPS shape...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-shapes}; N=${2:-2}; shift; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for r in $(seq 1 $N); do
  for s in "$@"; do
    timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --shape $s > $O/${s}_$r.json 2> $O/${s}_$r.log || { tail -5 $O/${s}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${s}_$r.json'));print('%-6s short20 %7.1f M kernel %5.1f us' % ('$s', d['value']/1e6, d['roofline']['kernel_us']))"
  done
done
echo DONE
