# Run-to-run spread of the driver's command (bench.py --gpus 1 --steps 20 --warmup 5), each in a
# fresh process as the driver runs it: bash tools/runs/gpu_repeat.sh TAG [N] [extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-repeat}; N=${2:-10}; shift; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/r$i.json 2> $O/r$i.log \
    || { tail -5 $O/r$i.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/r$i.json'));print('rep $i: %7.1f M/s %6.2f us/step enqueue %.1f us kernel %.1f us %s' % (d['value']/1e6, d['ms_per_step']*1e3, d['host_enqueue_ms']*1e3, d['roofline']['kernel_us'], d['config'].get('shape')))"
done
echo DONE
