# 20-step run split over two streams with a different shape for the small launch
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-split}; O=$R/gpurun_out/$TAG; mkdir -p $O
run() { local lab=$1; shift; for rep in 1 2; do
  timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup 5 --no-cpu-baseline $ARGS > $O/s.json 2>>$O/err.log || { echo "FAIL $lab"; exit 1; }
  echo "$lab $(python -c "import json;d=json.load(open('$O/s.json'));print(round(d['value']/1e6,1))")"; done; }
ARGS="" run base X=0
ARGS="--streams 2 --steps-per-launch 16" run "16+4 default" X=0
ARGS="--streams 2 --steps-per-launch 16" run "16+4 64:16" SSPP_SMALL_SHAPE=64:16
ARGS="--streams 2 --steps-per-launch 16" run "16+4 64:8" SSPP_SMALL_SHAPE=64:8
ARGS="--streams 2 --steps-per-launch 16" run "16+4 128:32" SSPP_SMALL_SHAPE=128:32
ARGS="--streams 2 --steps-per-launch 16" run "16+4 256:64" SSPP_SMALL_SHAPE=256:64
ARGS="--streams 2 --steps-per-launch 17" run "17+3 64:16" SSPP_SMALL_SHAPE=64:16
echo DONE
