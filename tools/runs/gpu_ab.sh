# A/B of variant builds on the driver's command (bench.py --gpus 1 --steps 20 --warmup 5) and the
# long run, interleaved: bash tools/runs/gpu_ab.sh TAG REPS variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-ab}; N=${2:-3}; shift; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for r in $(seq 1 $N); do
  for v in "$@"; do
    SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_$v.so timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.log || { tail -5 $O/${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'));print('%-8s short20 %7.1f M kernel %5.1f us' % ('$v', d['value']/1e6, d['roofline']['kernel_us']))"
  done
done
for v in "$@"; do
  SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_$v.so timeout -k 10 120 python3 bench.py --no-cpu-baseline > $O/${v}_long.json 2> $O/${v}_long.log || { tail -5 $O/${v}_long.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${v}_long.json'));print('%-8s long    %7.1f M kernel %5.1f us' % ('$v', d['value']/1e6, d['roofline']['kernel_us']))"
done
echo DONE
