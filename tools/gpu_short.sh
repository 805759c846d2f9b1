# The driver's short run (--steps 20 --warmup 5) under several launch splits.
#   gpurun -- bash tools/gpu_short.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-short}; O=$R/gpurun_out/$TAG; mkdir -p $O
for spl in 20 10 5 4 2; do
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --steps-per-launch $spl > $O/b.json 2>>$O/err.log || { echo "FAIL $spl"; exit 1; }
    echo "spl $spl $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s')")"
  done
done
for st in 8; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --steps-per-launch 3 --streams $st > $O/b.json 2>>$O/err.log || { echo "FAIL st$st"; exit 1; }
    echo "streams $st spl 3 $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s')")"
done
echo DONE
