# Sweep bench.py arguments on one config: bash tools/gpu_args.sh TAG CONFIG "args" "args" ...
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=$1; CFG=$2; shift 2; O=$R/gpurun_out/$TAG; mkdir -p $O
for a in "" "$@"; do
  timeout -k 10 200 python bench.py --config $CFG --no-cpu-baseline --roofline-launches 20 $a > $O/b.json 2>>$O/err.log || exit 1
  echo "[$a] $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step')")"
done
