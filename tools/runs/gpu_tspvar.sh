# TaskSpacePlanner benches (stacking, multi-goal) on the default library and on variant builds
# (sspp_amd/lib/variants/libsspp_NAME.so): bash tools/runs/gpu_tspvar.sh TAG [variants...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-tspvar}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for v in default "$@"; do
  L=""; [ $v != default ] && L=$R/sspp_amd/lib/variants/libsspp_$v.so
  for c in stacking multigoal; do
    SSPP_LIB_PATH=$L timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/${c}_$v.json 2> $O/${c}_$v.log \
      || { tail -5 $O/${c}_$v.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${c}_$v.json'));print('%-10s %-8s %7.2f M/s kernel %6.1f us' % ('$c', '$v', d['value']/1e6, d['roofline']['kernel_us']))"
  done
done
# the inline narrowphase (form 0) against the default deferred polygons (form 3), stacking
timeout -k 10 200 python3 bench.py --config stacking --tsp-form 0 --no-cpu-baseline > $O/stacking_form0.json 2> $O/stacking_form0.log \
  || { tail -5 $O/stacking_form0.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/stacking_form0.json'));print('stacking form0 %7.2f M/s kernel %6.1f us form %s' % (d['value']/1e6, d['roofline']['kernel_us'], d['config'].get('tsp_form')))"
echo DONE
