# round 6: phase priority in every k_sspp_c2f instance (A/B) — drop-in, default long run; shared streams
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06k; mkdir -p $O; cd $R
for v in product prioall product prioall; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -k 10 180 python3 bench.py --mode dropin --steps 400 --warmup 50 > $O/dropin_$v.json 2> $O/dropin_$v.log || { tail -20 $O/dropin_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/dropin_$v.json'));print('$v dropin: %.1f us/plan isolated %.1f; first %.0f max %.0f; parts %s' % (d['value'], d['isolated_step_kernel_us'], d['first_call_us'], d['first_call_us_max'], d['cold_call_parts_us']))"
  SSPP_LIB_PATH=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline > $O/default_$v.json 2> $O/default_$v.log || { tail -20 $O/default_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/default_$v.json'));print('$v default: %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
