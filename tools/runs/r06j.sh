# round 6: split-launch issue priority A/B: product (sampler 2, phase 1 1, consumers 0), consumers 3, none
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06j; mkdir -p $O; cd $R
for v in product cp3 noprio product cp3 noprio product cp3 noprio; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.log || { tail -20 $O/b_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$v.json'));print('$v: %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
timeout -k 10 180 python3 bench.py --mode dropin --steps 400 --warmup 50 > $O/bench_dropin.json 2> $O/bench_dropin.log || { tail -20 $O/bench_dropin.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_dropin.json'));print('dropin: %.1f us/plan; first %.0f max %.0f; cold %s; parts %s' % (d['value'], d['first_call_us'], d['first_call_us_max'], d['cold_calls_us'], d['cold_call_parts_us']))"
