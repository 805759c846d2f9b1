# round 6: stacking (DEF 1 form) at 3 waves per SIMD (159 VGPRs, no scratch) against 4 (22 spilled VGPRs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06n; mkdir -p $O; cd $R
timeout -k 10 300 python3 -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
for v in product def3 product def3; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config stacking --no-cpu-baseline > $O/stacking_$v.json 2> $O/stacking_$v.log || { tail -20 $O/stacking_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/stacking_$v.json'));print('$v stacking: %.2f M cand/s kernel_us %.1f rep %s' % (d['value']/1e6, d['roofline']['kernel_us'], d['config'].get('tsp_rep')))"
done
