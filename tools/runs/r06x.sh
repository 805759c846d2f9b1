# round 6: drop-in plan() with the survivor queue in the latency shape (product) against without (nolat)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06x; mkdir -p $O; cd $R
timeout -k 10 300 python3 -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_dropin_sspp.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_dropin.txt 2>&1 || { tail -30 $O/tests_dropin.txt; exit 1; }
tail -2 $O/tests_dropin.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in product nolat product nolat; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -k 10 180 python3 bench.py --mode dropin --steps 400 --warmup 50 > $O/dropin_$v.json 2> $O/dropin_$v.log || { tail -20 $O/dropin_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/dropin_$v.json'));print('$v dropin: %.1f us/plan isolated %.1f split %s feasible %s' % (d['value'], d['isolated_step_kernel_us'], d['config'].get('split'), d.get('feasible_per_plan')))"
done
