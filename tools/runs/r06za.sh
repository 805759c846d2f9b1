# round 6: stacking with the geom record re-loaded per near pair (product, 6 spilled VGPRs) against held (noleanone, 10)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06za; mkdir -p $O; cd $R
timeout -k 10 300 python3 -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
for v in product noleanone product noleanone; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config stacking --no-cpu-baseline > $O/stacking_$v.json 2> $O/stacking_$v.log || { tail -20 $O/stacking_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/stacking_$v.json'));print('$v stacking: %.2f M cand/s kernel_us %.1f rep %s' % (d['value']/1e6, d['roofline']['kernel_us'], d['config'].get('tsp_rep')))"
done
cd /tmp && export TMPDIR=/tmp
for v in product noleanone; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --config stacking --steps 4 --warmup 1 --roofline-launches 20 > $O/w_$v.log 2>&1 || { tail -5 $O/w_$v.log; exit 1; }
done
echo DONE
