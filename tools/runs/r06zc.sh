# round 6: multi-goal geom state: record re-load per near pair (product) against held type/index/size with the rotation cached per group (small)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06zc; mkdir -p $O; cd $R
timeout -k 10 300 python3 -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
: 


for v in product small product small; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config multigoal --no-cpu-baseline > $O/multigoal_$v.json 2> $O/multigoal_$v.log || { tail -20 $O/multigoal_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/multigoal_$v.json'));print('$v multigoal: %.2f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
