# round 6: A/B of kDeep through scalar registers (product) against the VGPR constant (nodeep)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06m; mkdir -p $O; cd $R
timeout -k 10 300 python3 -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
for v in product nodeep product nodeep; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  for c in stacking multigoal; do
    SSPP_LIB_PATH=$L timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/${c}_$v.json 2> $O/${c}_$v.log || { tail -20 $O/${c}_$v.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${c}_$v.json'));print('$v $c: %.2f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
  done
  SSPP_LIB_PATH=$L timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/short20_$v.json 2> $O/short20_$v.log || { tail -20 $O/short20_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/short20_$v.json'));print('$v short20: %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
