# round 6: unsplit 20-step launches (product, relaxed) against round 5's 53.5 us
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06e; mkdir -p $O; cd $R
for v in product relaxed; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --split 0 > $O/b_$v.json 2> $O/b_$v.log || { tail -20 $O/b_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$v.json'));print('$v unsplit: %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
timeout -k 10 180 python3 bench.py --gpus 1 --steps 400 --warmup 20 --no-cpu-baseline > $O/b_long.json 2> $O/b_long.log || { tail -20 $O/b_long.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_long.json'));print('product 400 steps (40/launch, unsplit): %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
