# round 6: split-launch issue priority A/B (beacon timeline + bench)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06h; mkdir -p $O; cd $R
timeout -k 5 300 python3 -c "import torch, numpy" > $O/import.txt 2>&1
BEACON_OUT=$O/beacons_prio.json SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_dbg.so timeout -k 5 60 python3 -u tools/split_beacons.py > $O/beacons_prio.txt 2>&1 || { cat $O/beacons_prio.txt; exit 1; }
grep -E "start|phase 1 done|pushed|left|last" $O/beacons_prio.txt
for v in product noprio product noprio; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.log || { tail -20 $O/b_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$v.json'));print('$v: %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
