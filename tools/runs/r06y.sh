# round 6: which k_sspp_c2f instance the drop-in runs (latency-shape split or not), kernel statistics per variant
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06y; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for v in product nolat; do
  if [ $v = product ]; then L=; else L=$R/sspp_amd/lib/variants/libsspp_$v.so; fi
  SSPP_LIB_PATH=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 $R/bench.py --mode dropin --steps 100 --warmup 20 > $O/$v.json 2> $O/$v.log || { tail -20 $O/$v.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$O/$v/run_kernel_stats.csv')):
    if 'c2f' in r['Name']: print('$v', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
