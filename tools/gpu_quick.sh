# tests (gpu) + robocrane throughput (native executor) + ablations; usage: bash tools/gpu_quick.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-quick}; mkdir -p $O; rm -f $O/*.json*
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for m in 0 2 4; do
  SSPP_ABLATE=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1000 --warmup 50 --roofline-launches 50 >> $O/bench.jsonl 2>>$O/err.log || exit 1
done
for g in 256 128; do for gg in 16; do
  SSPP_G1=$gg SSPP_NT=$g timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1000 --warmup 50 --roofline-launches 50 >> $O/bench.jsonl 2>>$O/err.log || exit 1; done
done
python -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['kernel_us'],1))
"
SSPP_PAIR_ORDER=0 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1000 --warmup 50 --roofline-launches 50 > $O/po0.json 2>>$O/err.log || exit 1
python -c "import json;d=json.load(open('$O/po0.json'));print('scene pair order', round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step')"
