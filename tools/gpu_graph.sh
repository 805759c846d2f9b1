set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/exec; mkdir -p $O; rm -f $O/*.json*
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for br in 2 3 4 6 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --streams $br --roofline-launches 50 >> $O/bench.jsonl 2>>$O/err.log || exit 1
done
SSPP_G1=32 timeout -k 10 200 python bench.py --no-cpu-baseline --streams 4 --roofline-launches 50 >> $O/bench.jsonl 2>>$O/err.log || exit 1
SSPP_G1=8 timeout -k 10 200 python bench.py --no-cpu-baseline --streams 4 --roofline-launches 50 >> $O/bench.jsonl 2>>$O/err.log || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --mode eager --streams 4 --roofline-launches 50 >> $O/bench.jsonl 2>>$O/err.log || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --streams 4 --steps 2000 --warmup 100 --roofline-launches 50 >> $O/bench.jsonl 2>>$O/err.log || exit 1
python -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print(d['config']['streams'], d['config']['launch'], d['steps'], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['kernel_us'],1))
"
