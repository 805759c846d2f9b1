# round 6: parity of the SSPP paths after the sampler change, then the driver's bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06g; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_dropin_sspp.py tests/test_ces.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for i in 1 2 3; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b20_$i.json 2> $O/b20_$i.log || { tail -20 $O/b20_$i.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b20_$i.json'));print('short20: %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
done
timeout -k 10 240 python3 bench.py --no-cpu-baseline > $O/b_default.json 2> $O/b_default.log || { tail -20 $O/b_default.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_default.json'));print('default: %.1f M cand/s kernel_us %.1f' % (d['value']/1e6, d['roofline']['kernel_us']))"
