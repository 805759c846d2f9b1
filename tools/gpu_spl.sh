set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/spl; mkdir -p $O; rm -f $O/*.json*
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for spl in 1 2 4 8 16; do for st in 2 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --streams $st --steps-per-launch $spl --steps 2048 --warmup 64 --roofline-launches 50 > $O/b.json 2>>$O/err.log || exit 1
  echo "spl $spl streams $st $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step')")"
done; done
for spl in 8 16; do
  SSPP_ABLATE=7 timeout -k 10 200 python bench.py --no-cpu-baseline --streams 4 --steps-per-launch $spl --steps 2048 --warmup 64 --roofline-launches 50 > $O/b.json 2>>$O/err.log || exit 1
  echo "ablate7 spl $spl $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step')")"
done
