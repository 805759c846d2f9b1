# Fused survivor queue: full GPU tests, then FQ off/on A/B on the driver's 20-step run, the long
# run and the drop-in latency.   gpurun --timeout 1100 -- bash tools/gpu_fq.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-fq}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for e in "SSPP_FQ=0" "SSPP_FQ=1" "SSPP_FQ=1 SSPP_FQ_NPG=2" "SSPP_FQ=1 SSPP_FQ_GS=8" "SSPP_FQ=1 SSPP_FQ_GS=32"; do
  for rep in 1 2; do
    timeout -k 10 200 env $e python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s20.json 2>>$O/err.log || { echo "FAIL $e"; exit 1; }
    echo "[$e] short20 $(python -c "import json;d=json.load(open('$O/s20.json'));print(round(d['value']/1e6,1))")"
  done
  timeout -k 10 200 env $e python bench.py --steps 2048 --warmup 64 --no-cpu-baseline > $O/long.json 2>>$O/err.log || { echo "FAIL $e long"; exit 1; }
  echo "[$e] long $(python -c "import json;d=json.load(open('$O/long.json'));print(round(d['value']/1e6,1), round(d['roofline']['kernel_us'],1))")"
done
timeout -k 10 200 python bench.py --mode dropin --no-cpu-baseline --steps 2000 --warmup 100 > $O/dropin.json 2>>$O/err.log || exit 1
python -c "import json;d=json.load(open('$O/dropin.json'));print('dropin', d['latency_us'], 'isolated', d['isolated_step_kernel_us'])"
echo DONE
