bash tools/gpu_tsp_w.sh tspw8 m4 m3
for v in m4; do for spl in 32; do
  timeout -k 10 120 env SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_$v.so python bench.py --no-cpu-baseline --steps 4096 --warmup 64 > gpurun_out/tspw8/r.json 2>>gpurun_out/tspw8/err.log && python -c "import json;d=json.load(open('gpurun_out/tspw8/r.json'));print('robocrane long $v', round(d['value']/1e6,1))"
  timeout -k 10 120 env SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_$v.so python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/tspw8/r.json 2>>gpurun_out/tspw8/err.log && python -c "import json;d=json.load(open('gpurun_out/tspw8/r.json'));print('robocrane short $v', round(d['value']/1e6,1))"
done; done
