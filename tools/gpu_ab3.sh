set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/ab3; mkdir -p $O; rm -f $O/*.json*
for m in 64 7; do for st in 1 2 4 8; do
  SSPP_ABLATE=$m timeout -k 10 200 python bench.py --no-cpu-baseline --streams $st --steps 2000 --warmup 50 --roofline-launches 200 > $O/b$m.json 2>>$O/err.log || exit 1
  echo "ablate $m streams $st $(python -c "import json;d=json.load(open('$O/b$m.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step', round(d['roofline']['kernel_us'],1))")"
done; done
for nt in 64 128; do
  SSPP_NT=$nt SSPP_ABLATE=64 timeout -k 10 200 python bench.py --no-cpu-baseline --streams 4 --steps 2000 --warmup 50 --roofline-launches 200 > $O/c.json 2>>$O/err.log || exit 1
  echo "NT $nt ablate 64 $(python -c "import json;d=json.load(open('$O/c.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step', round(d['roofline']['kernel_us'],1))")"
done
