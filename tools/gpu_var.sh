set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/var; mkdir -p $O; rm -f $O/*.json*
for lib in "" build/variants/libsspp_c2fw4.so build/variants/libsspp_c2fw5.so build/variants/libsspp_c2fw6.so; do for spl in 1 8; do
  SSPP_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --streams 4 --steps-per-launch $spl --steps 2048 --warmup 64 --roofline-launches 50 > $O/b.json 2>>$O/err.log || exit 1
  echo "lib $lib spl $spl $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,2),'us/step')")"
done; done
