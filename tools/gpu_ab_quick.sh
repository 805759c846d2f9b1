# Robocrane long + driver-shaped short bench per library variant (no tests).
#   gpurun -- bash tools/gpu_ab_quick.sh TAG variant[@ENV=V[,ENV=V]]...   (variant "default" = sspp_amd/lib)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-abq}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
for spec in "$@"; do
  v=${spec%%@*}; E=""; [ "$spec" != "$v" ] && E=$(echo ${spec#*@} | tr ',' ' ')
  L=""; [ "$v" != default ] && L="SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_$v.so"
  for a in "" "--steps 20 --warmup 5" "--steps 20 --warmup 5"; do
    timeout -k 10 200 env $L $E python bench.py --no-cpu-baseline $a $EXTRA > $O/b.json 2>>$O/err.log || { echo "FAIL $spec"; tail -5 $O/err.log; exit 1; }
    echo "$spec [$a] $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s', round(d['roofline']['kernel_us'],1),'us/kernel')")"
  done
done
echo DONE
