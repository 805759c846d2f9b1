# Ablation sweep of k_sspp_c2f (SSPP_ABLATE bits: 1 no sampling, 2 no collision, 4 no arc,
# 8 no phase 2, 16 no phase-1 pair scan, 32 no hull, 64 launch only) at the bench defaults.
#   gpurun -- bash tools/gpu_ablate2.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-abl}; O=$R/gpurun_out/$TAG; mkdir -p $O
for m in 0 1 2 4 8 16 32 64 1,8 ; do
  mm=$(python -c "print(sum(int(x) for x in '$m'.split(',')))")
  SSPP_ABLATE=$mm timeout -k 10 120 python bench.py --no-cpu-baseline --steps 4096 --warmup 64 --roofline-launches 20 > $O/b.json 2>>$O/err.log || { echo "FAIL $m"; exit 1; }
  echo "ablate $mm $(python -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']/1e6,1),'M/s',round(d['ms_per_step']*1e3,3),'us/step', round(d['roofline']['kernel_us'],2), 'us/kernel')")"
done
echo DONE
