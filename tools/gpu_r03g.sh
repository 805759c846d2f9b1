# Round-3: parity tests + benches, then c2f phase timelines from the timing variant.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-r03g}; O=$R/gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_r03b.sh $TAG || exit 1
export SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_wqt.so SSPP_KERNEL=1
timeout -k 10 120 python tools/wg_timing.py 20 $O/c2f_20.json > $O/c2f_20.log 2>&1 || { echo FAIL20; tail -5 $O/c2f_20.log; exit 1; }
echo DONE2
