# Round-3: k_sspp_c2f workgroup timelines (SSPP_WG_TIMING variant) for the driver's 20-step launch
# and a single step.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-c2ft}; O=$R/gpurun_out/$TAG; mkdir -p $O
export SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_wqt.so SSPP_KERNEL=1
timeout -k 10 120 python tools/wg_timing.py 20 $O/c2f_20.json > $O/c2f_20.log 2>&1 || { echo FAIL20; tail -5 $O/c2f_20.log; exit 1; }
SSPP_NT=256 SSPP_G1=64 timeout -k 10 120 python tools/wg_timing.py 1 $O/c2f_1_256_64.json > $O/c2f_1.log 2>&1 || { echo FAIL1; tail -5 $O/c2f_1.log; exit 1; }
SSPP_NT=64 SSPP_G1=16 timeout -k 10 120 python tools/wg_timing.py 1 $O/c2f_1_64_16.json > $O/c2f_1b.log 2>&1 || { echo FAIL1b; tail -5 $O/c2f_1b.log; exit 1; }
echo DONE
