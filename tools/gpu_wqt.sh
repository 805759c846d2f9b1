# Round-3: k_sspp_wq1/2 timelines from the SSPP_WG_TIMING variant.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-wqt}; O=$R/gpurun_out/$TAG; mkdir -p $O
export SSPP_LIB_PATH=$R/sspp_amd/lib/variants/libsspp_wqt.so
for spl in 1 20; do
  timeout -k 10 120 python tools/wq_timing.py $spl $O/wq_spl$spl.json > $O/wq_spl$spl.log 2>&1 || { echo "FAIL $spl"; tail -5 $O/wq_spl$spl.log; exit 1; }
done
SSPP_WQ_CPW=4 timeout -k 10 120 python tools/wq_timing.py 1 $O/wq_spl1_cpw4.json > $O/wq_spl1_cpw4.log 2>&1 || { echo "FAIL cpw4"; exit 1; }
echo DONE
