# k_sspp_c2f work statistics (SSPP_C2F_STATS variant) for the throughput and latency shapes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-st}; O=$R/gpurun_out/$TAG; mkdir -p $O
for sh in "SSPP_NT=64 SSPP_G1=4" "SSPP_NT=64 SSPP_G1=8" "SSPP_NT=256 SSPP_G1=64"; do
  echo "[$sh]"
  env $sh SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_st.so timeout -k 10 120 python tools/c2f_stats.py > $O/st.txt 2>&1 || { tail -5 $O/st.txt; exit 1; }
  cat $O/st.txt
done
echo DONE
