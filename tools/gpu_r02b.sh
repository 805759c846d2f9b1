set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_wgph.sh || exit 1
bash tools/gpu_round2.sh ${1:-r02b} || exit 1
