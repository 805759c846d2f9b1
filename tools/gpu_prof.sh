set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in 0 6 7; do
SSPP_ABLATE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ab$m -o run --output-format csv -- python3 $R/tools/ablate.py > $R/gpurun_out/prof_ab$m.log 2>&1 || exit 1
done
