# Round evidence on the final tree: tests, smoke, benches, rocprof stats/trace, then PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_round2.sh ${1:-r02c} || exit 1
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${1:-r02c}/short_rep$i.json 2>/dev/null || exit 1; head -c 200 gpurun_out/${1:-r02c}/short_rep$i.json; echo; done
bash tools/gpu_round2_pmc.sh ${2:-r02cpmc} || exit 1
