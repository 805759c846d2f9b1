# Kernel trace of a command: bash tools/gpu_trace.sh TAG cmd args...
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- "$@" > $O/trace.log 2>&1 || { echo TRACE FAILED; tail -5 $O/trace.log; exit 1; }
python3 - "$O/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'].replace('(anonymous namespace)::', '')[:50], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us avg', round(float(r['MinNs']) / 1e3, 2), 'min')
PY
