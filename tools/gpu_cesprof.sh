# CES kernel durations (rocprofv3) at a few sizes: bash tools/gpu_cesprof.sh
for n in "50 0" "4096 0" "16384 3"; do
  bash tools/gpu_trace.sh trc python3 $GRAFT_REPO_ROOT/tools/ces_timing.py $n | grep k_ces | sed "s/^/[$n] /"
done
