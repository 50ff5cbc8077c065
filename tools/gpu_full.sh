#!/bin/bash
# tests -> bench -> rocprofv3 kernel stats (stops at the first crash-type exit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh || exit $?
export TMPDIR=/tmp
rm -rf gpurun_out/prof; mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
python3 tools/prof_summary.py gpurun_out/prof/run_results.db 2>/dev/null | head -40
exit $rc
