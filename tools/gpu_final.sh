#!/bin/bash
# GPU box, end of a session: the whole -m gpu suite, smoke(), the bench line, and the fenced
# rocprofv3 window of the fp32x3 bench step (stops at the first failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-final}
TAG=$T TEST_TIMEOUT=700 BENCH_TIMEOUT=420 bash tools/gpu_tests_bench.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
PREC=fp32x3 STEPS=10 bash tools/gpu_prof_bench.sh > gpurun_out/${T}_prof_bench.log 2>&1 || { tail -5 gpurun_out/${T}_prof_bench.log; exit 1; }
head -6 gpurun_out/bench_prof_grid_fp32x3.txt | cut -c1-150
