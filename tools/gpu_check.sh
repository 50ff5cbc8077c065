#!/bin/bash
# GPU-box validation: parity tests, then a short bench. Stops at the first crash-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc (crash/timeout): stopping"; exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
brc=$?
tail -5 gpurun_out/bench.log
echo "pytest rc=$rc bench rc=$brc"
exit $brc
