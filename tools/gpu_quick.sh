#!/bin/bash
# All GPU tests, then per-encoder timings (ENCS) at B=256. Stops at the first crash-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for e in ${ENCS:-image image_mbv2}; do
  timeout -k 10 120 python tools/encoder_profile.py --enc $e --iters 10 || exit $?
done
