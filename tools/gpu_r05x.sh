#!/bin/bash
# Round 5, step x: the whole -m gpu suite and smoke on the final tree (as the round-end driver runs them).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05x_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05x_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r05x_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r05x_smoke.log; exit $rc
