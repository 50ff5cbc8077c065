#!/bin/bash
# GPU box: the round-4 new tests first (short), then the whole -m gpu suite and the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04}
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_fp32x3.py -k "fused_qkv or overflow or untuned or mixed or small_act or mobilenet_v2_fp32x3" > gpurun_out/${TAG}_new.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/${TAG}_new.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_new.log | head -20; exit $rc; }
TAG=$TAG bash tools/gpu_tests_bench.sh
