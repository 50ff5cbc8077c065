#!/bin/bash
# Round 5, step j: the split tiles' direct epilogue (transposed MFMAs, no LDS staging): fp32x3 tests first,
# then the whole -m gpu suite, then cross-build A/Bs with bit-identity checks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32x3.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05j_pytest_x3.log 2>&1
rc=$?; tail -2 gpurun_out/r05j_pytest_x3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05j_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05j_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in "text fp32x3 3" "image fp32x3 3" "pipeline fp32x3 3" "image_mbv2 fp32x3 2"; do
  set -- $cfg
  ENC=$1 PREC=$2 ROUNDS=$3 bash tools/gpu_ab_lib.sh > gpurun_out/r05j_ab_$1_$2.txt 2>&1 || { cat gpurun_out/r05j_ab_$1_$2.txt; exit 1; }
  cat gpurun_out/r05j_ab_$1_$2.txt
done
