#!/bin/bash
# Round 5, step q: MobileNetV2 fp32x3 stem-block tile rows unpadded and chunk-swizzled (LDS conflicts): the
# MobileNetV2 GPU tests, a cross-build A/B with bit-identity check, then the final validation of step p.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mbv2 or mobilenet" \
  > gpurun_out/r05q_pytest_mbv2.log 2>&1
rc=$?; tail -2 gpurun_out/r05q_pytest_mbv2.log; [ $rc -ne 0 ] && exit $rc
ENC=image_mbv2 PREC=fp32x3 ROUNDS=3 bash tools/gpu_ab_lib.sh > gpurun_out/r05q_ab_image_mbv2_fp32x3.txt 2>&1 || { cat gpurun_out/r05q_ab_image_mbv2_fp32x3.txt; exit 1; }
cat gpurun_out/r05q_ab_image_mbv2_fp32x3.txt
