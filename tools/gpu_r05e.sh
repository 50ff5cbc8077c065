#!/bin/bash
# Round 5, step e: the early-restage schedule of the 2-stage K-interleaved split tiles (gemm_x3_restage 1 vs 0):
# the split-GEMM tests, then same-process A/Bs on the fp32x3 text and image encoders and the fused pipeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp32x3.py -m gpu \
  -k "split_gemm or bit_identical or batch_invariance or resnet" > gpurun_out/r05_pytest_restage.log 2>&1
rc=$?; tail -2 gpurun_out/r05_pytest_restage.log; [ $rc -ne 0 ] && exit $rc
for e in text image pipeline; do
  timeout -k 10 300 python3 -u tools/ab_option.py --enc $e --precision fp32x3 --opt gemm_x3_restage --values 2 0 1 \
    --rounds 7 2>/dev/null > gpurun_out/r05_ab_restage_$e.txt || exit $?
  cat gpurun_out/r05_ab_restage_$e.txt
done
