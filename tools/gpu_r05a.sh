#!/bin/bash
# Round 5, step a: the fp32x3 / fp32 GPU tests (activation-plane scales, golden pins), then the
# MobileNetV2 fp32x3 LDS-swizzle build against the previous one (bit identity + time), the
# mbv2_x3_occ A/B, and a default bench line. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fp32x3.py \
  tests/test_gpu_fp32.py tests/test_gpu_mbv2.py -m gpu -s > gpurun_out/r05_pytest_x3scale.log 2>&1
rc=$?; tail -4 gpurun_out/r05_pytest_x3scale.log; [ $rc -ne 0 ] && exit $rc
ENC=image_mbv2 PREC=fp32x3 ROUNDS=3 bash tools/gpu_ab_lib.sh > gpurun_out/r05_ab_lib_mbv2x3_swz.txt 2>&1 || exit $?
tail -3 gpurun_out/r05_ab_lib_mbv2x3_swz.txt
timeout -k 10 300 python -u tools/ab_option.py --enc image_mbv2 --precision fp32x3 --opt mbv2_x3_occ --values 3 4 \
  --rounds 7 > gpurun_out/r05_ab_mbv2x3_occ.txt 2>&1 || exit $?
tail -4 gpurun_out/r05_ab_mbv2x3_occ.txt
timeout -k 10 600 python -u bench.py --steps 20 --json-out gpurun_out/r05_bench_a.json > gpurun_out/r05_bench_a.log 2>&1 || exit $?
tail -c 600 gpurun_out/r05_bench_a.log
