#!/bin/bash
# f16 MobileNetV2 layered tail (mbv2_layered16 k): the oracle / batch-invariance tests, the A/B over k at
# B = 256, then the f16 MobileNetV2 profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_mbv2.py > gpurun_out/r04_mbv2_layered16_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r04_mbv2_layered16_tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r04_mbv2_layered16_tests.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u tools/ab_option.py --enc image_mbv2 --opt mbv2_layered16 --values ${VALS:-0 7 8 11 12 14 15} \
  --precision f16 > gpurun_out/r04_ab_mbv2_layered16.txt 2>&1 || exit 1
grep enc gpurun_out/r04_ab_mbv2_layered16.txt
PREC=f16 ENCS="image_mbv2" bash tools/gpu_enc_prof.sh
