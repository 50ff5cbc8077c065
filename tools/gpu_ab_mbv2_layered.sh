#!/bin/bash
# fp32x3 MobileNetV2 layered tail (mbv2_layered k: features[k..17] as GEMM -> depthwise -> GEMM): the
# oracle / batch-invariance tests, the A/B over k at B = 256, then the fp32x3 MobileNetV2 profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_fp32x3.py -k "mobilenet" > gpurun_out/r04_mbv2_layered_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r04_mbv2_layered_tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert|mbv2_layered" gpurun_out/r04_mbv2_layered_tests.log | head -20; exit $rc; }
grep -E "mbv2_layered" gpurun_out/r04_mbv2_layered_tests.log | head
timeout -k 10 300 python3 -u tools/ab_option.py --enc image_mbv2 --opt mbv2_layered --values ${VALS:-0 7 8 11 12 14 15} \
  --precision fp32x3 > gpurun_out/r04_ab_mbv2_layered.txt 2>&1 || exit 1
grep enc gpurun_out/r04_ab_mbv2_layered.txt
PREC=fp32x3 ENCS="image_mbv2" bash tools/gpu_enc_prof.sh
