#!/bin/bash
# fp32x3 layer1 seam kernels (OPT = pw_chain_x3, VALS 0 1 2): the bit-identity test, then the image encoder
# alone and the fused step at B = 256 (interleaved in one process), then the fp32x3 image profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_fp32x3.py -k "seams_bit_identical or resnet_fp32x3" \
  > gpurun_out/r04_seamx3_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r04_seamx3_tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r04_seamx3_tests.log | head -20; exit $rc; }
OPT=${OPT:-pw_chain_x3}; VALS=${VALS:-0 1 2}; PVALS=${PVALS:-0 2}
timeout -k 10 300 python3 -u tools/ab_option.py --enc image --opt $OPT --values $VALS --precision fp32x3 \
  > gpurun_out/r04_ab_${OPT}_image.txt 2>&1 || exit 1
tail -4 gpurun_out/r04_ab_${OPT}_image.txt
timeout -k 10 300 python3 -u tools/ab_option.py --enc pipeline --opt $OPT --values $PVALS --precision fp32x3 \
  > gpurun_out/r04_ab_${OPT}_pipeline.txt 2>&1 || exit 1
tail -3 gpurun_out/r04_ab_${OPT}_pipeline.txt
PREC=fp32x3 ENCS="image" bash tools/gpu_enc_prof.sh
