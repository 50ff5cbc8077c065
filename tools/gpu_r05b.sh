#!/bin/bash
# Round 5, step b: MobileNetV2 fp32x3 layout A/Bs (mbv2_x3_sesw, mbv2_x3_occ), then the round-4 library
# (libmec_hip_base.so, built from commit 50e1d48) against this tree's, alternating processes, on the fp32x3
# text and image encoders and the fused pipeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_option.py --enc image_mbv2 --precision fp32x3 --opt mbv2_x3_sesw --values 1 0 \
  --rounds 7 > gpurun_out/r05_ab_mbv2x3_sesw.txt 2>&1 || exit $?
tail -2 gpurun_out/r05_ab_mbv2x3_sesw.txt
timeout -k 10 300 python -u tools/ab_option.py --enc image_mbv2 --precision fp32x3 --opt mbv2_x3_occ --values 3 4 \
  --rounds 7 > gpurun_out/r05_ab_mbv2x3_occ2.txt 2>&1 || exit $?
tail -2 gpurun_out/r05_ab_mbv2x3_occ2.txt
for e in image_mbv2 text image pipeline; do
  ENC=$e PREC=fp32x3 ROUNDS=3 bash tools/gpu_ab_lib.sh > gpurun_out/r05_ab_lib_r04_$e.txt 2>&1 || exit $?
  tail -7 gpurun_out/r05_ab_lib_r04_$e.txt
done
