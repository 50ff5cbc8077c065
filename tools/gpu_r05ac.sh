#!/bin/bash
# Round 5, step ac: MobileNetV2 fp32x3 knobs re-checked on the round-5 kernels: where the layered tail
# starts (mbv2_layered) and tiles per workgroup (mbv2_x3_tpw), interleaved rounds, bit-identity.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_option.py --enc image_mbv2 --precision fp32x3 --opt mbv2_layered \
  --values 8 7 9 10 --rounds 5 > gpurun_out/r05ac_ab_mbv2_layered.txt 2>&1 || { tail -5 gpurun_out/r05ac_ab_mbv2_layered.txt; exit 1; }
grep '"ms"' gpurun_out/r05ac_ab_mbv2_layered.txt
timeout -k 10 400 python -u tools/ab_option.py --enc image_mbv2 --precision fp32x3 --opt mbv2_x3_tpw \
  --values 2 1 3 4 --rounds 5 > gpurun_out/r05ac_ab_mbv2_tpw.txt 2>&1 || { tail -5 gpurun_out/r05ac_ab_mbv2_tpw.txt; exit 1; }
grep '"ms"' gpurun_out/r05ac_ab_mbv2_tpw.txt
