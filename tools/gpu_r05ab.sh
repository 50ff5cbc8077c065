#!/bin/bash
# Round 5, step ab: ResNet50's tile-group order (gemm_glds_group_m on the image handle only: ENC image, and
# the fused step where ab_option sets every handle, BERT included), interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_option.py --enc image --precision fp32x3 --opt gemm_glds_group_m \
  --values 8 16 2 0 --rounds 5 > gpurun_out/r05ab_ab_groupm_image.txt 2>&1 || { tail -5 gpurun_out/r05ab_ab_groupm_image.txt; exit 1; }
grep '"ms"' gpurun_out/r05ab_ab_groupm_image.txt
