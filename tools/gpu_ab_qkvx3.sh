#!/bin/bash
# fp32x3 fused QKV + attention (bert_qkv_attn 1) vs the split QKV GEMM + attention kernel (0): text alone
# and the fused step at B = 256, interleaved in one process; then the fp32x3 text and MobileNetV2 encoder
# kernel profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ab_option.py --enc text --opt bert_qkv_attn --values 0 1 --precision fp32x3 \
  > gpurun_out/r04_ab_qkvx3_text.txt 2>&1 || exit 1
tail -3 gpurun_out/r04_ab_qkvx3_text.txt
timeout -k 10 300 python3 -u tools/ab_option.py --enc pipeline --opt bert_qkv_attn --values 0 1 --precision fp32x3 \
  > gpurun_out/r04_ab_qkvx3_pipeline.txt 2>&1 || exit 1
tail -3 gpurun_out/r04_ab_qkvx3_pipeline.txt
PREC=fp32x3 ENCS="text image_mbv2" bash tools/gpu_enc_prof.sh && PREC=f16 ENCS="image_mbv2" bash tools/gpu_enc_prof.sh
