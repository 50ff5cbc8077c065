#!/bin/bash
# Fused-step A/B of per-class tile pins for the ResNet GEMMs (tag 7 = 3x3 convs, 8 = 1x1 convs):
# fp32 engine (gemm_f32_tag = tag * 100000 + tile 0..8) and f16 (gemm_bn_tag = tag * 100000 + id).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_resnet_tags.txt; : > $out
run() {  # precision, option, values...
  local p=$1 o=$2; shift 2
  timeout -k 10 400 python3 tools/ab_option.py --enc pipeline --precision $p --opt $o --rounds 5 --iters ${ITERS:-3} --values "$@" > gpurun_out/ab_tmp.txt 2>&1 || { tail -20 gpurun_out/ab_tmp.txt; exit 1; }
  grep '^{' gpurun_out/ab_tmp.txt | tee -a $out
}
ITERS=2 run fp32 gemm_f32_tag 700000 700004 700008 700001 700005 700002 700006 && \
ITERS=2 run fp32 gemm_f32_tag 800000 800004 800008 800001 800005 800002 800006 800003 800007
