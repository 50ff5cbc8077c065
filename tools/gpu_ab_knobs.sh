#!/bin/bash
# Fused-step (B = 256) A/B of result-preserving knobs, interleaved rounds (tools/ab_option.py).
# f16: ResNet kernel routes, residual prefetch, fusion samples per workgroup, O-proj + LN form;
# fp32: BERT per-launch-class tiles (gemm_f32_tag = tag * 100000 + tile: 5 FFN2, 3 O-proj, 1 QKV).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_knobs.txt; : > $out
run() {  # precision, option, values...
  local p=$1 o=$2; shift 2
  timeout -k 10 300 python3 tools/ab_option.py --enc pipeline --precision $p --opt $o --rounds 7 --values "$@" > gpurun_out/ab_tmp.txt 2>&1 || { tail -20 gpurun_out/ab_tmp.txt; exit 1; }
  grep '^{' gpurun_out/ab_tmp.txt | tee -a $out
}
run f16 conv3x3_halo 1 0 && run f16 conv3x3_direct 1 0 && run f16 pw_chain 2 1 0 && \
run f16 gemm_prefetch_r 1 0 && run f16 fusion_r 4 2 1 && \
run fp32 gemm_f32_tag 500000 500004 500008 500001 500005 && \
run fp32 gemm_f32_tag 300000 300004 300008 300001 300005 300002 300006
