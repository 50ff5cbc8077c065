#!/bin/bash
# Fused-step A/B of BERT per-launch-class tiles (gemm_bn_tag = tag * 100000 + tile id):
# tag 5 = FFN2, 3 = O-projection, 4 = FFN1. Interleaved rounds, medians (tools/ab_option.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name, values...
  local n=$1; shift
  timeout -k 10 300 python3 tools/ab_option.py --enc pipeline --opt gemm_bn_tag --rounds 7 --values "$@" > gpurun_out/ab_$n.txt 2>&1 || { tail -20 gpurun_out/ab_$n.txt; exit 1; }
  grep '^{' gpurun_out/ab_$n.txt
}
run ffn2 540256 511128 550256 510256 541256 && \
run oproj 311128 340256 341256 310128 350256 && \
run ffn1 440256 441256 410256 450256
