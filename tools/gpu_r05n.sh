#!/bin/bash
# Round 5, step n: BERT FFN1 pinned to 70256 (the shipped pin) or to the one-stage 72128 (gemm_x3_tag 4),
# BERT alone and the fused step, interleaved rounds in one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in text pipeline; do
  timeout -k 10 400 python -u tools/ab_option.py --enc $e --precision fp32x3 --opt gemm_x3_tag \
    --values 470256 472128 --rounds 7 > gpurun_out/r05n_ab_x3tag_ffn1_$e.txt 2>&1 || { tail -5 gpurun_out/r05n_ab_x3tag_ffn1_$e.txt; exit 1; }
  grep '"ms"' gpurun_out/r05n_ab_x3tag_ffn1_$e.txt
done
