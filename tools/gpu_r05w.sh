#!/bin/bash
# Round 5, step w: fused fp32x3 step, BERT FFN2 and FFN1 tile pins (gemm_x3_tag) against the shipped 70256.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_option.py --enc pipeline --precision fp32x3 --opt gemm_x3_tag \
  --values 570256 570128 571128 --rounds 7 > gpurun_out/r05w_ab_x3tag_ffn2.txt 2>&1 || { tail -5 gpurun_out/r05w_ab_x3tag_ffn2.txt; exit 1; }
grep '"ms"' gpurun_out/r05w_ab_x3tag_ffn2.txt
timeout -k 10 400 python -u tools/ab_option.py --enc pipeline --precision fp32x3 --opt gemm_x3_tag \
  --values 470256 470128 --rounds 7 > gpurun_out/r05w_ab_x3tag_ffn1.txt 2>&1 || { tail -5 gpurun_out/r05w_ab_x3tag_ffn1.txt; exit 1; }
grep '"ms"' gpurun_out/r05w_ab_x3tag_ffn1.txt
