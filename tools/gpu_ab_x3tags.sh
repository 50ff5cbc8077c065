#!/bin/bash
# GPU box: the fp32x3 fused step with BERT FFN2 / O-proj pinned to each interleaved split tile
# (gemm_x3_tag, tag * 100000 + id; 0 = autotune), interleaved rounds in one process
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_option.py --enc pipeline --precision fp32x3 --opt gemm_x3_tag \
  --values 500000 570256 570128 571128 --rounds 5 > gpurun_out/ab_x3tag_ffn2.txt 2>&1 || { tail -5 gpurun_out/ab_x3tag_ffn2.txt; exit 1; }
grep '"ms"' gpurun_out/ab_x3tag_ffn2.txt
timeout -k 10 400 python -u tools/ab_option.py --enc pipeline --precision fp32x3 --opt gemm_x3_tag \
  --values 300000 370256 370128 371128 --rounds 5 > gpurun_out/ab_x3tag_oproj.txt 2>&1 || { tail -5 gpurun_out/ab_x3tag_oproj.txt; exit 1; }
grep '"ms"' gpurun_out/ab_x3tag_oproj.txt
