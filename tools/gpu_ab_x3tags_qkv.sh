#!/bin/bash
# GPU box: the fp32x3 fused step with BERT's QKV GEMM pinned to each interleaved split tile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_option.py --enc pipeline --precision fp32x3 --opt gemm_x3_tag \
  --values 100000 170128 171128 170256 --rounds 5 > gpurun_out/ab_x3tag_qkv.txt 2>&1 || { tail -5 gpurun_out/ab_x3tag_qkv.txt; exit 1; }
grep '"ms"' gpurun_out/ab_x3tag_qkv.txt
