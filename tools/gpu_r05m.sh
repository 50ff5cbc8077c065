#!/bin/bash
# Round 5, step m: the fused fp32x3 step with BERT FFN2 / O-projection pinned to 70256 (the shipped pins),
# the new one-stage 72128 and 70128 (gemm_x3_tag, tag * 100000 + id), interleaved rounds in one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_option.py --enc pipeline --precision fp32x3 --opt gemm_x3_tag \
  --values 570256 572128 --rounds 7 > gpurun_out/r05m_ab_x3tag_ffn2.txt 2>&1 || { tail -5 gpurun_out/r05m_ab_x3tag_ffn2.txt; exit 1; }
grep '"ms"' gpurun_out/r05m_ab_x3tag_ffn2.txt
timeout -k 10 400 python -u tools/ab_option.py --enc pipeline --precision fp32x3 --opt gemm_x3_tag \
  --values 370256 372128 370128 --rounds 5 > gpurun_out/r05m_ab_x3tag_oproj.txt 2>&1 || { tail -5 gpurun_out/r05m_ab_x3tag_oproj.txt; exit 1; }
grep '"ms"' gpurun_out/r05m_ab_x3tag_oproj.txt
timeout -k 10 400 python -u tools/ab_option.py --enc pipeline --precision fp32x3 --opt gemm_x3_tag \
  --values 170256 172128 --rounds 5 > gpurun_out/r05m_ab_x3tag_qkv.txt 2>&1 || { tail -5 gpurun_out/r05m_ab_x3tag_qkv.txt; exit 1; }
grep '"ms"' gpurun_out/r05m_ab_x3tag_qkv.txt
