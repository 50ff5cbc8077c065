#!/bin/bash
# A/B of the BERT FFN2 tile (gemm_bn_tag = 5 * 100000 + tile id) on the text encoder and the fused step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_option.py --enc text --opt gemm_bn_tag --values 511128 540256 510256 520256 530256 550256 > gpurun_out/ab_ffn2_text.txt 2>&1 || { tail -20 gpurun_out/ab_ffn2_text.txt; exit 1; }
cat gpurun_out/ab_ffn2_text.txt | tail -12
timeout -k 10 300 python3 tools/ab_option.py --enc pipeline --opt gemm_bn_tag --values 511128 540256 > gpurun_out/ab_ffn2_pipe.txt 2>&1 || { tail -20 gpurun_out/ab_ffn2_pipe.txt; exit 1; }
cat gpurun_out/ab_ffn2_pipe.txt | tail -6
