#!/bin/bash
# A/B of the ping-pong GEMM tile order (gemm_group_m) on BERT alone and on the fused step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_option.py --enc text --opt gemm_group_m --rounds 7 --values 0 4 8 16 > gpurun_out/ab_group_text.txt 2>&1 || { tail -20 gpurun_out/ab_group_text.txt; exit 1; }
grep '^{' gpurun_out/ab_group_text.txt
timeout -k 10 300 python3 tools/ab_option.py --enc pipeline --opt gemm_group_m --rounds 7 --values 0 4 8 16 > gpurun_out/ab_group_pipe.txt 2>&1 || { tail -20 gpurun_out/ab_group_pipe.txt; exit 1; }
grep '^{' gpurun_out/ab_group_pipe.txt
