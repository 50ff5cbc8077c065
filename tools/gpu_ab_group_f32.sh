#!/bin/bash
# fp32 engine: A/B of the tile order (gemm_group_m) on BERT alone and on the fused step, then
# the FFN1 PMC traffic at the default order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_option.py --enc text --precision fp32 --opt gemm_group_m --rounds 5 --iters 3 --values 0 4 8 > gpurun_out/ab_group_text32.txt 2>&1 || { tail -20 gpurun_out/ab_group_text32.txt; exit 1; }
grep '^{' gpurun_out/ab_group_text32.txt
timeout -k 10 300 python3 tools/ab_option.py --enc pipeline --precision fp32 --opt gemm_group_m --rounds 5 --iters 2 --values 0 8 > gpurun_out/ab_group_pipe32.txt 2>&1 || { tail -20 gpurun_out/ab_group_pipe32.txt; exit 1; }
grep '^{' gpurun_out/ab_group_pipe32.txt
bash tools/pmc_ffn1_f32.sh | tail -3
