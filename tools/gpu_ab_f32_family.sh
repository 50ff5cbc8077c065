#!/bin/bash
# fp32 engine: autotune over both MFMA families (0) vs one family (16 / 32) on the encoders and the fused step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in image text; do
  timeout -k 10 400 python3 tools/ab_option.py --enc $e --precision fp32 --opt gemm_f32_family --rounds 5 --iters 3 --values 0 16 32 > gpurun_out/ab_fam_$e.txt 2>&1 || { tail -20 gpurun_out/ab_fam_$e.txt; exit 1; }
  grep '^{' gpurun_out/ab_fam_$e.txt
done
timeout -k 10 400 python3 tools/ab_option.py --enc pipeline --precision fp32 --opt gemm_f32_family --rounds 5 --iters 2 --values 0 16 > gpurun_out/ab_fam_pipe.txt 2>&1 || { tail -20 gpurun_out/ab_fam_pipe.txt; exit 1; }
grep '^{' gpurun_out/ab_fam_pipe.txt
