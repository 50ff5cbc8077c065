#!/bin/bash
# Round 5, step r: GEMM epilogue stores non-temporal (gemm_nt_store 0 / 1), same-process A/Bs with
# bit-identity: BERT, ResNet50, the fused step (fp32x3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in text image pipeline; do
  timeout -k 10 400 python -u tools/ab_option.py --enc $e --precision fp32x3 --opt gemm_nt_store \
    --values 0 1 --rounds 7 > gpurun_out/r05r_ab_ntstore_$e.txt 2>&1 || { tail -5 gpurun_out/r05r_ab_ntstore_$e.txt; exit 1; }
  grep '"ms"' gpurun_out/r05r_ab_ntstore_$e.txt
done
