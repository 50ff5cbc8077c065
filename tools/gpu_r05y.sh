#!/bin/bash
# Round 5, step y: the split GEMMs' tile order (gemm_glds_group_m: groups of G M panels walked M-fastest
# inside each XCD's range; 0 = row-major) in the fused fp32x3 step and BERT alone, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in pipeline text; do
  timeout -k 10 400 python -u tools/ab_option.py --enc $e --precision fp32x3 --opt gemm_glds_group_m \
    --values 8 4 16 0 --rounds 5 > gpurun_out/r05y_ab_groupm_$e.txt 2>&1 || { tail -5 gpurun_out/r05y_ab_groupm_$e.txt; exit 1; }
  grep '"ms"' gpurun_out/r05y_ab_groupm_$e.txt
done
