#!/bin/bash
# Round 5, step z: gemm_glds_group_m 8 (default) vs 4, longer interleaved A/Bs: the fused step at fp32x3
# and f16, ResNet50 alone at fp32x3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "pipeline fp32x3 9" "pipeline f16 5" "image fp32x3 5"; do
  set -- $cfg
  timeout -k 10 500 python -u tools/ab_option.py --enc $1 --precision $2 --opt gemm_glds_group_m \
    --values 8 4 --rounds $3 > gpurun_out/r05z_ab_groupm_$1_$2.txt 2>&1 || { tail -5 gpurun_out/r05z_ab_groupm_$1_$2.txt; exit 1; }
  grep '"ms"' gpurun_out/r05z_ab_groupm_$1_$2.txt
done
