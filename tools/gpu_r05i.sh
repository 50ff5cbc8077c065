#!/bin/bash
# Round 5, step i: the fp32 GELU of the split / f32 GEMM epilogues on packed math (gelu_f32_x2): the whole
# -m gpu suite, then cross-build A/Bs with bit-identity checks (fp32x3 text + fused step, exact-fp32 text).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05i_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05i_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in "text fp32x3 3" "pipeline fp32x3 3" "text fp32 1"; do
  set -- $cfg
  ENC=$1 PREC=$2 ROUNDS=$3 bash tools/gpu_ab_lib.sh > gpurun_out/r05i_ab_$1_$2.txt 2>&1 || { cat gpurun_out/r05i_ab_$1_$2.txt; exit 1; }
  cat gpurun_out/r05i_ab_$1_$2.txt
done
