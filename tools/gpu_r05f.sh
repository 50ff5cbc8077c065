#!/bin/bash
# Round 5, step f: the GEMM engine's operand loads issued from asm (glds16) so its fragment reads keep
# counted lgkmcnt waits, and the split tiles' fragment reads in two groups: the whole -m gpu suite on the
# new build, then cross-build A/Bs (libmec_hip_base.so = the previous build) with bit-identity checks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05f_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05f_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in "pipeline fp32x3 3" "text fp32x3 2" "image fp32x3 2" "pipeline f16 2"; do
  set -- $cfg
  ENC=$1 PREC=$2 ROUNDS=$3 bash tools/gpu_ab_lib.sh > gpurun_out/r05f_ab_$1_$2.txt 2>&1 || { cat gpurun_out/r05f_ab_$1_$2.txt; exit 1; }
  cat gpurun_out/r05f_ab_$1_$2.txt
done
