#!/bin/bash
# Round 5, step s: one-stage split tiles 73128 / 73064 (128 x 128 / 128 x 64) as
# autotune candidate: fp32x3 tests, the tiles the autotuner picks (MEC_GEMM_TRACE), cross-build A/Bs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32x3.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05s_pytest_x3.log 2>&1
rc=$?; tail -2 gpurun_out/r05s_pytest_x3.log; [ $rc -ne 0 ] && exit $rc
for e in text image; do
  MEC_GEMM_TRACE=1 timeout -k 10 200 python3 tools/encoder_profile.py --enc $e --iters 2 --precision fp32x3 \
    > gpurun_out/r05s_trace_$e.log 2>&1 || { tail -5 gpurun_out/r05s_trace_$e.log; exit 1; }
  grep "MEC_GEMM" gpurun_out/r05s_trace_$e.log | grep -o "M=[0-9]* N=[0-9]* K=[0-9]*.*tile=[0-9]*" | sed 's/ H=.*split/ split/' | sort | uniq -c
done
for cfg in "text fp32x3 3" "image fp32x3 3" "pipeline fp32x3 3"; do
  set -- $cfg
  ENC=$1 PREC=$2 ROUNDS=$3 bash tools/gpu_ab_lib.sh > gpurun_out/r05s_ab_$1_$2.txt 2>&1 || { cat gpurun_out/r05s_ab_$1_$2.txt; exit 1; }
  cat gpurun_out/r05s_ab_$1_$2.txt
done
