#!/bin/bash
# Round 5, step v: rocprofv3 kernel stats of the fp32x3 bench window on the final libraries, then the FFN1
# PMC traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PREC=fp32x3 bash tools/gpu_prof_bench.sh > gpurun_out/r05v_prof.log 2>&1 || { tail -5 gpurun_out/r05v_prof.log; exit 1; }
head -6 gpurun_out/bench_prof_grid_fp32x3.txt
bash tools/pmc_ffn1_x3.sh > gpurun_out/r05v_pmc_ffn1.log 2>&1 || { tail -5 gpurun_out/r05v_pmc_ffn1.log; exit 1; }
tail -16 gpurun_out/r05v_pmc_ffn1.log
