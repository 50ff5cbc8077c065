#!/bin/bash
# Round 5, step p (final validation, tile 72128 in on the shipped libraries): the whole -m gpu suite and the default bench
# line (gpu_tests_bench.sh, TAG r05p), smoke, then the rocprofv3 kernel stats of the fp32x3 bench window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r05p bash tools/gpu_tests_bench.sh || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r05p_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r05p_smoke.log; [ $rc -ne 0 ] && exit $rc
PREC=fp32x3 bash tools/gpu_prof_bench.sh > gpurun_out/r05p_prof.log 2>&1 || { tail -5 gpurun_out/r05p_prof.log; exit 1; }
head -12 gpurun_out/bench_prof_grid_fp32x3.txt
ENC=image_mbv2 PREC=fp32x3 bash tools/pmc_sq.sh > gpurun_out/r05p_pmcsq.log 2>&1 || { tail -5 gpurun_out/r05p_pmcsq.log; exit 1; }
head -8 gpurun_out/pmcsq_fp32x3_image_mbv2.txt | cut -c1-72,200-260
