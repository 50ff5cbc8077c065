#!/bin/bash
# Round 5, step aa: BERT handles at gemm_glds_group_m 4 (engine.TextEncoder): the whole -m gpu suite, the
# default bench line, smoke, and the FFN1 PMC traffic passes on the shipped configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r05aa bash tools/gpu_tests_bench.sh || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r05aa_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r05aa_smoke.log; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_ffn1_x3.sh > gpurun_out/r05aa_pmc_ffn1.log 2>&1 || { tail -5 gpurun_out/r05aa_pmc_ffn1.log; exit 1; }
tail -14 gpurun_out/r05aa_pmc_ffn1.log
