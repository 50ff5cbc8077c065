#!/bin/bash
# rocprofv3 kernel-trace stats of one bench.py precision's timed window (between the two
# spin markers), by kernel and by grid; writes gpurun_out/bench_prof_<prec>.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=${PREC:-f16}
rm -rf gpurun_out/prof_bench_$P; mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_$P -o run -- python3 bench.py --precision $P --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-configs --no-parity > gpurun_out/prof_bench_$P.log 2>&1 || { tail -5 gpurun_out/prof_bench_$P.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_bench_$P/run_results.db --window spin --steps ${STEPS:-10} > gpurun_out/bench_prof_$P.txt
python3 tools/prof_summary.py gpurun_out/prof_bench_$P/run_results.db --window spin --steps ${STEPS:-10} --by-grid > gpurun_out/bench_prof_grid_$P.txt
tail -c 600 gpurun_out/prof_bench_$P.log
head -30 gpurun_out/bench_prof_$P.txt
