#!/bin/bash
# Same-box A/B of the fused bench: the in-tree library against another build of the same ABI
# (MEC_LIB), alternated ROUNDS times; prints each run's f16 samples/s and ms/step.
#   [BENCH_FLAGS=--serial] bash tools/ab_bench.sh build/ab/libmec_prev.so [ROUNDS]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OTHER=$1; R=${2:-2}
for i in $(seq 1 $R); do
  for lib in "$OTHER" tree; do
    if [ "$lib" = tree ]; then
      timeout -k 10 300 python bench.py --precision f16 --no-cpu-baseline --no-configs --no-parity ${BENCH_FLAGS} > gpurun_out/ab_bench.log 2>&1 || { tail -5 gpurun_out/ab_bench.log; exit 1; }
    else
      MEC_LIB=$lib timeout -k 10 300 python bench.py --precision f16 --no-cpu-baseline --no-configs --no-parity ${BENCH_FLAGS} > gpurun_out/ab_bench.log 2>&1 || { tail -5 gpurun_out/ab_bench.log; exit 1; }
    fi
    python3 -c "
import json,sys
for l in open('gpurun_out/ab_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$lib', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step', 'FFN1 frac', round(d['roofline']['frac'],3))
"
  done
done
