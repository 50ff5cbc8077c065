#!/bin/bash
# default bench (both precisions, parity, per-config, CPU baseline), then the per-rank
# multi-GPU batch (1024) on one GPU at both precisions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -c 3000 gpurun_out/bench.log
timeout -k 10 600 python bench.py --batch 1024 --steps 5 --warmup 2 --no-cpu-baseline --no-configs --no-parity > gpurun_out/bench_b1024.log 2>&1 || { tail -30 gpurun_out/bench_b1024.log; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/bench_b1024.log'):
    if l.startswith('{'):
        d = json.loads(l); print('B=1024', d['precision'], round(d['value'], 1), 'samples/s', round(d['ms_per_step'], 2), 'ms/step')
PY
