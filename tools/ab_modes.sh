#!/bin/bash
# Same-box A/B of the fused bench's scheduling modes (bench.py flags), alternated ROUNDS times.
#   bash tools/ab_modes.sh [ROUNDS] -- "" "--serial" "--text-priority 0" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-2}; shift; [ "$1" = "--" ] && shift
for i in $(seq 1 $R); do
  for mode in "$@"; do
    timeout -k 10 300 python bench.py --precision f16 --no-cpu-baseline --no-configs --no-parity $mode > gpurun_out/ab_modes.log 2>&1 || { tail -5 gpurun_out/ab_modes.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ab_modes.log'):
    if l.startswith('{'):
        d=json.loads(l); print('mode [$mode]', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')
"
  done
done
