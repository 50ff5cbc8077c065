#!/bin/bash
# GPU box: the fp32x3 fused step under each stream scheduling mode (bench.py flags), one process per mode
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python -u bench.py --precision fp32x3 --no-configs --no-parity --no-cpu-baseline --steps 20 "$@" \
    --json-out gpurun_out/modes.json > gpurun_out/modes.log 2>&1 || { tail -5 gpurun_out/modes.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/modes.json')); print(sys.argv[1:], round(d['value']), round(d['ms_per_step'],2))" "$@"
}
run
run --text-priority 0 --image-priority 1
run --text-priority 0
run --serial
run
