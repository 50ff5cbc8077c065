#!/bin/bash
# GPU tests (whole -m gpu suite), smoke, then the default bench. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/bench.log'):
    if l.startswith('{'):
        d = json.loads(l)
        print(d['precision'], round(d['value']), 'samples/s', round(d['ms_per_step'], 2), 'ms/step; FFN1 frac',
              round(d['roofline']['frac'], 3), 'iso', round(d['roofline']['frac_isolated'] or 0, 3),
              {k: (v['probs_max_abs_err'], v['argmax_agree']) for k, v in d.get('parity', {}).items() if k != 'rows'})
PY
