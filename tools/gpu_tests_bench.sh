#!/bin/bash
# GPU box: the whole -m gpu suite, then the default bench line (stops at the first failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  ${PYTEST_ARGS} > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/${TAG}_pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/${TAG}_pytest_gpu.log | head -20; exit $rc; fi
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS} --json-out gpurun_out/${TAG}_bench.json \
  > gpurun_out/${TAG}_bench.log 2>&1
brc=$?
python3 -c "
import json,sys; d=json.load(open('gpurun_out/${TAG}_bench.json'))
f=d.get('f16_fast_path',{})
print('fp32', round(d['value']), 'ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],3), '| f16', round(f.get('value',0)), 'ms', round(f.get('ms_per_step',0),2))
" 2>/dev/null || tail -5 gpurun_out/${TAG}_bench.log
exit $brc
