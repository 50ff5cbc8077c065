#!/bin/bash
# GPU box: the [CLS]-last-layer tests + the text / fp32x3 suites, then the bench line, then
# (PROF=1) the x3 encoder profiles and the fenced bench-window profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-cls}
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_cls_last.py tests/test_gpu_fp32x3.py tests/test_gpu_parity.py} -m gpu -x -v -s \
  --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/${T}_pytest.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python -u bench.py --json-out gpurun_out/${T}_bench.json > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
python3 tools/summ_bench.py gpurun_out/${T}_bench.json 2>/dev/null || tail -c 1500 gpurun_out/${T}_bench.log
[ -z "$PROF" ] && exit 0
PREC=fp32x3 ENCS="text image" bash tools/gpu_enc_prof.sh && PREC=fp32x3 STEPS=10 bash tools/gpu_prof_bench.sh
