#!/bin/bash
# Round 5, step t: BERT FFN2 pinned to the one-stage 72128 outside the fused step (no longer an autotune
# candidate): the whole -m gpu suite, cross-build A/Bs (BERT alone, the fused step, ResNet50), then the
# default bench line and smoke on the final libraries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05t_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05t_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in "text fp32x3 3" "pipeline fp32x3 3" "image fp32x3 2"; do
  set -- $cfg
  ENC=$1 PREC=$2 ROUNDS=$3 bash tools/gpu_ab_lib.sh > gpurun_out/r05t_ab_$1_$2.txt 2>&1 || { cat gpurun_out/r05t_ab_$1_$2.txt; exit 1; }
  cat gpurun_out/r05t_ab_$1_$2.txt
done
NO_TESTS=1
timeout -k 10 600 python -u bench.py --json-out gpurun_out/r05t_bench.json > gpurun_out/r05t_bench.log 2>&1 || { tail -5 gpurun_out/r05t_bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05t_bench.json')); f=d['f16_fast_path']
print('fp32x3', round(d['value']), round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],3), {k: round(v['ms_per_batch'],3) for k,v in d['per_config'].items()})"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r05t_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r05t_smoke.log; exit $rc
