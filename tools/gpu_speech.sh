#!/bin/bash
# Speech DNN: the flow-kernel tests, then rocprofv3 kernel stats of the speech encoder alone at
# B=32 and B=256 (the layer-split dataflow kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_speech_flow.py tests/test_gpu_parity.py -k "flow or speech" -x -v -s \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_speech.log 2>&1 || { tail -40 gpurun_out/pytest_speech.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_speech.log | tail -2
for B in 32 256; do
  for impl in 0; do
    d=gpurun_out/prof_speech_b${B}_i$impl
    rm -rf $d
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run -- \
      python3 tools/encoder_profile.py --enc speech --iters 50 --batch $B > $d.log 2>&1 || { echo "rocprof B=$B impl=$impl rc=$?"; tail -5 $d.log; exit 1; }
    python3 tools/prof_summary.py $d/run_results.db --window spin --steps 50 > gpurun_out/speech_b${B}_i$impl.txt
    echo "B=$B impl=$impl $(grep ms_per_iter $d.log)"
    head -3 gpurun_out/speech_b${B}_i$impl.txt | cut -c1-200
  done
done
timeout -k 10 120 python tools/speech_probe.py 32 > gpurun_out/speech_probe.log 2>&1 && tail -6 gpurun_out/speech_probe.log
