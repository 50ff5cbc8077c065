#!/bin/bash
# Per-encoder isolated rocprofv3 kernel profiles (text, image, speech, fusion), summaries
# written to gpurun_out/enc_<name>.txt. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for e in ${ENCS:-text image speech fusion}; do
  rm -rf gpurun_out/prof_${PREC:-f16}_$e
  MEC_GEMM_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${PREC:-f16}_$e -o run -- \
    python3 tools/encoder_profile.py --enc $e --iters 5 --precision ${PREC:-f16} > gpurun_out/enc_${PREC:-f16}_$e.log 2>&1 || { echo "rocprof $e rc=$?"; exit 1; }
  python3 tools/prof_summary.py gpurun_out/prof_${PREC:-f16}_$e/run_results.db --window spin --steps 5 --by-grid > gpurun_out/enc_${PREC:-f16}_$e.txt
  python3 tools/prof_summary.py gpurun_out/prof_${PREC:-f16}_$e/run_results.db --window spin --steps 5 --sequence > gpurun_out/seq_${PREC:-f16}_$e.txt
  grep ms_per_iter gpurun_out/enc_${PREC:-f16}_$e.log
  tail -1 gpurun_out/enc_${PREC:-f16}_$e.txt
done
