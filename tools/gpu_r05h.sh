#!/bin/bash
# Round 5, step h: price the split GEMM epilogue: the probe build's FFN1 tile with (gemm_debug 0) and
# without (gemm_debug 2) its epilogue, kernel trace by grid.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 2; do
  rm -rf gpurun_out/prof_ffn1_noepi_$v
  MEC_LIB=multimodal-emotion-classification_amd/mec/libmec_hip_probes.so timeout -k 10 240 rocprofv3 --kernel-trace --stats \
    -d gpurun_out/prof_ffn1_noepi_$v -o run -- \
    python3 tools/encoder_profile.py --enc text --iters 5 --precision fp32x3 --opt gemm_debug=$v \
    > gpurun_out/prof_ffn1_noepi_$v.log 2>&1 || { tail -5 gpurun_out/prof_ffn1_noepi_$v.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/prof_ffn1_noepi_$v/run_results.db --window spin --steps 5 --by-grid \
    > gpurun_out/r05_ffn1_noepi_$v.txt
  head -5 gpurun_out/r05_ffn1_noepi_$v.txt
done
