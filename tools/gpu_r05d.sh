#!/bin/bash
# Round 5, step d: the fp32x3 FFN1 tile with and without its K-loop operand loads (probe build, gemm_debug 1)
# under rocprofv3, the FFN1 PMC passes (traffic json), then the whole -m gpu suite, smoke and the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
  rm -rf gpurun_out/prof_ffn1_noload_$v
  L=multimodal-emotion-classification_amd/mec/libmec_hip.so
  [ $v = 1 ] && L=multimodal-emotion-classification_amd/mec/libmec_hip_probes.so
  MEC_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ffn1_noload_$v -o run -- \
    python3 tools/encoder_profile.py --enc text --iters 5 --precision fp32x3 --opt gemm_debug=$v \
    > gpurun_out/prof_ffn1_noload_$v.log 2>&1 || { tail -5 gpurun_out/prof_ffn1_noload_$v.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/prof_ffn1_noload_$v/run_results.db --window spin --steps 5 --by-grid \
    > gpurun_out/r05_ffn1_noload_$v.txt
  head -4 gpurun_out/r05_ffn1_noload_$v.txt
done
bash tools/pmc_ffn1_x3.sh > gpurun_out/r05_pmc_ffn1.log 2>&1 || { tail -5 gpurun_out/r05_pmc_ffn1.log; exit 1; }
tail -20 gpurun_out/r05_pmc_ffn1.log
TAG=r05d bash tools/gpu_tests_bench.sh || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r05d_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r05d_smoke.log; exit $rc
