#!/bin/bash
# Round 5, step g: (1) the FFN1 tile's clock with and without its K-loop operand loads (pmc_ffn1_clock.sh);
# (2) MobileNetV2 stem / depthwise FMAs packed (v_pk_fma_f32): MobileNetV2 GPU tests, then cross-build A/Bs
# (bit-identity) at fp32x3 and f16; (3) PMC roofline tables of MobileNetV2 (fp32x3, f16) and ResNet50 (fp32x3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/pmc_ffn1_clock.sh > gpurun_out/r05g_ffn1_clock.log 2>&1 || { tail -20 gpurun_out/r05g_ffn1_clock.log; exit 1; }
tail -25 gpurun_out/r05g_ffn1_clock.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mbv2 or mobilenet" \
  > gpurun_out/r05g_pytest_mbv2.log 2>&1
rc=$?; tail -2 gpurun_out/r05g_pytest_mbv2.log; [ $rc -ne 0 ] && exit $rc
for cfg in "image_mbv2 fp32x3" "image_mbv2 f16"; do
  set -- $cfg
  ENC=$1 PREC=$2 ROUNDS=3 bash tools/gpu_ab_lib.sh > gpurun_out/r05g_ab_$1_$2.txt 2>&1 || { cat gpurun_out/r05g_ab_$1_$2.txt; exit 1; }
  cat gpurun_out/r05g_ab_$1_$2.txt
done
ENCS=image_mbv2 PREC=fp32x3 bash tools/pmc_encoders.sh > gpurun_out/r05g_pmc_mbv2_x3.log 2>&1 || { tail -5 gpurun_out/r05g_pmc_mbv2_x3.log; exit 1; }
ENCS=image_mbv2 PREC=f16 bash tools/pmc_encoders.sh > gpurun_out/r05g_pmc_mbv2_f16.log 2>&1 || { tail -5 gpurun_out/r05g_pmc_mbv2_f16.log; exit 1; }
ENCS=image PREC=fp32x3 bash tools/pmc_encoders.sh > gpurun_out/r05g_pmc_image_x3.log 2>&1 || { tail -5 gpurun_out/r05g_pmc_image_x3.log; exit 1; }
head -30 gpurun_out/pmcrep_fp32x3_image_mbv2.txt
