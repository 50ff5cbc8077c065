#!/bin/bash
# Round 5, step c: the round-4 library (libmec_hip_base.so, commit 50e1d48) against this tree's on the fp32x3
# fused pipeline (after the cscale skip), then this tree's activation-plane scales on / off
# (x3_plane_scale, read at handle creation) on the text and image encoders and the pipeline, alternating
# processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ENC=pipeline PREC=fp32x3 ROUNDS=3 bash tools/gpu_ab_lib.sh > gpurun_out/r05_ab_lib_r04_pipeline_c.txt 2>&1 || exit $?
tail -7 gpurun_out/r05_ab_lib_r04_pipeline_c.txt
for e in text image pipeline; do
  OUT=gpurun_out/r05_ab_planescale_$e.txt; : > $OUT
  for r in 1 2 3; do
    for v in 1 0; do
      timeout -k 10 240 python3 -u tools/ab_option.py --enc $e --precision fp32x3 --opt gemm_autotune --values 1 \
        --rounds 5 --set x3_plane_scale=$v 2>/dev/null | sed "s/^/x3_plane_scale=$v /" >> $OUT || exit 1
    done
  done
  cat $OUT
done
ENCS=image_mbv2 PREC=fp32x3 bash tools/gpu_enc_prof.sh || exit $?
head -14 gpurun_out/enc_fp32x3_image_mbv2.txt
ENC=image_mbv2 PREC=fp32x3 bash tools/pmc_sq.sh || exit $?
