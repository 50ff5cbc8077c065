#!/bin/bash
# fp32x3 fused QKV + attention with 1 or 2 heads per workgroup (bert_qkv_attn_x3_heads): the
# bit-identity test, then text alone and the fused step at B = 256 (interleaved in one process).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_fp32x3.py -k "fused_qkv or text_fp32x3" > gpurun_out/r04_qkvx3_heads_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r04_qkvx3_heads_tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r04_qkvx3_heads_tests.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u tools/ab_option.py --enc text --opt bert_qkv_attn_x3_heads --values 2 1 --precision fp32x3 \
  > gpurun_out/r04_ab_qkvx3_heads_text.txt 2>&1 || exit 1
grep enc gpurun_out/r04_ab_qkvx3_heads_text.txt
timeout -k 10 300 python3 -u tools/ab_option.py --enc pipeline --opt bert_qkv_attn_x3_heads --values 2 1 --precision fp32x3 \
  > gpurun_out/r04_ab_qkvx3_heads_pipeline.txt 2>&1 || exit 1
grep enc gpurun_out/r04_ab_qkvx3_heads_pipeline.txt
PREC=fp32x3 ENCS="text" bash tools/gpu_enc_prof.sh
