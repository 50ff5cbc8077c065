#!/bin/bash
# f16 fused QKV + attention with 1 or 2 heads per workgroup (bert_qkv_attn_heads): the bit-identity
# test, then text alone and the f16 fused step at B = 256 (interleaved in one process).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "qkv_attn" > gpurun_out/r04_qkv_heads_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r04_qkv_heads_tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r04_qkv_heads_tests.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u tools/ab_option.py --enc text --opt bert_qkv_attn_heads --values 2 1 --precision f16 \
  > gpurun_out/r04_ab_qkv_heads_text.txt 2>&1 || exit 1
grep enc gpurun_out/r04_ab_qkv_heads_text.txt
timeout -k 10 300 python3 -u tools/ab_option.py --enc pipeline --opt bert_qkv_attn_heads --values 2 1 --precision f16 \
  > gpurun_out/r04_ab_qkv_heads_pipeline.txt 2>&1 || exit 1
grep enc gpurun_out/r04_ab_qkv_heads_pipeline.txt
