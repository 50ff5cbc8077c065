#!/bin/bash
# fp32x3 BERT FFN1 tile in the fused step (gemm_x3_tag 4*100000 + tile): 70256 (the pin) vs the
# 256 x 128 / 128 x 128 interleaved tiles, whose smaller LDS footprint lets an image-stream workgroup
# share a CU; then BERT alone.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_mbv2.py \
  tests/test_gpu_fp32x3.py -k "tail or tile_forms or chunked" > gpurun_out/r04_newtests2.log 2>&1 \
  || { tail -30 gpurun_out/r04_newtests2.log; exit 1; }
tail -3 gpurun_out/r04_newtests2.log
timeout -k 10 400 python3 -u tools/ab_option.py --enc pipeline --opt gemm_x3_tag --values 470256 470128 471128 \
  --precision fp32x3 > gpurun_out/r04_ab_ffn1x3_pipeline.txt 2>&1 || exit 1
tail -3 gpurun_out/r04_ab_ffn1x3_pipeline.txt
timeout -k 10 300 python3 -u tools/ab_option.py --enc text --opt gemm_x3_tag --values 470256 470128 471128 \
  --precision fp32x3 > gpurun_out/r04_ab_ffn1x3_text.txt 2>&1 || exit 1
tail -3 gpurun_out/r04_ab_ffn1x3_text.txt
timeout -k 10 400 python3 -u tools/ab_option.py --enc image --opt resnet_chunk --values 0 16 32 64 \
  --precision fp32x3 > gpurun_out/r04_ab_chunk_x3_image.txt 2>&1 || exit 1
tail -4 gpurun_out/r04_ab_chunk_x3_image.txt
timeout -k 10 400 python3 -u tools/ab_option.py --enc pipeline --opt resnet_chunk --values 0 32 64 \
  --precision fp32x3 > gpurun_out/r04_ab_chunk_x3_pipeline.txt 2>&1 || exit 1
tail -3 gpurun_out/r04_ab_chunk_x3_pipeline.txt
timeout -k 10 300 python3 -u tools/ab_option.py --enc image_mbv2 --opt mbv2_x3_tile --values 0 4 \
  --precision fp32x3 > gpurun_out/r04_ab_mbv2x3_tile.txt 2>&1 || exit 1
tail -2 gpurun_out/r04_ab_mbv2x3_tile.txt
timeout -k 10 300 python3 -u tools/ab_option.py --enc image_mbv2 --opt mbv2_tail --values 0 1 \
  --precision f16 > gpurun_out/r04_ab_mbv2_tail.txt 2>&1 || exit 1
tail -2 gpurun_out/r04_ab_mbv2_tail.txt
