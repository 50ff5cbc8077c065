#!/bin/bash
# Round 5, step u: the fused fp32x3 step with the split-tile autotune candidates restricted (gemm_x3_cands,
# process default before the handles are created; bit i = 70256, 70128, 71128, 71064, 70064), alternating
# processes, bit-identity against mask 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/r05u_ab_x3cands_pipeline.txt
: > $OUT
for r in 1 2 3; do
  for m in 0 3 7 11 19; do
    timeout -k 10 240 python3 -u tools/ab_option.py --enc pipeline --precision fp32x3 --set gemm_x3_cands=$m \
      --opt gemm_autotune --values 1 --rounds 5 --save gpurun_out/ab_cands_$m.npz 2>/dev/null | sed "s/^/mask $m /" >> $OUT || exit 1
  done
done
cat $OUT
python3 - <<'PY'
import numpy as np
a = np.load('gpurun_out/ab_cands_0.npz')
for m in (3, 7, 11, 19):
    b = np.load('gpurun_out/ab_cands_%d.npz' % m)
    print(m, 'bit-identical:', all(np.array_equal(a[k], b[k]) for k in a.files))
PY
