#!/bin/bash
# Cross-build A/B: mec/libmec_hip_base.so (the previous build, copied aside) against mec/libmec_hip.so,
# alternating processes (ROUNDS each), on one encoder (ENC, PREC); the outputs of both builds are
# compared bit for bit. Usage: ENC=image_mbv2 PREC=fp32x3 bash tools/gpu_ab_lib.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ENC=${ENC:-image_mbv2}; PREC=${PREC:-fp32x3}; ROUNDS=${ROUNDS:-3}; OPT=${OPT:-gemm_autotune}; VAL=${VAL:-1}
OUT=gpurun_out/ab_lib_${ENC}_${PREC}.txt
: > $OUT
for r in $(seq $ROUNDS); do
  for lib in base new; do
    if [ $lib = base ]; then L=multimodal-emotion-classification_amd/mec/libmec_hip_base.so; else L=multimodal-emotion-classification_amd/mec/libmec_hip.so; fi
    MEC_LIB=$L timeout -k 10 240 python3 -u tools/ab_option.py --enc $ENC --precision $PREC --opt $OPT --values $VAL \
      --rounds 5 --save gpurun_out/ab_lib_$lib.npz 2>/dev/null | sed "s/^/$lib /" >> $OUT || exit 1
  done
done
cat $OUT
python3 - <<'PY'
import numpy as np
a, b = np.load('gpurun_out/ab_lib_base.npz'), np.load('gpurun_out/ab_lib_new.npz')
print('bit-identical:', all(np.array_equal(a[k], b[k]) for k in a.files),
      [float(np.abs(a[k].astype(np.float64) - b[k]).max()) for k in a.files])
PY
