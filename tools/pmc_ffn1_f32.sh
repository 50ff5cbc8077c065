#!/bin/bash
# HBM traffic of the fp32 BERT FFN1 GEMM (the fp32 bench line's roofline kernel): separate
# rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, MFMA busy) over the fp32 text encoder at
# B=256, then profiles/ffn1_f32_traffic.json (FETCH_SIZE doubled: MI355X_MICROARCH.md gfx950).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ffn1_f32
rm -rf $OUT; mkdir -p $OUT
i=0
for SET in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "gemm_f32_kernel" -d $OUT/p$i -o p -f csv -- \
    python3 tools/encoder_profile.py --enc text --precision fp32 --iters 3 --opt gemm_f32_tag=400008 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($SET) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 - <<'PY'
import csv, glob, json, os
from collections import defaultdict
root = 'gpurun_out/pmc_ffn1_f32'
vals = defaultdict(list)
for f in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
    for row in csv.DictReader(open(f)):
        k, g = row.get('Kernel_Name', ''), row.get('Grid_Size', '')
        vals[(k, g, row['Counter_Name'])].append(float(row['Counter_Value']))
# FFN1: M = 32768, N = 3072 -> grid = blocks * threads; pick the 256x256 tile kernels (FFN1 only)
ffn = {key: v for key, v in vals.items() if '<256, 256, 2, 4, 2, 0, 16>' in key[0] and key[1] == '786432'}
for key, v in sorted(ffn.items()):
    print(key[0][:70], key[1], key[2], len(v), sum(v) / len(v))
by_k = defaultdict(dict)
for (k, g, c), v in ffn.items():
    v = sorted(v)[len(v) // 4:] or v  # drop the autotune's first launches
    by_k[(k, g)][c] = sum(v) / len(v)
(k, g), c = next(iter(by_k.items()))
fetch = 2 * c['FETCH_SIZE'] * 1024  # KB units; x2 gfx950 correction
write = c['WRITE_SIZE'] * 1024
tile = 8 if ', 16>' in k else 4
out = {'tile': tile, 'M': 32768, 'kernel': k[:90], 'bytes_per_launch': fetch + write,
       'fetch_bytes_corrected': fetch, 'write_bytes': write,
       'algorithmic_bytes': 4 * (32768 * 768 + 3072 * 768 + 32768 * 3072),
       'mfma_busy_frac': c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(c.get('GRBM_GUI_ACTIVE', 1) / 8 * 1024, 1),
       'source': 'rocprofv3 --pmc, separate FETCH_SIZE / WRITE_SIZE / SQ passes (tools/pmc_ffn1_f32.sh) over the '
                 'fp32 text encoder at B=256; FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950)'}
json.dump(out, open('gpurun_out/ffn1_f32_traffic.json', 'w'), indent=1)
print(json.dumps(out, indent=1))
PY
