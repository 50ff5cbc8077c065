#!/bin/bash
# HBM traffic of the fp32x3 BERT FFN1 GEMM (the headline's roofline kernel): separate rocprofv3
# --pmc passes (FETCH_SIZE, WRITE_SIZE, MFMA busy, L2 hits / misses) over the fp32x3 text encoder at B=256 with
# the split tile pinned to the FFN1 pin (TILE, default 70256: the K-interleaved split tile), then
# profiles/ffn1_x3_traffic.json (FETCH_SIZE doubled: MI355X_MICROARCH.md gfx950).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TILE=${TILE:-70256}
OUT=gpurun_out/pmc_ffn1_x3
EXTRA=${GM:+--opt gemm_glds_group_m=$GM}  # optional glds tile order
rm -rf $OUT; mkdir -p $OUT
i=0
for SET in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "gemm_glds_kernel|gemm_pp_kernel" -d $OUT/p$i -o p -f csv -- \
    python3 tools/encoder_profile.py --enc text --precision fp32x3 --iters 3 --opt gemm_bn=$TILE $EXTRA > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($SET) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
TILE=$TILE GM=$GM python3 - <<'PY'
import csv, glob, json, os
from collections import defaultdict
root = 'gpurun_out/pmc_ffn1_x3'
vals = defaultdict(list)
for f in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
    for row in csv.DictReader(open(f)):
        k, g = row.get('Kernel_Name', ''), row.get('Grid_Size', '')
        vals[(k, g, row['Counter_Name'])].append(float(row['Counter_Value']))
# FFN1: M = 32768, N = 3072 on a 256 x 256 tile -> 1536 blocks x 512 threads (QKV: 1152, N = 768: 384)
ffn = {key: v for key, v in vals.items() if key[1] == '786432'}
by_k = defaultdict(dict)
for (k, g, c), v in ffn.items():
    v = sorted(v)[len(v) // 4:] or v  # drop the first launches
    by_k[(k, g)][c] = sum(v) / len(v)
(k, g), c = next(iter(by_k.items()))
fetch = 2 * c['FETCH_SIZE'] * 1024  # KB units; x2 gfx950 correction
write = c['WRITE_SIZE'] * 1024
out = {'tile': int(os.environ['TILE']), 'M': 32768, 'kernel': k[:100], 'bytes_per_launch': fetch + write,
       'fetch_bytes_corrected': fetch, 'write_bytes': write,
       'algorithmic_bytes': 4 * (32768 * 768 + 3072 * 768 + 32768 * 3072),
       'mfma_busy_frac': c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(c.get('GRBM_GUI_ACTIVE', 1) / 8 * 1024, 1),
       'l2_hits': c.get('TCC_HIT_sum'), 'l2_misses': c.get('TCC_MISS_sum'),
       'l2_hit_rate': c.get('TCC_HIT_sum', 0) / max(c.get('TCC_HIT_sum', 0) + c.get('TCC_MISS_sum', 0), 1),
       'source': 'rocprofv3 --pmc, separate FETCH_SIZE / WRITE_SIZE / SQ / TCC hit-miss passes (tools/pmc_ffn1_x3.sh) over the '
                 'fp32x3 text encoder at B=256; FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950); algorithmic '
                 'bytes = fp32-equivalent operands (each hi+lo pair is 4 B)'}
out['gemm_glds_group_m'] = int(os.environ['GM']) if os.environ.get('GM') else 'TextEncoder default (4)'
json.dump(out, open('gpurun_out/ffn1_x3_traffic%s.json' % ('_gm' + os.environ['GM'] if os.environ.get('GM') else ''), 'w'), indent=1)
print(json.dumps(out, indent=1))
PY
