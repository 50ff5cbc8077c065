#!/bin/bash
# HBM traffic of the f16 BERT FFN1 GEMM (gemm_pp_kernel with GELU, M = 32768, N = 3072, K = 768)
# per tile order (gemm_group_m): separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE
# over the text encoder at B = 256 (FETCH_SIZE doubled: MI355X_MICROARCH.md, gfx950), then
# gpurun_out/ffn1_traffic_gm<G>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for G in ${GROUPS_M:-0 8}; do
  OUT=gpurun_out/pmc_ffn1_gm$G
  rm -rf $OUT; mkdir -p $OUT
  i=0
  for SET in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "gemm_pp_kernel" -d $OUT/p$i -o p -f csv -- \
      python3 tools/encoder_profile.py --enc text --iters 3 --opt gemm_group_m=$G > $OUT/p$i.log 2>&1
    rc=$?
    echo "group_m $G pass $i ($SET) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
  done
  python3 - $OUT $G <<'PY'
import csv, glob, json, os, sys
from collections import defaultdict
root, G = sys.argv[1], int(sys.argv[2])
vals = defaultdict(list)
for f in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
    for row in csv.DictReader(open(f)):
        if 'gemm_pp_kernel' in row.get('Kernel_Name', '') and row.get('Grid_Size') == str(1536 * 512):
            vals[row['Counter_Name']].append(float(row['Counter_Value']))
c = {}
for k, v in vals.items():
    v = sorted(v)[len(v) // 4:] or v  # drop the autotune's first launches
    c[k] = sum(v) / len(v)
fetch = 2 * c['FETCH_SIZE'] * 1024  # KB units; x2 gfx950 correction
write = c['WRITE_SIZE'] * 1024
out = {'group_m': G, 'M': 32768, 'N': 3072, 'K': 768, 'bytes_per_launch': fetch + write,
       'fetch_bytes_corrected': fetch, 'write_bytes': write,
       'algorithmic_bytes': 2 * (32768 * 768 + 3072 * 768 + 32768 * 3072),
       'algorithmic_read_bytes': 2 * (32768 * 768 + 3072 * 768),
       'mfma_busy_frac': c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(c.get('GRBM_GUI_ACTIVE', 1) / 8 * 1024, 1),
       'samples': {k: len(v) for k, v in vals.items()},
       'source': 'rocprofv3 --pmc, separate FETCH_SIZE / WRITE_SIZE / SQ passes (tools/pmc_ffn1_f16.sh) over the '
                 'f16 text encoder at B=256; FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950)'}
json.dump(out, open(f'gpurun_out/ffn1_traffic_gm{G}.json', 'w'), indent=1)
print(json.dumps(out))
PY
done
