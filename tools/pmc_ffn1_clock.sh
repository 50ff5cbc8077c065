#!/bin/bash
# Is the fp32x3 FFN1 tile bound by its operand loads or by the MFMA clock? Same binary (the probe build),
# the FFN1 split tile with (gemm_debug 0) and without (gemm_debug 1) its K-loop operand loads: per launch
# duration (kernel trace), MFMA-busy SIMD cycles and GRBM_GUI_ACTIVE (one --pmc pass each), so the
# effective clock GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS give-back) and the MFMA
# busy fraction of both. -> gpurun_out/ffn1_x3_clock.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ffn1_clock
rm -rf $OUT; mkdir -p $OUT
L=multimodal-emotion-classification_amd/mec/libmec_hip_probes.so
for v in 0 1; do
  MEC_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
    --kernel-include-regex "gemm_glds_kernel" -d $OUT/c$v -o c -f csv -- \
    python3 tools/encoder_profile.py --enc text --precision fp32x3 --iters 3 --opt gemm_bn=70256 --opt gemm_debug=$v \
    > $OUT/c$v.log 2>&1
  rc=$?; echo "gemm_debug=$v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/c$v.log; exit $rc; fi
done
python3 - <<'PY'
import csv, glob, json, os
from collections import defaultdict
root = 'gpurun_out/pmc_ffn1_clock'
res = {}
for v in (0, 1):
    cnt = defaultdict(dict)
    for f in glob.glob(os.path.join(root, 'c%d' % v, '**', '*counter_collection.csv'), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get('Grid_Size') != '786432':  # FFN1: 1536 blocks x 512 threads
                continue
            cnt[row['Dispatch_Id']][row['Counter_Name']] = float(row['Counter_Value'])
    dur = {}
    for f in glob.glob(os.path.join(root, 'c%d' % v, '**', '*kernel_trace.csv'), recursive=True):
        for row in csv.DictReader(open(f)):
            dur[row['Dispatch_Id']] = (int(row['End_Timestamp']) - int(row['Start_Timestamp'])) * 1e-9
    ids = sorted((d for d in cnt if d in dur), key=int)
    ids = ids[len(ids) // 4:] or ids  # drop the first launches (autotune / warm-up)
    n = len(ids)
    d = sum(dur[i] for i in ids) / n
    g = sum(cnt[i]['GRBM_GUI_ACTIVE'] for i in ids) / n
    mb = sum(cnt[i]['SQ_VALU_MFMA_BUSY_CYCLES'] for i in ids) / n
    res['gemm_debug_%d' % v] = {
        'launches': n, 'avg_ms': d * 1e3, 'effective_clock_ghz': g / 8 / d * 1e-9,
        'mfma_busy_frac': mb / (g / 8 * 1024), 'mfma_busy_simd_cycles': mb}
a, b = res['gemm_debug_0'], res['gemm_debug_1']
res['note'] = ('gemm_debug 1 = the same tile with no operand loads in its K loop (probe build, wrong results); '
               'clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)')
res['duration_ratio'] = a['avg_ms'] / b['avg_ms']
res['clock_ratio'] = b['effective_clock_ghz'] / a['effective_clock_ghz']
json.dump(res, open('gpurun_out/ffn1_x3_clock.json', 'w'), indent=1)
print(json.dumps(res, indent=1))
PY
