#!/bin/bash
# SQ-counter passes for the kernels of one encoder run whose name matches MATCH; one counter
# group per rocprofv3 run (no tracing domains). Prints per-kernel average counter values.
#   MATCH=conv3x3 ENC=image bash tools/pmc_kernel.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmck; rm -rf $O; mkdir -p $O
CMD="python3 tools/encoder_profile.py --enc ${ENC:-image} --iters 3 ${EXTRA}"
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $SET -d $O/p$i -o p -f csv -- $CMD > $O/p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -3 $O/p$i.log; exit 1; }
done
python3 - "$O" "${MATCH:-conv3x3}" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], '**', '*counter_collection.csv'), recursive=True):
    for row in csv.DictReader(open(f)):
        if sys.argv[2] in row['Kernel_Name']:
            acc[(row['Kernel_Name'][:60], row['Grid_Size'])][row['Counter_Name']].append(float(row['Counter_Value']))
for k, c in acc.items():
    print(k)
    for n, v in sorted(c.items()):
        print(f'   {n:28s} {sum(v) / len(v):14.4g}  (n={len(v)})')
PY
