#!/bin/bash
# Per-encoder kernel trace + PMC passes (HBM bytes, MFMA busy) -> tools/pmc_report.py tables in
# gpurun_out/pmcrep_<enc>.txt. One counter group per rocprofv3 run (no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for e in ${ENCS:-text image image_mbv2 speech fusion}; do
  O=gpurun_out/pmcenc_${PREC:-f16}_$e; rm -rf $O; mkdir -p $O
  CMD="python3 tools/encoder_profile.py --enc $e --iters 3 --batch ${BATCH:-256} --precision ${PREC:-f16}"
  timeout -k 10 180 rocprofv3 --kernel-trace -d $O/trace -o run -- $CMD > $O/trace.log 2>&1 || { echo "trace $e rc=$?"; exit 1; }
  i=0
  for SET in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $SET -d $O/p$i -o p -f csv -- $CMD > $O/p$i.log 2>&1 || { echo "pmc $e pass $i rc=$?"; tail -3 $O/p$i.log; exit 1; }
  done
  python3 tools/pmc_report.py $(ls $O/trace/*/run_results.db $O/trace/run_results.db 2>/dev/null | head -1) $O > gpurun_out/pmcrep_${PREC:-f16}_$e.txt
  echo "== $e"; head -24 gpurun_out/pmcrep_${PREC:-f16}_$e.txt
done
