#!/bin/bash
# PMC passes (counters only, no tracing domains) on one GEMM shape via tools/bench_gemm.py.
# usage: bash tools/pmc.sh SHAPE BN [regex]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SHAPE=${1:-bert_ffn1}; BN=${2:-0}; RX=${3:-gemm_glds}
OUT=gpurun_out/pmc_${SHAPE}
rm -rf $OUT; mkdir -p $OUT
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "$RX" -d $OUT/p$i -o p -f csv -- python3 tools/bench_gemm.py --only $SHAPE --impl 2 --bn $BN --iters 5 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT
