#!/bin/bash
# One SQ counter pass (wave-cycle stall split, LDS bank conflicts) over one encoder:
#   ENC=image_mbv2 PREC=fp32x3 bash tools/pmc_sq.sh  -> gpurun_out/pmcsq_<prec>_<enc>.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmcsq${TAG:+_$TAG}_${PREC:-f16}_${ENC:-image_mbv2}; rm -rf $O; mkdir -p $O
CMD="python3 tools/encoder_profile.py --enc ${ENC:-image_mbv2} --iters 3 --batch ${BATCH:-256} --precision ${PREC:-f16} ${EXTRA}"
# EXTRA: more encoder_profile.py arguments (e.g. --opt pw_seam_x3=0); COUNTERS overrides the pass (at most 8 SQ_ and 2 GRBM_ counters per pass)
C=${COUNTERS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS}
timeout -s KILL 180 rocprofv3 --pmc $C -d $O/p -o p -f csv -- $CMD > $O/p.log 2>&1 || { echo "pmc rc=$?"; tail -3 $O/p.log; exit 1; }
python3 tools/pmc_sq.py $O > $O.txt
cut -c1-72,74-76,200-300 $O.txt | head -30
