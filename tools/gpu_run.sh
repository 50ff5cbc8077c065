#!/bin/bash
# One parametrized GPU runner (replaces the per-step gpu_rNN*.sh launchers). Each argument is one step,
# run in order; the first failing step ends the call (no GPU step runs after a failure or a time limit).
#   tests                  the whole -m gpu suite            -> gpurun_out/$TAG_pytest_gpu.log
#   tests:<pytest -k expr> a subset of it
#   bench[:<extra args>]   the default bench line            -> gpurun_out/$TAG_bench.json (+ .log)
#   smoke                  __graft_entry__.smoke()           -> gpurun_out/$TAG_smoke.log
#   enc:<enc>:<prec>       rocprofv3 stats of one encoder alone at B = 256 (tools/gpu_enc_prof.sh)
#   prof:<prec>            rocprofv3 stats of bench.py's timed window (tools/gpu_prof_bench.sh)
#   ab:<enc>:<prec>:<n>    cross-build A/B, mec/libmec_hip_base.so vs mec/libmec_hip.so (tools/gpu_ab_lib.sh)
#   opt:<enc>:<prec>:<opt>:<v1,v2,..>[:<batch>]  same-build option A/B (tools/ab_option.py)
#   py:<script> [args]     any python script under tools/ (bounded to 300 s)
# Usage: TAG=r06a bash tools/gpu_run.sh tests bench smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06}
for step in "$@"; do
  echo "== $step ($(date +%T))"
  case "$step" in
    tests|tests:*)
      K=""; [ "$step" != tests ] && K="${step#tests:}"
      if [ -n "$K" ]; then
        timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" \
          > gpurun_out/${TAG}_pytest_gpu.log 2>&1
      else
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
          > gpurun_out/${TAG}_pytest_gpu.log 2>&1
      fi
      rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc ;;
    bench|bench:*)
      X=""; [ "$step" != bench ] && X="${step#bench:}"
      timeout -k 10 600 python -u bench.py $X --json-out gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_bench.log 2>&1 \
        || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
      python3 tools/summ_bench.py gpurun_out/${TAG}_bench.json || exit 1 ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" \
        > gpurun_out/${TAG}_smoke.log 2>&1
      rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc ;;
    enc:*)
      IFS=: read -r _ E P <<< "$step"
      ENCS=$E PREC=$P bash tools/gpu_enc_prof.sh || exit 1
      cp gpurun_out/enc_${P}_$E.txt gpurun_out/${TAG}_enc_${P}_$E.txt ;;
    prof:*)
      P="${step#prof:}"
      PREC=$P bash tools/gpu_prof_bench.sh > gpurun_out/${TAG}_prof_$P.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof_$P.log; exit 1; }
      cp gpurun_out/bench_prof_grid_$P.txt gpurun_out/${TAG}_kernel_stats_bench_grid_$P.txt
      cp gpurun_out/bench_prof_$P.txt gpurun_out/${TAG}_kernel_stats_bench_$P.txt
      head -12 gpurun_out/bench_prof_grid_$P.txt ;;
    ab:*)
      IFS=: read -r _ E P N <<< "$step"
      ENC=$E PREC=$P ROUNDS=${N:-3} bash tools/gpu_ab_lib.sh > gpurun_out/${TAG}_ab_${E}_$P.txt 2>&1 \
        || { cat gpurun_out/${TAG}_ab_${E}_$P.txt; exit 1; }
      tail -8 gpurun_out/${TAG}_ab_${E}_$P.txt ;;
    opt:*)
      IFS=: read -r _ E P O V NB <<< "$step"
      timeout -k 10 400 python3 -u tools/ab_option.py --enc $E --precision $P --opt $O --values ${V//,/ } --rounds 5 --batch ${NB:-256} \
        > gpurun_out/${TAG}_opt_${O}_${E}_$P.txt 2>&1 || { tail -5 gpurun_out/${TAG}_opt_${O}_${E}_$P.txt; exit 1; }
      tail -12 gpurun_out/${TAG}_opt_${O}_${E}_$P.txt ;;
    py:*)
      timeout -k 10 300 python3 -u tools/${step#py:} || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
