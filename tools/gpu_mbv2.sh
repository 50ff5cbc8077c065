cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mb_tests.log 2>&1
rc=$?; tail -15 gpurun_out/mb_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 120 python tools/encoder_profile.py --enc image_mbv2 --iters 10 && \
timeout -k 10 120 python tools/encoder_profile.py --enc image --iters 10 && \
rm -rf gpurun_out/prof_mb && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mb -o run -- python3 tools/encoder_profile.py --enc image_mbv2 --iters 5 > gpurun_out/prof_mb.log 2>&1 && \
python3 tools/prof_summary.py gpurun_out/prof_mb/run_results.db --window spin --steps 5 --by-grid 2>&1 | head -40
