timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fp32.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_fp32.log; [ $rc -eq 0 ] || exit $rc
PREC=fp32 ENCS="text image" bash tools/gpu_enc_prof.sh
