mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_fp32.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_fp32.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline --no-configs > gpurun_out/bench_fp32.log 2>&1
rc=$?; tail -c 1500 gpurun_out/bench_fp32.log; exit $rc
