cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for e in text image pipeline; do
  timeout -k 10 300 python -u tools/ab_option.py --enc $e --opt gemm_x3_order --values 0 1 --precision fp32x3 --rounds 5 > gpurun_out/ab_x3order_$e.txt 2>&1 || { tail -20 gpurun_out/ab_x3order_$e.txt; exit 1; }
  tail -4 gpurun_out/ab_x3order_$e.txt
done
