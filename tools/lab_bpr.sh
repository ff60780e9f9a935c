# bias partials reduced by the split-K reduce launch: tests, then C5 twice
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad_bias or gemm_residual or bias_grad" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_bpr1.log 2>&1 || { echo "tests1 rc=$?"; tail -30 gpurun_out/t_bpr1.log; exit 1; }
tail -1 gpurun_out/t_bpr1.log
timeout -k 10 600 python -u -m pytest tests/test_stack_plans_gpu.py tests/test_benched_path_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_bpr2.log 2>&1 || { echo "tests2 rc=$?"; tail -30 gpurun_out/t_bpr2.log; exit 1; }
tail -1 gpurun_out/t_bpr2.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bpr_c5_$rep.log 2>&1 || exit 2
  echo c5_$rep $(grep -o '"value": [0-9.]*' gpurun_out/bpr_c5_$rep.log)
done
