# fused weight + bias gradients: tests, then C5 paired over MMDX_WGRAD_BIAS_FUSED
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad_bias or bias_grad or gemm" tests/test_stack_plans_gpu.py \
  tests/test_vit_gpu.py tests/test_text_gpu.py tests/test_dp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_wgb.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_wgb.log; exit 1; }
tail -1 gpurun_out/t_wgb.log
for rep in 1 2; do
  for f in 1 0; do
    MMDX_WGRAD_BIAS_FUSED=$f timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/wgb_${f}_$rep.log 2>&1 || exit 2
    echo wgb_${f}_$rep $(grep -o '"value": [0-9.]*' gpurun_out/wgb_${f}_$rep.log)
  done
done
