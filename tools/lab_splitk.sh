# bias-gradient grid + split-K target: kernel / stack tests, then C5 paired over MMDX_SPLITK_TARGET
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_stack_plans_gpu.py tests/test_vit_gpu.py \
  tests/test_text_gpu.py tests/test_gemm8_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sk.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_sk.log; exit 1; }
tail -1 gpurun_out/t_sk.log
for rep in 1 2; do
  for t in 512 256 1024; do
    MMDX_SPLITK_TARGET=$t timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sk_${t}_$rep.log 2>&1 || exit 2
    echo sk_${t}_$rep $(grep -o '"value": [0-9.]*' gpurun_out/sk_${t}_$rep.log)
  done
done
