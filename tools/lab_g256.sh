# 256x256 forward tiles from 90 tiles up (default): GEMM kernel tests, stack plans, the benched
# C5 / C4 steps against the oracle, then C5 / C4 bench lines
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm8_gpu.py tests/test_stack_plans_gpu.py tests/test_vit_gpu.py tests/test_text_gpu.py tests/test_benched_path_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_g256.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_g256.log; exit 1; }
tail -1 gpurun_out/t_g256.log
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g256_c5.log 2>&1 || exit 2
echo c5 $(grep -o '"value": [0-9.]*' gpurun_out/g256_c5.log)
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/g256_c4.log 2>&1 || exit 2
echo c4 $(grep -o '"value": [0-9.]*' gpurun_out/g256_c4.log)
