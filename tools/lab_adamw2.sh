# AdamW defaults (unrolled kernel, 16K chunks): optimizer / AMP / benched-path tests
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_amp_gpu.py tests/test_benched_path_gpu.py tests/test_dp_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_adamw2.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_adamw2.log; exit 1; }
tail -1 gpurun_out/t_adamw2.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "adamw or clip" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_adamw3.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_adamw3.log; exit 1; }
tail -1 gpurun_out/t_adamw3.log
