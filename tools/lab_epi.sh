# GEMM epilogue change: GEMM / stack / AMP tests, then C5 A/B (HEAD epilogue vs new), paired
set -u
mkdir -p gpurun_out
L=/root/repo/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib/libmmdx_hip.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" tests/test_gemm8_gpu.py \
  tests/test_stack_plans_gpu.py tests/test_vit_gpu.py tests/test_amp_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/t_epi.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_epi.log; exit 1; }
tail -2 gpurun_out/t_epi.log
for rep in 1 2; do
  for arm in /root/repo/abtmp/libmmdx_head.so $L; do
    n=$(basename $arm .so)_$rep
    MMDX_LIB_PATH=$arm timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/epi_$n.log 2>&1 || exit 2
    echo $n $(grep -o '"value": [0-9.]*' gpurun_out/epi_$n.log)
  done
done
