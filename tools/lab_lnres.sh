# residual LN backward (ViT): tests, then C5 twice
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_ln_dropout_gpu.py tests/test_stack_plans_gpu.py tests/test_vit_gpu.py tests/test_benched_path_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_lnres.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_lnres.log; exit 1; }
tail -1 gpurun_out/t_lnres.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lnres_c5_$rep.log 2>&1 || exit 2
  echo c5_$rep $(grep -o '"value": [0-9.]*' gpurun_out/lnres_c5_$rep.log)
done
