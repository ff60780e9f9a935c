# LayerNorm backward with the residual-gradient load hoisted: LN tests, then C5 paired against
# the residual-GEMM commit's library (2a52c86, separate add passes)
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ln_dropout_gpu.py tests/test_stack_plans_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_lnres2.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_lnres2.log; exit 1; }
tail -1 gpurun_out/t_lnres2.log
for rep in 1 2 3; do
  for arm in A B; do
    if [ $arm = A ]; then export MMDX_LIB_PATH=$R/abtmp/libmmdx_2a.so; else unset MMDX_LIB_PATH; fi
    timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lnres2_c5_${arm}$rep.log 2>&1 || exit 2
    echo c5_$arm$rep $(grep -o '"value": [0-9.]*' gpurun_out/lnres2_c5_${arm}$rep.log)
  done
done
