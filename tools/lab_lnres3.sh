# ViT LN backward residual as a knob (MMDX_VIT_LN_ADDIN, default 0 = separate add): tests under
# both settings, then C5 paired: A = residual-GEMM commit's library, B = default, C = knob on
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ln_dropout_gpu.py tests/test_stack_plans_gpu.py tests/test_vit_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_lnres3a.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_lnres3a.log; exit 1; }
tail -1 gpurun_out/t_lnres3a.log
MMDX_VIT_LN_ADDIN=1 timeout -k 10 400 python -u -m pytest tests/test_stack_plans_gpu.py tests/test_vit_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_lnres3b.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_lnres3b.log; exit 1; }
tail -1 gpurun_out/t_lnres3b.log
for rep in 1 2 3; do
  for arm in A B C; do
    unset MMDX_LIB_PATH MMDX_VIT_LN_ADDIN
    case $arm in A) export MMDX_LIB_PATH=$R/abtmp/libmmdx_2a.so;; C) export MMDX_VIT_LN_ADDIN=1;; esac
    timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lnres3_c5_${arm}$rep.log 2>&1 || exit 2
    echo c5_$arm$rep $(grep -o '"value": [0-9.]*' gpurun_out/lnres3_c5_${arm}$rep.log)
  done
done
