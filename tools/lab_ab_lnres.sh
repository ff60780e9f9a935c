# C5 / C4 A/B, paired on one box: library at the residual-GEMM commit (2a52c86) against the
# current one (LayerNorm backward residual + bias partials in the split-K reduce)
set -u
mkdir -p gpurun_out
A=$GRAFT_REPO_ROOT/abtmp/libmmdx_2a.so
for rep in 1 2 3; do
  for arm in A B; do
    if [ $arm = A ]; then export MMDX_LIB_PATH=$A; else unset MMDX_LIB_PATH; fi
    timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ablr_c5_${arm}$rep.log 2>&1 || exit 2
    echo c5_$arm$rep $(grep -o '"value": [0-9.]*' gpurun_out/ablr_c5_${arm}$rep.log)
  done
done
for arm in A B; do
  if [ $arm = A ]; then export MMDX_LIB_PATH=$A; else unset MMDX_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ablr_c4_$arm.log 2>&1 || exit 2
  echo c4_$arm $(grep -o '"value": [0-9.]*' gpurun_out/ablr_c4_$arm.log)
done
