# C5 A/B/C paired on one box: residual-GEMM commit (2a52c86), + LayerNorm backward residual
# (6e8ae97), current (+ bias partials in the split-K reduce)
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for arm in A L B; do
    case $arm in A) export MMDX_LIB_PATH=$R/abtmp/libmmdx_2a.so;; L) export MMDX_LIB_PATH=$R/abtmp/libmmdx_6e.so;; B) unset MMDX_LIB_PATH;; esac
    timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab3w_c5_${arm}$rep.log 2>&1 || exit 2
    echo c5_$arm$rep $(grep -o '"value": [0-9.]*' gpurun_out/ab3w_c5_${arm}$rep.log)
  done
done
