# C5 launch-heuristic re-sweep on the final kernels (paired, two reps): 256x256 forward tile
# threshold and split-K target
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in base f140 f0 s192 s384; do
    unset MMDX_GEMM256_FWD_MIN MMDX_SPLITK_TARGET
    case $arm in f140) export MMDX_GEMM256_FWD_MIN=140;; f0) export MMDX_GEMM256_FWD_MIN=0;; s192) export MMDX_SPLITK_TARGET=192;; s384) export MMDX_SPLITK_TARGET=384;; esac
    timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/k2_c5_$arm$rep.log 2>&1 || exit 2
    echo c5_$arm$rep $(grep -o '"value": [0-9.]*' gpurun_out/k2_c5_$arm$rep.log)
  done
done
