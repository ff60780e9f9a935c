# 256x256 forward tile threshold (MMDX_GEMM256_FWD_MIN) on the final kernels: C5 arms that add
# the BERT-base N = 768 (96 tiles), ViT-B N = 768 (150), BERT QKV (288) / FFN-up (384) shapes;
# then C4 at 140 vs 400
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in 90 60 30 1; do
    MMDX_GEMM256_FWD_MIN=$arm timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/k4_c5_$arm.$rep.log 2>&1 || exit 2
    echo c5_$arm.$rep $(grep -o '"value": [0-9.]*' gpurun_out/k4_c5_$arm.$rep.log)
  done
done
for rep in 1 2; do
  for arm in 400 90 30; do
    MMDX_GEMM256_FWD_MIN=$arm timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/k4_c4_$arm.$rep.log 2>&1 || exit 2
    echo c4_$arm.$rep $(grep -o '"value": [0-9.]*' gpurun_out/k4_c4_$arm.$rep.log)
  done
done
