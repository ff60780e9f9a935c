# split-K target sweep: C5 over 128 / 192 / 256, C4 over 512 / 256 (paired, 2 reps)
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for t in 256 128 192; do
    MMDX_SPLITK_TARGET=$t timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sk2_${t}_$rep.log 2>&1 || exit 2
    echo c5_sk_${t}_$rep $(grep -o '"value": [0-9.]*' gpurun_out/sk2_${t}_$rep.log)
  done
  for t in 512 256; do
    MMDX_SPLITK_TARGET=$t timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/sk2c4_${t}_$rep.log 2>&1 || exit 2
    echo c4_sk_${t}_$rep $(grep -o '"value": [0-9.]*' gpurun_out/sk2c4_${t}_$rep.log)
  done
done
