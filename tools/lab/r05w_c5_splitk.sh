# C5 dense split-K target re-check on the round-5 GEMM tiles (MMDX_SPLITK_TARGET)
set -o pipefail
for r in 1 2; do for t in 256 192 384 512; do
  MMDX_SPLITK_TARGET=$t timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5s_${t}_$r.log 2>&1 || exit 3
  echo "target=$t $r $(grep -o '"value": [0-9.]*' gpurun_out/c5s_${t}_$r.log | head -1)"
done; done
