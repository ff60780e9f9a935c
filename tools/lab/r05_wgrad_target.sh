# conv weight-gradient split-K target re-sweep on the round-5 kernels (MMDX_WGRAD_TARGET), C4
set -o pipefail
for r in 1 2; do for t in 512 256 384 768 1024; do
  MMDX_WGRAD_TARGET=$t timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/wt_${t}_$r.log 2>&1 || exit 3
  echo "target=$t $r $(grep -o '"value": [0-9.]*' gpurun_out/wt_${t}_$r.log | head -1)"
done; done
