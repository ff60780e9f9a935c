# paired A/B of the conv wgrad split target 512 vs 256 at C4 (x3), C3 and C2 (x2)
set -o pipefail
for cfg in c4 c4 c4 c3 c3 c2 c2; do for t in 512 256; do
  MMDX_WGRAD_TARGET=$t timeout -k 10 300 python -u bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/wta_${cfg}_$t.log 2>&1 || exit 3
  echo "$cfg target=$t $(grep -o '"value": [0-9.]*' gpurun_out/wta_${cfg}_$t.log | head -1)"
done; done
