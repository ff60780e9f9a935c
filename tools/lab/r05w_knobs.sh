# C4 env-knob check on the wgrad-target-256 tree: weight-gradient tile variants and targets
set -o pipefail
for r in 1 2; do for arm in base w8w t192 t320; do
  unset MMDX_WGRAD_8W MMDX_WGRAD_TARGET
  case $arm in w8w) export MMDX_WGRAD_8W=1;; t192) export MMDX_WGRAD_TARGET=192;; t320) export MMDX_WGRAD_TARGET=320;; esac
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/wk_${arm}_$r.log 2>&1 || exit 3
  echo "$arm $r $(grep -o '"value": [0-9.]*' gpurun_out/wk_${arm}_$r.log | head -1)"
done; done
