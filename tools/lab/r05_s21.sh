# r05 session 21: layer1 3x3 weight gradient with tap-aligned 64-column tiles (MMDX_WGRAD_TAP_BN)
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run s21_par 600 env MMDX_WGRAD_TAP_BN=1 python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_trunk_launches_gpu.py -m gpu
run s21_cb0 300 python tools/conv_bench.py --filter "C64 K64 3x3" --ops wgrad
run s21_cb1 300 env MMDX_WGRAD_TAP_BN=1 python tools/conv_bench.py --filter "C64 K64 3x3" --ops wgrad
for rep in 1 2; do
  run s21_c4_0_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s21_c4_1_$rep 300 env MMDX_WGRAD_TAP_BN=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
