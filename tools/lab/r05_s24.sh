# r05 session 24: 8-wave tiles for the other 4-wave tile families (A/B knobs): conv 128x64
# (MMDX_CONV_8W64), 1x1 weight gradients 128x128 (MMDX_WGRAD_8W), dense GEMMs 128x128
# (MMDX_GEMM_8W128); parity of the new default (8-wave 128x128 conv tiles) and the knobs
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run s24_par 600 env MMDX_CONV_8W64=1 MMDX_WGRAD_8W=1 MMDX_GEMM_8W128=1 python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_trunk_launches_gpu.py tests/test_kernels_gpu.py tests/test_gemm8_gpu.py -m gpu
run s24_cb_w0 300 python tools/conv_bench.py --ops wgrad
run s24_cb_w1 300 env MMDX_WGRAD_8W=1 python tools/conv_bench.py --ops wgrad
run s24_cb_64 300 env MMDX_CONV_8W64=1 python tools/conv_bench.py --ops fwd,dgrad
run s24_gb0 300 python tools/gemm_bench.py
run s24_gb1 300 env MMDX_GEMM_8W128=1 python tools/gemm_bench.py
for rep in 1 2; do
  run s24_c4_0_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s24_c4_w_$rep 300 env MMDX_WGRAD_8W=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s24_c4_64_$rep 300 env MMDX_CONV_8W64=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s24_c5_0_$rep 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run s24_c5_g_$rep 300 env MMDX_GEMM_8W128=1 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
