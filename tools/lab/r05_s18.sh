# r05 session 18: 256 x 64 tiles for the narrow-N conv GEMMs (MMDX_CONV_N64_WIDE = 2 / 3):
# per-launch parity, isolated shapes, paired C4
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run s18_par2 600 env MMDX_CONV_N64_WIDE=2 python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_trunk_launches_gpu.py tests/test_kernels_gpu.py -m gpu -k "conv or trunk or launch"
run s18_par3 600 env MMDX_CONV_N64_WIDE=3 python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_trunk_launches_gpu.py -m gpu
run s18_cb0 300 python tools/conv_bench.py --filter K64 --ops fwd,dgrad
run s18_cb2 300 env MMDX_CONV_N64_WIDE=2 python tools/conv_bench.py --filter K64 --ops fwd,dgrad
run s18_cb3 300 env MMDX_CONV_N64_WIDE=3 python tools/conv_bench.py --filter K64 --ops fwd,dgrad
for rep in 1 2; do
  run s18_c4_0_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s18_c4_2_$rep 300 env MMDX_CONV_N64_WIDE=2 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s18_c4_3_$rep 300 env MMDX_CONV_N64_WIDE=3 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
