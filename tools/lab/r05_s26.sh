# r05 session 26: parity suites for the 8-wave defaults; C2 paired 8-wave on / off (three pairs)
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run s26_par 900 python -u -m pytest -q --timeout 500 --timeout-method thread tests/test_conv8_gpu.py tests/test_gemm8_gpu.py tests/test_trunk_launches_gpu.py tests/test_kernels_gpu.py tests/test_benched_path_gpu.py -m gpu
for rep in 1 2 3; do
  run s26_c2_0_$rep 300 env MMDX_CONV_8W128=0 MMDX_GEMM_8W128=0 python bench.py --config c2 --steps 60 --warmup 10 --no-cpu-baseline
  run s26_c2_1_$rep 300 python bench.py --config c2 --steps 60 --warmup 10 --no-cpu-baseline
  run s26_c2_g_$rep 300 env MMDX_GEMM_8W128=0 python bench.py --config c2 --steps 60 --warmup 10 --no-cpu-baseline
done
