# r05 session 20: 8-wave 256x64 narrow-N conv tiles by default (M >= 262144): parity, paired
# C4 / C3 / C2 against MMDX_CONV_N64_WIDE=0
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run s20_par 900 python -u -m pytest -q -x --timeout 800 --timeout-method thread tests/test_trunk_launches_gpu.py tests/test_kernels_gpu.py tests/test_conv8_gpu.py tests/test_bn_fin_gpu.py -m gpu
run s20_bench 900 python -u -m pytest -q -x --timeout 800 --timeout-method thread tests/test_benched_path_gpu.py -m gpu -k "c4 or c3 or c2"
for rep in 1 2; do
  run s20_c4_new_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s20_c4_old_$rep 300 env MMDX_CONV_N64_WIDE=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
run s20_c3_new 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run s20_c3_old 300 env MMDX_CONV_N64_WIDE=0 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run s20_c2_new 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
run s20_c2_old 300 env MMDX_CONV_N64_WIDE=0 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
