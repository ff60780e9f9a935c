# r05 session 19: narrow-N conv tiles, variants 4 (512x64, 8 waves) / 5 (256x64, 8 waves)
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run s19_par4 600 env MMDX_CONV_N64_WIDE=4 python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_trunk_launches_gpu.py -m gpu
run s19_par5 600 env MMDX_CONV_N64_WIDE=5 python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_trunk_launches_gpu.py -m gpu
run s19_cb4 300 env MMDX_CONV_N64_WIDE=4 python tools/conv_bench.py --filter K64 --ops fwd,dgrad
run s19_cb5 300 env MMDX_CONV_N64_WIDE=5 python tools/conv_bench.py --filter K64 --ops fwd,dgrad
for rep in 1 2; do
  run s19_c4_0_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s19_c4_2_$rep 300 env MMDX_CONV_N64_WIDE=2 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s19_c4_4_$rep 300 env MMDX_CONV_N64_WIDE=4 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s19_c4_5_$rep 300 env MMDX_CONV_N64_WIDE=5 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
run s19_c2_0 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
run s19_c2_2 300 env MMDX_CONV_N64_WIDE=2 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
