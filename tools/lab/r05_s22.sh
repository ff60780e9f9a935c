# r05 session 22: 128x128 conv tiles in 8 waves of 64x32 (MMDX_CONV_8W128) vs the 4-wave default
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run s22_par 600 env MMDX_CONV_8W128=1 python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_trunk_launches_gpu.py -m gpu
run s22_cb0 300 python tools/conv_bench.py --ops fwd,dgrad
run s22_cb1 300 env MMDX_CONV_8W128=1 python tools/conv_bench.py --ops fwd,dgrad
for rep in 1 2; do
  run s22_c4_0_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s22_c4_1_$rep 300 env MMDX_CONV_8W128=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
