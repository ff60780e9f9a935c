# round 6: phase-dgrad kernels without scratch (kernel arguments never written; per-phase
# geometry read from the kernarg segment) — conv tile tests, conv kernel tests, per-launch trunk
# test, isolated dgrad table and paired C4 against the previous build (abtmp/prephase)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; grep -E "passed|failed|TOTAL dgrad" $R/gpurun_out/$label.log | tail -1; [ $rc -le 1 ] || exit $rc; }
run p8_t 600 python -u -m pytest tests/test_conv8_gpu.py tests/test_kernels_gpu.py tests/test_trunk_launches_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "conv or resnet"
run p8_cb_new 300 python -u tools/conv_bench.py --ops dgrad
MMDX_LIB_PATH=$R/abtmp/prephase/libmmdx_hip.so run p8_cb_old 300 python -u tools/conv_bench.py --ops dgrad
for i in 1 2; do
  MMDX_LIB_PATH=$R/abtmp/prephase/libmmdx_hip.so run p8_old_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run p8_new_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
