# round 6: BN backward reduce AND apply templated on the ReLU mode (p13 was apply only) — BN
# tests, then C4 / C3 paired
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; [ $rc -le 1 ] || exit $rc; }
MMDX_LIB_PATH=$R/abtmp/bnmode2/libmmdx_hip.so run p14_t 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_trunk_launches_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for i in 1 2; do
  run p14_c4_def_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/bnmode2/libmmdx_hip.so run p14_c4_bm2_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run p14_c3_def_$i 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/bnmode2/libmmdx_hip.so run p14_c3_bm2_$i 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
done
