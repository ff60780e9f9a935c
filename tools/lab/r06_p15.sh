# round 6: MODE-3 (recompute-from-x) BN backward apply — the 32 non-residual units of C4 —
# reads the forward's scale as its bit-equal a = gamma*rstd (abtmp/shsc: 84 -> 76 VGPRs,
# 5 -> 6 waves) and additionally a 7-waves target for the dense-gradient instances
# (abtmp/shw7: 72 VGPRs, no scratch); BN tests on both, C4 paired x2, C3 x1
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; [ $rc -le 1 ] || exit $rc; }
for v in shsc shw7; do
  MMDX_LIB_PATH=$R/abtmp/$v/libmmdx_hip.so run p15_t_$v 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_trunk_launches_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
done
for i in 1 2; do
  run p15_c4_def_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  for v in shsc shw7; do
    MMDX_LIB_PATH=$R/abtmp/$v/libmmdx_hip.so run p15_c4_${v}_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  done
done
run p15_c3_def_1 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
for v in shsc shw7; do
  MMDX_LIB_PATH=$R/abtmp/$v/libmmdx_hip.so run p15_c3_${v}_1 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
done
