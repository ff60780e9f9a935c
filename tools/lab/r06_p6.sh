# round 6: default with nontemporal BN-pass loads (x / residual / dy) — BN kernel tests and the
# per-launch trunk test, then C4 paired against ntld2 (+ NT loads in the BN backward reduce and
# the masked-dy source)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; grep -E "passed|failed" $R/gpurun_out/$label.log | tail -1; [ $rc -le 1 ] || exit $rc; }
run p6_t 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_trunk_launches_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "batchnorm or bn_ or maxpool_bn or dgrad_fused_bn or resnet50-128 or resnet18"
for i in 1 2; do
  run p6_def_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntld2/libmmdx_hip.so run p6_ntld2_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
