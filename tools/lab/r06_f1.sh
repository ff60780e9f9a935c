# round 6, fused BN finalize + apply (MMDX_BN_FUSE): bit-equality tests, the BN kernel tests
# and the per-launch trunk test with fusion on, paired C4 benches (0 = two launches, 3 = fused)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -3 $R/gpurun_out/$label.log | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
run f1_eq 400 python -u -m pytest tests/test_bn_fuse_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
MMDX_BN_FUSE=3 run f1_kern 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "batchnorm or bn_ or maxpool_bn or dgrad_fused_bn"
MMDX_BN_FUSE=3 run f1_trunk 600 python -u -m pytest tests/test_trunk_launches_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "resnet50-128"
for i in 1 2; do
  for m in 0 3; do
    MMDX_BN_FUSE=$m run f1_b${m}_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  done
done
for m in 1 2; do  # (per-direction)
  MMDX_BN_FUSE=$m run f1_b${m}_1 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
