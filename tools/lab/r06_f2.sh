# round 6: fused BN finalize + apply in isolation (tools/lab/bn_fuse_bench.py): v1 (apply-side
# arrival atomics, build in abtmp/v1) vs v2 (epoch flags); v2 bit-equality tests; paired C4
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -12 $R/gpurun_out/$label.log | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
MMDX_LIB_PATH=$R/abtmp/v1/libmmdx_hip.so run f2_iso_v1 300 python -u tools/lab/bn_fuse_bench.py
run f2_iso_v2 300 python -u tools/lab/bn_fuse_bench.py
run f2_eq 400 python -u -m pytest tests/test_bn_fuse_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for i in 1 2; do
  for m in 0 3; do
    MMDX_BN_FUSE=$m run f2_b${m}_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  done
done
