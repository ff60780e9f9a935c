# round 6: 32x32x16 MFMA tiles for the 8-wave 128 x 128 conv fwd / dgrad (MMDX_CONV_MF32):
# tile tests, per-launch fp64 trunk test under MF32, isolated per-shape tables, paired C4
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -3 $R/gpurun_out/$label.log | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
run mf_t8 400 python -u -m pytest tests/test_conv8_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider
MMDX_CONV_MF32=1 run mf_trunk 600 python -u -m pytest tests/test_trunk_launches_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "resnet50-128 or resnet18"
for m in 0 1; do
  MMDX_CONV_MF32=$m run mf_cb$m 300 python -u tools/conv_bench.py --ops fwd,dgrad
done
for i in 1 2; do
  for m in 0 1; do
    MMDX_CONV_MF32=$m run mf_b${m}_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  done
done
