# round 6: the downsample BN backward on the weight-gradient stream (MMDX_DS_BWD_SIDE): bitwise
# test, per-launch trunk test under it, paired C4
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; grep -E "passed|failed" $R/gpurun_out/$label.log | tail -1; [ $rc -le 1 ] || exit $rc; }
run d1_t 400 python -u -m pytest tests/test_trunk_streams_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
MMDX_DS_BWD_SIDE=1 run d1_trunk 600 python -u -m pytest tests/test_trunk_launches_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "resnet50-128"
for i in 1 2 3; do
  run d1_b0_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_DS_BWD_SIDE=1 run d1_b1_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
