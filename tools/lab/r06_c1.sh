# round 6: weight-gradient stream confined to n CUs (MMDX_WGRAD_CUS, CU-masked HIP stream),
# C4 paired benches; the per-launch trunk test with a masked stream
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-150; [ $rc -le 1 ] || exit $rc; }
run c1_lstm 300 python -u -m pytest tests/test_text_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "lstm"
MMDX_WGRAD_CUS=128 run c1_trunk 400 python -u -m pytest tests/test_trunk_launches_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "resnet50-128"
for i in 1 2; do
  for n in 0 224 192 160 128; do
    MMDX_WGRAD_CUS=$n run c1_b${n}_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  done
done
