# round 6, call 3: persistent conv kernel (MMDX_CONV_PERSIST bit mask: 1 pointwise, 2 tap
# gathers, 4 the 256 x 64 tiles) — bit-identity tests, isolated per-shape tables, paired C4
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run s3_t8 400 python -u -m pytest tests/test_conv8_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for m in 0 1 7; do
  MMDX_CONV_PERSIST=$m run s3_cb$m 300 python -u tools/conv_bench.py --ops fwd,dgrad
done
for i in 1 2; do
  for m in 0 1 7; do
    MMDX_CONV_PERSIST=$m run s3_b${m}_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  done
done
