# r05 session 17: C5 tile-size knobs re-swept on the split-major / grouped-order kernels
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-120; [ $rc -le 1 ] || exit $rc; }
for rep in 1 2; do
  run s17_def_$rep 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run s17_all256_300_$rep 300 env MMDX_GEMM256_MIN=300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run s17_all256_150_$rep 300 env MMDX_GEMM256_MIN=150 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run s17_ns3_$rep 300 env MMDX_GEMM256_NS=3 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run s17_g8_$rep 300 env MMDX_GEMM8_MIN=200 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
