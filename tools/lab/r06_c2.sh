# round 6: weight-gradient stream CU mask, narrower settings (MMDX_WGRAD_CUS), C4 paired
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; [ $rc -le 1 ] || exit $rc; }
for i in 1 2; do
  for n in 0 128 96 64 32; do
    MMDX_WGRAD_CUS=$n run c2_b${n}_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  done
done
