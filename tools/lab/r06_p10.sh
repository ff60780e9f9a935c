# round 6: nontemporal loads of the conv epilogue's accumulation sources (accmask identity
# gradient, beta*C of the accumulating dgrads, phase dgrad beta*C) — ntacc vs the default
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; [ $rc -le 1 ] || exit $rc; }
for i in 1 2 3; do
  run p10_def_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntacc/libmmdx_hip.so run p10_ntacc_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
