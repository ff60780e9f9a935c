# round 6: more nontemporal variants on top of the default (NT conv / GEMM epilogue stores):
# ntpp = + phase-dgrad epilogue and weight-gradient split-K slabs NT stores;
# ntld = + nontemporal loads of x / residual / dy in the BN apply and backward-apply passes;
# ntstem = + the direct stem conv's output stores NT
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; [ $rc -le 1 ] || exit $rc; }
for i in 1 2; do
  run p5_def_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntpp/libmmdx_hip.so run p5_ntpp_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntld/libmmdx_hip.so run p5_ntld_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntstem/libmmdx_hip.so run p5_ntstem_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
