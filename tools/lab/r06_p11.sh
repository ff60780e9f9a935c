# round 6: nontemporal slab loads in the split-K reduces (conv wgrad_reduce / _z, dense
# splitk_reduce4) — ntred vs the default, C4 and C5 paired
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; [ $rc -le 1 ] || exit $rc; }
for i in 1 2; do
  run p11_c4_def_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntred/libmmdx_hip.so run p11_c4_red_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run p11_c5_def_$i 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntred/libmmdx_hip.so run p11_c5_red_$i 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
