# round 6: the nontemporal stores / loads on the other configs — C2, C3, C5 paired against a
# build without them (abtmp/nont; same code otherwise)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; [ $rc -le 1 ] || exit $rc; }
for i in 1 2 3; do
  MMDX_LIB_PATH=$R/abtmp/nont/libmmdx_hip.so run p9_c2_nont_$i 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
  run p9_c2_nt_$i 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
done
for i in 1 2; do
  MMDX_LIB_PATH=$R/abtmp/nont/libmmdx_hip.so run p9_c3_nont_$i 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
  run p9_c3_nt_$i 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/nont/libmmdx_hip.so run p9_c5_nont_$i 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run p9_c5_nt_$i 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
