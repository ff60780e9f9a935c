# round 6: nontemporal epilogue stores — tests on the new default (conv / GEMM epilogues), then
# paired steps: base (plain stores, abtmp/base) / default (conv + GEMM epilogues NT) / ntbn
# (also the BN apply / backward-apply outputs NT, abtmp/ntbn) / ntall (+ phase-dgrad epilogue and
# the weight gradients' split-K slabs NT, abtmp/ntall); C5 base vs default
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; grep -E "passed|failed|^\{" $R/gpurun_out/$label.log | cut -c1-130; [ $rc -le 1 ] || exit $rc; }
run p4_t 600 python -u -m pytest tests/test_conv8_gpu.py tests/test_trunk_launches_gpu.py tests/test_gemm8_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not resnet50-256"
for i in 1 2; do
  MMDX_LIB_PATH=$R/abtmp/base/libmmdx_hip.so run p4_c4_base_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run p4_c4_nt_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntbn/libmmdx_hip.so run p4_c4_ntbn_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntall/libmmdx_hip.so run p4_c4_ntall_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
for i in 1 2; do
  MMDX_LIB_PATH=$R/abtmp/base/libmmdx_hip.so run p4_c5_base_$i 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run p4_c5_nt_$i 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
