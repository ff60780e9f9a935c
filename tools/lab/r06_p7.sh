# round 6: nontemporal LDS-DMA operand loads: ntA = the k-major conv activations (im2col /
# dgrad / pointwise A operands; weights stay cached), ntR = the weight-gradient operands
# (dy^T, im2col^T); paired C4 against the default
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; [ $rc -le 1 ] || exit $rc; }
for i in 1 2; do
  run p7_def_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntA/libmmdx_hip.so run p7_ntA_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntR/libmmdx_hip.so run p7_ntR_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
MMDX_LIB_PATH=$R/abtmp/ntA/libmmdx_hip.so run p7_cb_ntA 300 python -u tools/conv_bench.py --ops fwd,dgrad
run p7_cb_def 300 python -u tools/conv_bench.py --ops fwd,dgrad,wgrad
MMDX_LIB_PATH=$R/abtmp/ntR/libmmdx_hip.so run p7_cb_ntR 300 python -u tools/conv_bench.py --ops wgrad
