# round 6: cost of the scattered BN-statistics slab stores in the conv epilogues: isolated
# fwd / dgrad with a lab build that computes the statistics but skips their stores
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; grep TOTAL $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
for i in 1 2; do
  run p2_base_$i 300 python -u tools/conv_bench.py --ops fwd,dgrad
  MMDX_LIB_PATH=$R/abtmp/nostats/libmmdx_hip.so run p2_nost_$i 300 python -u tools/conv_bench.py --ops fwd,dgrad
done
