# round 6: nontemporal 16-B stores in the conv / GEMM epilogues (lab build abtmp/nt) vs stock:
# isolated fwd / dgrad families and paired C4 steps
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; grep -E "TOTAL (fwd|dgrad)|^\{" $R/gpurun_out/$label.log | cut -c1-140; [ $rc -le 1 ] || exit $rc; }
run p3_cb_base 300 python -u tools/conv_bench.py --ops fwd,dgrad
MMDX_LIB_PATH=$R/abtmp/nt/libmmdx_hip.so run p3_cb_nt 300 python -u tools/conv_bench.py --ops fwd,dgrad
for i in 1 2; do
  run p3_b_base_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/nt/libmmdx_hip.so run p3_b_nt_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
