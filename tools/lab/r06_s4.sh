# round 6, call 4: register-epilogue store pattern probe (lab build MMDX_LAB_EPI=4: BN
# statistics as now, then 16-B stores of 8 channels per lane straight from the accumulators, no
# LDS staging; wrong values, timing only) vs the product kernels, isolated
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run s4_cb 300 python -u tools/conv_bench.py --ops fwd,dgrad
run s4_lab4 300 python -u tools/conv_bench.py --ops fwd,dgrad --lib multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab/libmmdx_lab4.so
run s4_cb2 300 python -u tools/conv_bench.py --ops fwd,dgrad
run s4_lab4b 300 python -u tools/conv_bench.py --ops fwd,dgrad --lib multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab/libmmdx_lab4.so
