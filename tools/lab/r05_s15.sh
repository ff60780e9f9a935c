# r05 session 15: full GPU suite on the current tree, C4 / C3 grouped-tile A/B (G 4 vs row-major)
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
L=$R/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab
run s15_suite 1100 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu
grep -E "FAILED|ERROR" gpurun_out/s15_suite.log | head -20
for rep in 1 2; do
  run s15_c4_g4_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s15_c4_g1_$rep 300 env MMDX_LIB_PATH=$L/g1/libmmdx_hip.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
run s15_c3_g4 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run s15_c3_g1 300 env MMDX_LIB_PATH=$L/g1/libmmdx_hip.so python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
