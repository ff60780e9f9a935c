# r05 session 13: conv weight-gradient split-major XCD threshold (tiles per split) 32 / 64 / all:
# isolated wgrad table, paired C4 benches, PMC traffic per kernel
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
L=$R/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab
run s13_w32 300 python tools/conv_bench.py --ops wgrad
run s13_w64 300 python tools/conv_bench.py --ops wgrad --lib $L/sx64/libmmdx_hip.so
run s13_wall 300 python tools/conv_bench.py --ops wgrad --lib $L/sx1k/libmmdx_hip.so
for rep in 1 2; do
  run s13_c4_32_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s13_c4_64_$rep 300 env MMDX_LIB_PATH=$L/sx64/libmmdx_hip.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s13_c4_all_$rep 300 env MMDX_LIB_PATH=$L/sx1k/libmmdx_hip.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
cd /tmp && export TMPDIR=/tmp
export MMDX_LIB_PATH=$L/sx1k/libmmdx_hip.so
run s13_pmcf 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_sxall -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run s13_pmcw 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_sxall -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
