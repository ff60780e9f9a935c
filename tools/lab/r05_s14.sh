# r05 session 14: grouped tile order for wide GEMM grids (MMDX_TILE_GROUP 8 default vs 1 / 4):
# kernel tests, paired C5 / C4 benches, C5 and C4 PMC traffic
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
L=$R/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab
run s14_tests 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm8_gpu.py tests/test_conv8_gpu.py tests/test_trunk_launches_gpu.py -m gpu
for rep in 1 2; do
  run s14_c5_g8_$rep 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run s14_c5_g1_$rep 300 env MMDX_LIB_PATH=$L/g1/libmmdx_hip.so python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run s14_c5_g4_$rep 300 env MMDX_LIB_PATH=$L/g4/libmmdx_hip.so python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
for rep in 1 2; do
  run s14_c4_g8_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s14_c4_g1_$rep 300 env MMDX_LIB_PATH=$L/g1/libmmdx_hip.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
cd /tmp && export TMPDIR=/tmp
run s14_pmcf5 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf5_g8 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
run s14_pmcw5 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw5_g8 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
run s14_pmcf 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_g8 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run s14_pmcw 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_g8 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
