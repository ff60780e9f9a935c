# r05 session 11: dense split-K GEMMs in split-major XCD order (all tiles of a K split on one
# XCD) vs the per-split tile swizzle: C5 / C4 benches paired, C5 GEMM traffic
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
ALT=$R/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab/dx1024/libmmdx_hip.so
for rep in 1 2; do
  run s11_c5_def_$rep 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
  run s11_c5_dx_$rep 300 env MMDX_LIB_PATH=$ALT python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
run s11_c4_def 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
run s11_c4_dx 300 env MMDX_LIB_PATH=$ALT python bench.py --steps 30 --warmup 5 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
export MMDX_LIB_PATH=$ALT
run s11_pmcf5 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf5_dx -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
run s11_pmcw5 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw5_dx -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
