# round 6 measurement set M2 on the final kernels (4443e03): C4 PMC passes — HBM traffic
# (FETCH_SIZE, WRITE_SIZE), MFMA busy, instruction mix per kernel (VALU / SALU / MFMA)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export MMDX_GIT_REV=4443e03
cd /tmp && export TMPDIR=/tmp
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run m2_f 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_r06 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run m2_w 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_r06 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run m2_m 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm_r06 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run m2_i 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES --output-format csv -d $R/gpurun_out/pmci_r06 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
