# final round-5 measurement set on the wgrad-target-256 tree: full GPU suite + smoke, C4 bench
# line (CPU baseline), C4 kernel trace, C4 PMC traffic / MFMA passes
set -o pipefail
R=$(pwd)
export MMDX_GIT_REV=aa7a9db
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run w_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run w_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run w_c4 600 python bench.py --steps 30 --warmup 5
run w_c5 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
run w_c2 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
run w_c3 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
run w_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r05w -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
run w_pmcf 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_r05w -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run w_pmcw 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_r05w -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run w_pmcm 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm_r05w -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c4
