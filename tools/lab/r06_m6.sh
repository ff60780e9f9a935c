# round 6 final measurement set (d74559f, after the BN ReLU-mode kernels): full GPU suite, smoke,
# C4 line (CPU baseline), C4 launch table, C5 / C3 / C2 lines, C4 kernel trace + stats, PMC passes
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export MMDX_GIT_REV=d74559f
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
run m6_suite 800 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider
run m6_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run m6_c4 400 python bench.py --steps 30 --warmup 5
MMDX_BENCH_EVENT_STEPS=10 MMDX_BENCH_LAUNCH_TABLE=$R/gpurun_out/m6_c4_launch_table.txt run m6_c4lt 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
run m6_c5 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
run m6_c3 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run m6_c2 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
run m6_prof 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06h -o run -- python3 $R/bench.py --steps 14 --warmup 3 --no-cpu-baseline
run m6_pf 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_r06h -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run m6_pw 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_r06h -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run m6_pm 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm_r06h -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
