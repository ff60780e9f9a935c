# round 6 measurement set M1 on the final kernels (2cf7e25): full GPU suite (verbose), smoke,
# C4 bench line (CPU baseline), C4 per-launch table, C5 / C2 / C3 lines
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export MMDX_GIT_REV=2cf7e25
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
run m1_suite 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider
run m1_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run m1_c4 400 python bench.py --steps 30 --warmup 5
MMDX_BENCH_EVENT_STEPS=10 MMDX_BENCH_LAUNCH_TABLE=$R/gpurun_out/m1_c4_launch_table.txt run m1_c4lt 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
run m1_c5 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
run m1_c2 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
run m1_c3 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
