# round 6: does recording the timeline's events slow the step?  wall time of the marked steps
# with all marks vs start + optimizer only (C4, C5)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-100; [ $rc -le 1 ] || exit $rc; }
export MMDX_BENCH_TIMELINE=40
run t2_c4a 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
MMDX_BENCH_TIMELINE_MARKS=optimizer run t2_c4b 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
MMDX_BENCH_TIMELINE_MARKS=text_bwd,image_bwd,optimizer run t2_c4c 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run t2_c5a 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
MMDX_BENCH_TIMELINE_MARKS=optimizer run t2_c5b 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
MMDX_BENCH_TIMELINE_MARKS=text_bwd,image_bwd,optimizer run t2_c5c 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
