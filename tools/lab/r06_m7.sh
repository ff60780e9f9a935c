# round 6: repeat of the C4 headline line (m6_c4 read 7572 on that box, its launch-table run
# right after 9626) and of the C2 line, on a fresh box
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export MMDX_GIT_REV=d74559f
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run m7_c4a 400 python bench.py --steps 30 --warmup 5
run m7_c4b 400 python bench.py --steps 30 --warmup 5
run m7_c2a 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
run m7_c2b 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
