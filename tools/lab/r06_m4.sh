# round 6 closing check (4597da7): conv / kernel / per-launch trunk tests, smoke, C4 line with the
# CPU baseline, C3 / C5 lines
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export MMDX_GIT_REV=4597da7
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-160; [ $rc -le 1 ] || exit $rc; }
run m4_t 700 python -u -m pytest tests/test_conv8_gpu.py tests/test_kernels_gpu.py tests/test_trunk_launches_gpu.py tests/test_benched_path_gpu.py -q --timeout 400 --timeout-method thread -p no:cacheprovider
run m4_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run m4_c4 400 python bench.py --steps 30 --warmup 5
run m4_c3 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run m4_c5 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
