# round 6: step timeline (MMDX_BENCH_TIMELINE: when each part of the step ends, per stream)
# on C4 / C3 / C2 / C5, after the BN argument-struct refactor's kernel tests
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
run t1_kern 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_trunk_launches_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "batchnorm or bn_ or maxpool_bn or dgrad_fused_bn or resnet50-128"
export MMDX_BENCH_TIMELINE=10
run t1_c4 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
run t1_c3 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run t1_c2 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
run t1_c5 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
