# round 6, call 1: baseline on the round-5 kernels with the new bench (busy-time roofline,
# --gpus N launcher rehearsed with gloo on one GPU), isolated conv table, kernel-trace csv
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run s1_c4 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
MMDX_DIST_BACKEND=gloo run s1_g2 300 python bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu-baseline
run s1_cb 300 python -u tools/conv_bench.py --json $R/gpurun_out/s1_cb.json
cd /tmp && export TMPDIR=/tmp
run s1_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06a -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
