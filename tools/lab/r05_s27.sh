# r05 session 27: where C4 / C5 time goes after the 8-wave defaults (kernel traces) + conv table
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run s27_cb 300 python tools/conv_bench.py --json gpurun_out/s27_conv_shapes.json
cd /tmp && export TMPDIR=/tmp
run s27_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s27 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
run s27_prof5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof5_s27 -o run -- python3 $R/bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline
