# round 6, call 2: the retired-variant tree — full GPU suite (+ C3 per-launch parity), smoke,
# C4 bench, the --gpus 2 launcher (gloo ranks on one GPU), B=128 vs 256 dispatch diff,
# isolated conv table, kernel-trace csv
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run s2_suite 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
run s2_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run s2_c4 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
MMDX_DIST_BACKEND=gloo run s2_g2 300 python bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
run s2_d128 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/disp128 -o run -- python3 $R/tools/trunk_step.py --batch 128
run s2_d256 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/disp256 -o run -- python3 $R/tools/trunk_step.py --batch 256
run s2_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06b -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
cd $R
run s2_cb 300 python -u tools/conv_bench.py --json $R/gpurun_out/s2_cb.json
# epilogue decomposition of the conv kernels (lab builds: 1 = no BN statistics, 2 = statistics
# only (no staging / store), 3 = no epilogue): isolated fwd / dgrad / wgrad tables
for v in 1 2 3; do
  run s2_lab$v 300 python -u tools/conv_bench.py --lib multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab/libmmdx_lab$v.so --json $R/gpurun_out/s2_lab$v.json
done
