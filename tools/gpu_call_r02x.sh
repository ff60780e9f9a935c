#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
ALT=$R/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_alt/libmmdx_hip.so
bash run_gpu.sh tpool 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "pool or stem" --timeout 120 --timeout-method thread || exit 1
MMDX_LIB_PATH=$ALT bash run_gpu.sh tpool_alt 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "pool" --timeout 120 --timeout-method thread || exit 1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_rows -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_rows.log 2>&1 || exit 3
MMDX_LIB_PATH=$ALT timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_alt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_alt.log 2>&1 || exit 3
cd $R
for k in 1 2; do
bash run_gpu.sh b_rows$k 300 python bench.py --steps 40 --no-cpu-baseline || exit 2
MMDX_LIB_PATH=$ALT bash run_gpu.sh b_alt$k 300 python bench.py --steps 40 --no-cpu-baseline || exit 2
done
