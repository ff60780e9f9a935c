#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
bash run_gpu.sh tests 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread || exit 1
bash run_gpu.sh bench1 300 python bench.py --steps 40 --no-cpu-baseline || exit 2
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_w -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_w.log 2>&1 || exit 3
