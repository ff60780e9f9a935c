#!/bin/bash
# final lines of the session: default bench (with the CPU baseline), kernel-trace stats
set -u
R=$GRAFT_REPO_ROOT
bash run_gpu.sh bench 400 python bench.py || exit 2
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_o -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_o.log 2>&1 || exit 3
