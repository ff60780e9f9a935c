#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 10 --no-cpu-baseline > $R/gpurun_out/trace.log 2>&1 || exit 2
