#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
bash run_gpu.sh dp 300 python -u -m pytest tests/test_dp_gpu.py -q -x --timeout 200 --timeout-method thread || exit 1
bash run_gpu.sh smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 2
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace2 -o run -- python3 $R/bench.py --steps 10 --no-cpu-baseline > $R/gpurun_out/trace2.log 2>&1 || exit 3
