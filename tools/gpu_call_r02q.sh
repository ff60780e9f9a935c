#!/bin/bash
# final lines: C4 default bench, the other configs, kernel-trace stats
set -u
bash run_gpu.sh bench 300 python bench.py || exit 2
bash run_gpu.sh c3 300 python bench.py --config c3 --steps 20 --no-cpu-baseline || exit 3
bash run_gpu.sh c2 300 python bench.py --config c2 --steps 20 --no-cpu-baseline || exit 4
bash run_gpu.sh c5 400 python bench.py --config c5 --steps 10 --no-cpu-baseline || exit 5
MMDX_DP_REHEARSE=1 bash run_gpu.sh rccl 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --steps 30 --no-cpu-baseline || exit 6
