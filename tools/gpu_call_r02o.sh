#!/bin/bash
# hardware-queue A/B: plain step and one-rank RCCL rehearsal at GPU_MAX_HW_QUEUES 4 vs 8
set -u
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q bash run_gpu.sh plain_q$q 300 python bench.py --steps 30 --no-cpu-baseline || exit 2
  GPU_MAX_HW_QUEUES=$q MMDX_DP_REHEARSE=1 bash run_gpu.sh dp_q$q 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2952$q bench.py --steps 30 --no-cpu-baseline || exit 3
done
GPU_MAX_HW_QUEUES=4 bash run_gpu.sh plain_q4b 300 python bench.py --steps 30 --no-cpu-baseline || exit 2
GPU_MAX_HW_QUEUES=8 bash run_gpu.sh plain_q8b 300 python bench.py --steps 30 --no-cpu-baseline || exit 2
