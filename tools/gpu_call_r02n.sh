#!/bin/bash
# host-side profile of the one-rank RCCL rehearsal vs the plain step (cProfile)
set -u
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29521
MMDX_DP_REHEARSE=1 bash run_gpu.sh cprof_dp 300 python -m cProfile -o gpurun_out/dp.prof bench.py --steps 30 --no-cpu-baseline || exit 2
bash run_gpu.sh cprof 300 python -m cProfile -o gpurun_out/plain.prof bench.py --steps 30 --no-cpu-baseline || exit 3
