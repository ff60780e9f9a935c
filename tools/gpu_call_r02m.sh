#!/bin/bash
# DP rehearsal kernel trace + bench lines of the other configs
set -u
R=$GRAFT_REPO_ROOT
bash run_gpu.sh bench 300 python bench.py --steps 30 || exit 2
MMDX_DP_REHEARSE=1 bash run_gpu.sh rccl 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 bench.py --steps 30 --no-cpu-baseline || exit 3
export TMPDIR=/tmp
cd /tmp
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29518 MMDX_DP_REHEARSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_dp -o run -- python3 $R/bench.py --steps 10 --no-cpu-baseline > $R/gpurun_out/prof_dp.log 2>&1 || exit 4
cd $R
bash run_gpu.sh c3 300 python bench.py --config c3 --steps 20 --no-cpu-baseline || exit 5
bash run_gpu.sh c2 300 python bench.py --config c2 --steps 20 --no-cpu-baseline || exit 6
bash run_gpu.sh c5 400 python bench.py --config c5 --steps 10 --no-cpu-baseline || exit 7
