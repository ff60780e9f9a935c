#!/bin/bash
# DP rehearsal A/B: early trunk tail and early text/fusion launch on/off
set -u
run() { MMDX_DP_REHEARSE=1 bash run_gpu.sh $1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $2 bench.py --steps 30 --no-cpu-baseline; }
run dp_base 29531 || exit 2
MMDX_DP_EARLY_TAIL=0 run dp_notail 29532 || exit 2
MMDX_DP_EARLY_TAIL=0 MMDX_DP_TEXT_EARLY=0 run dp_none 29533 || exit 2
MMDX_DP_TEXT_EARLY=0 run dp_notext 29534 || exit 2
bash run_gpu.sh plain 300 python bench.py --steps 30 --no-cpu-baseline || exit 2
