#!/bin/bash
# round-2 session GPU call: parity suite, bench, one-rank RCCL rehearsal, kernel-trace stats,
# PMC traffic + MFMA passes.  Stops at the first GPU step that faults or times out.
set -u
R=$GRAFT_REPO_ROOT
bash run_gpu.sh tests 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread || exit 1
bash run_gpu.sh bench 300 python bench.py --steps 30 || exit 2
MMDX_DP_REHEARSE=1 bash run_gpu.sh rccl 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 bench.py --steps 30 --no-cpu-baseline || exit 3
bash tools/gpu_round.sh r02l prof,pmc || exit 4
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm_r02l -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmcm.log 2>&1 || exit 5
cd $R
python tools/pmc_mfma.py gpurun_out/pmcm_r02l -o gpurun_out/r02l_mfma_util.json
