#!/bin/bash
# final-code PMC passes (conv traffic, MFMA utilisation) and the other configs' lines
set -u
R=$GRAFT_REPO_ROOT
bash tools/gpu_round.sh r02s pmc || exit 1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm_r02s -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmcm.log 2>&1 || exit 2
cd $R
python tools/pmc_mfma.py gpurun_out/pmcm_r02s -o gpurun_out/r02s_mfma_util.json
bash run_gpu.sh c3 300 python bench.py --config c3 --steps 20 --no-cpu-baseline || exit 3
bash run_gpu.sh c2 300 python bench.py --config c2 --steps 20 --no-cpu-baseline || exit 4
bash run_gpu.sh c5 400 python bench.py --config c5 --steps 10 --no-cpu-baseline || exit 5
bash run_gpu.sh c4 300 python bench.py --steps 40 --no-cpu-baseline || exit 6
