# r05 final measurements on the committed tree (8-wave 128x128 defaults): bench lines (C4 with the CPU baseline, C5, C3,
# C2), C4 / C5 kernel traces, PMC traffic + MFMA passes for C4 and C5
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run f_c4 600 python bench.py --steps 30 --warmup 5
run f_c5 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
run f_c3 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run f_c2 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
run f_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r05f -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
run f_prof5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof5_r05f -o run -- python3 $R/bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline
run f_pmcf 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_r05f -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run f_pmcw 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_r05f -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run f_pmcm 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm_r05f -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c4
run f_pmcf5 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf5_r05f -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
run f_pmcw5 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw5_r05f -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
run f_pmcm5 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm5_r05f -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
