# r05 session 10: default LSTM pair (8-wave fwd, partitioned bwd) vs coop bwd; round-5
# measurement artefacts: isolated conv table, C4 kernel trace, C4 PMC (traffic, MFMA), C5 PMC
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
run s10_text 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_text_gpu.py tests/test_graph_capture_gpu.py -m gpu
for rep in 1 2; do
  run s10_c4_def_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s10_c4_cbw_$rep 300 env MMDX_LSTM_BWD_COOP=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
run s10_c3 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run s10_c3_cbw 300 env MMDX_LSTM_BWD_COOP=1 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run s10_convb 600 python tools/conv_bench.py --json gpurun_out/r05_conv_shapes.json
cd /tmp && export TMPDIR=/tmp
run s10_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r05 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
run s10_pmcf 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_r05 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run s10_pmcw 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_r05 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run s10_pmcm 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm_r05 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c4
run s10_pmcm5 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm5_r05 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
run s10_pmcf5 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf5_r05 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
run s10_pmcw5 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw5_r05 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5
run s10_prof5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof5_r05 -o run -- python3 $R/bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline
