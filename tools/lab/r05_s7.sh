# r05 session 7: cooperative LSTM forward reordered (saves / operand loads during the gates),
# fast gate functions; probe, the LSTM tests, C4 bench pair
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-400; [ $rc -le 1 ] || exit $rc; }
run s7_probe 300 python tools/lab/lstm_probe.py
cat gpurun_out/s7_probe.log | head -30
run s7_text 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_text_gpu.py tests/test_graph_capture_gpu.py -m gpu
run s7_bench_c4 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
run s7_bench_c4b 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
run s7_bench_c3 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run s7_benched 900 python -u -m pytest -q --timeout 800 --timeout-method thread tests/test_benched_path_gpu.py -m gpu -k "c3 or c4 or bilstm"
