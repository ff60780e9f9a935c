# r05 session 8: cooperative LSTM backward (W_hh^T in registers, dG slices exchanged),
# gate-interleaved saves; tests, probe, benches
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-400; [ $rc -le 1 ] || exit $rc; }
run s8_text 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_text_gpu.py -m gpu -k "lstm or bilstm"
run s8_probe 300 python tools/lab/lstm_probe.py
head -12 gpurun_out/s8_probe.log
run s8_tests 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_text_gpu.py tests/test_graph_capture_gpu.py -m gpu
run s8_bench_c4 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
run s8_bench_c4b 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
run s8_benched 900 python -u -m pytest -q --timeout 800 --timeout-method thread tests/test_benched_path_gpu.py -m gpu -k "c3 or c4 or bilstm"
cd /tmp && export TMPDIR=/tmp
run s8_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s8prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
