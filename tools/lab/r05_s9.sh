# r05 session 9: 4-wave register-W forward (coop4) with unit-interleaved xg; tests, probe, A/B
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-400; [ $rc -le 1 ] || exit $rc; }
run s9_text 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_text_gpu.py -m gpu -k "lstm or bilstm"
run s9_probe4 300 python tools/lab/lstm_probe.py
grep -v "dir[01] wg" gpurun_out/s9_probe4.log | head -24
run s9_probe8 300 env MMDX_LSTM_FWD_COOP4=0 python tools/lab/lstm_probe.py
grep -v "dir[01] wg" gpurun_out/s9_probe8.log | head -12
run s9_tests 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_text_gpu.py tests/test_graph_capture_gpu.py -m gpu
for rep in 1 2; do
  run s9_c4_new_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s9_c4_old_$rep 300 env MMDX_LSTM_FWD_COOP4=0 MMDX_LSTM_BWD_COOP=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
run s9_benched 900 python -u -m pytest -q --timeout 800 --timeout-method thread tests/test_benched_path_gpu.py -m gpu -k "c3 or c4 or bilstm"
cd /tmp && export TMPDIR=/tmp
run s9_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s9prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
