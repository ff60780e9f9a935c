# r05 session 16: batch-partitioned LSTM backward with next-step operand prefetch and dG via
# LDS chunks (W_hh stream depth 8 with a small spill vs depth 4): probe, tests, C4 pairs
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
L=$R/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab
run s16_text 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_text_gpu.py -m gpu -k "lstm or bilstm"
run s16_probe_d8 300 python tools/lab/lstm_probe.py
grep "alone" gpurun_out/s16_probe_d8.log
run s16_probe_d4 300 env MMDX_LIB_PATH=$L/d4/libmmdx_hip.so python tools/lab/lstm_probe.py
grep "alone" gpurun_out/s16_probe_d4.log
for rep in 1 2; do
  run s16_c4_d8_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s16_c4_d4_$rep 300 env MMDX_LIB_PATH=$L/d4/libmmdx_hip.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
cd /tmp && export TMPDIR=/tmp
run s16_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_s16 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
