# r05 session 28: strided-dgrad phase tiles back to 4 waves (MMDX_DGRAD_PHASE_8W A/B), the
# cooperative BiLSTM backward re-checked beside the 8-wave trunk, conv PMC traffic
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
run s28_par 600 python -u -m pytest -q --timeout 500 --timeout-method thread tests/test_conv8_gpu.py -m gpu
for rep in 1 2; do
  run s28_c4_0_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s28_c4_p_$rep 300 env MMDX_DGRAD_PHASE_8W=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s28_c4_l_$rep 300 env MMDX_LSTM_BWD_COOP=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
cd /tmp && export TMPDIR=/tmp
run s28_pmcf 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_s28 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run s28_pmcw 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw_s28 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
