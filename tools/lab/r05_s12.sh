# r05 session 12: text tower backward issued before the image trunk's (the trunk plan call
# blocks the host ~9.8 ms, so the text backward used to start only at the end of the step)
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-200; [ $rc -le 1 ] || exit $rc; }
for rep in 1 2; do
  run s12_c4_first_$rep 300 env MMDX_TEXT_BWD_FIRST=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s12_c4_def_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
run s12_c4_first_cbw 300 env MMDX_TEXT_BWD_FIRST=1 MMDX_LSTM_BWD_COOP=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
run s12_c5_first 300 env MMDX_TEXT_BWD_FIRST=1 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
run s12_c5_def 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
run s12_c3_first 300 env MMDX_TEXT_BWD_FIRST=1 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run s12_c3_def 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
run s12_c2_first 300 env MMDX_TEXT_BWD_FIRST=1 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
run s12_c2_def 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
export MMDX_TEXT_BWD_FIRST=1
run s12_tr 420 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $R/gpurun_out/s12tr -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
