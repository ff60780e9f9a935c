# r05 session 6: DP tail (small arenas packed, grads rebound to bucket views) and the
# whole-step hipGraph option (MMDX_GRAPH_STEP) at C2 / C4
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log | cut -c1-400; [ $rc -le 1 ] || exit $rc; }
run s6_dp_tests 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_dp_gpu.py -m gpu
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517
run s6_dptrace 300 env MMDX_DP_REHEARSE=1 MMDX_DP_TRACE=1 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
grep dp-trace gpurun_out/s6_dptrace.log | cut -c1-600
for rep in 1 2; do
  run s6_dp_$rep 300 env MMDX_DP_REHEARSE=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s6_plain_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
unset RANK LOCAL_RANK WORLD_SIZE MASTER_ADDR MASTER_PORT
for rep in 1 2; do
  run s6_c2_eager_$rep 300 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
  run s6_c2_graph_$rep 300 env MMDX_GRAPH_STEP=1 python bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline
done
run s6_c4_graph 300 env MMDX_GRAPH_STEP=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
run s6_c2_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c2prof -o run -- python3 $R/bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline
