# r05: where the one-rank RCCL rehearsal's overhead goes.  Kernel + marker traces of the C4
# bench with and without the data-parallel path (one rank, RCCL process group from env://,
# no launcher: rocprofv3 runs python itself), then the paired benches without the profiler.
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -2 $R/gpurun_out/$label.log; [ $rc -le 1 ] || exit $rc; }
export TMPDIR=/tmp
cd /tmp
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517
run rccl2_tr_dp 420 env MMDX_DP_REHEARSE=1 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $R/gpurun_out/rccl2_dp -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
run rccl2_tr_plain 420 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $R/gpurun_out/rccl2_plain -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline
cd $R
for rep in 1 2; do
  run rccl2_b_dp_$rep 300 env MMDX_DP_REHEARSE=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run rccl2_b_plain_$rep 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
