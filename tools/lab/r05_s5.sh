# r05 session 5: which collectives the one-rank RCCL rehearsal issues per step and what the
# host spends in launch()/finish(); cProfile of the C4 and C2 host steps
set -o pipefail
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -3 gpurun_out/$label.log; [ $rc -le 1 ] || exit $rc; }
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517
run s5_dptrace 300 env MMDX_DP_REHEARSE=1 MMDX_DP_TRACE=1 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
unset RANK LOCAL_RANK WORLD_SIZE MASTER_ADDR MASTER_PORT
run s5_host_c4 300 python tools/host_profile.py --config c4 --steps 10
run s5_host_c4_idle 300 python tools/host_profile.py --config c4 --steps 10 --idle
run s5_host_c2 300 python tools/host_profile.py --config c2 --steps 20
