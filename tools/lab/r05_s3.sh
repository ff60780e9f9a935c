# r05 session 3: fused BN finalize (mmdx_conv_fwd_bnfin) — kernel tests, the trunk's per-launch
# checks, the benched bf16 steps, then paired C4 benches with the fusion on / off
set -o pipefail
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -3 gpurun_out/$label.log; [ $rc -le 1 ] || exit $rc; }
run s3_fin 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_fin_gpu.py -m gpu
run s3_trunk 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_trunk_launches_gpu.py tests/test_graph_capture_gpu.py -m gpu
run s3_bench_path 900 python -u -m pytest -q -s --timeout 600 --timeout-method thread tests/test_benched_path_gpu.py -m gpu -k "c4 or c2"
for rep in 1 2; do
  run s3_fin1_$rep 300 env MMDX_BN_FIN=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run s3_fin0_$rep 300 env MMDX_BN_FIN=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
