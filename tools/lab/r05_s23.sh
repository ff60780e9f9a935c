# r05 sessions 2+3: the round's changed tests on the rebuilt library, the fused BN finalize
# (kernel tests, per-launch trunk checks, benched steps), the quartered im2col^T wgrad A/B
# (isolated table per arm), paired C4 benches with the fused finalize on / off
set -o pipefail
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -3 gpurun_out/$label.log; [ $rc -le 1 ] || exit $rc; }
run t_fin 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_bn_fin_gpu.py -m gpu
run t_changed 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_amp_gpu.py tests/test_kernels_gpu.py tests/test_gemm8_gpu.py tests/test_attention_flash_gpu.py -m gpu
run t_trunk 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_trunk_launches_gpu.py tests/test_graph_capture_gpu.py -m gpu
run t_bench 900 python -u -m pytest -q -s --timeout 600 --timeout-method thread tests/test_benched_path_gpu.py -m gpu
run wg_rq1 300 env MMDX_WGRAD_RQ=1 python tools/conv_bench.py --ops wgrad
run wg_rq0 300 env MMDX_WGRAD_RQ=0 python tools/conv_bench.py --ops wgrad
for rep in 1 2; do
  run b_fin1_$rep 300 env MMDX_BN_FIN=1 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run b_fin0_$rep 300 env MMDX_BN_FIN=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
run b_rq0 300 env MMDX_WGRAD_RQ=0 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
