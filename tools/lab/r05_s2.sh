# r05 session 2: re-run the round's changed tests on the rebuilt library, then the quartered
# im2col^T wgrad A/B (isolated table, both arms) and the trunk per-launch checks
set -o pipefail
R=$(pwd)
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -3 gpurun_out/$label.log; [ $rc -le 1 ] || exit $rc; }
run t_changed 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_amp_gpu.py tests/test_kernels_gpu.py tests/test_gemm8_gpu.py tests/test_attention_flash_gpu.py -m gpu
run t_c5 600 python -u -m pytest -q -s --timeout 500 --timeout-method thread "tests/test_benched_path_gpu.py::test_benched_step_reduced_precision_vs_oracle[c5]" -m gpu
run t_trunk 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_trunk_launches_gpu.py -m gpu
run wg_rq1 300 env MMDX_WGRAD_RQ=1 python tools/conv_bench.py --ops wgrad
run wg_rq0 300 env MMDX_WGRAD_RQ=0 python tools/conv_bench.py --ops wgrad
run wg_rq1b 300 env MMDX_WGRAD_RQ=1 python tools/conv_bench.py --ops wgrad
