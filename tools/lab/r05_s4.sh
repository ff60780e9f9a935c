# r05 session 4: re-runs (fp32 relu epilogue case x3, bn_fin tolerances, C5 update gate), then
# the one-rank RCCL rehearsal traces
set -o pipefail
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -3 gpurun_out/$label.log; [ $rc -le 1 ] || exit $rc; }
for i in 1 2 3; do
  run s4_epi_$i 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "bias_addend_preact or gelu_bwd or residual"
done
run s4_fin 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_bn_fin_gpu.py -m gpu
run s4_c5 600 python -u -m pytest -q -s --timeout 500 --timeout-method thread "tests/test_benched_path_gpu.py::test_benched_step_reduced_precision_vs_oracle[c5]" -m gpu
bash tools/lab/r05_rccl.sh
