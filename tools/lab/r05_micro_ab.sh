# A/B of the session-start library (abtmp/libmmdx_base.so) against the current build:
# conv parity tests on the current build, isolated conv table and paired C4 benches
set -o pipefail
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv8_gpu.py tests/test_conv_halo_gpu.py tests/test_trunk_launches_gpu.py > gpurun_out/m_tests.log 2>&1 || { tail -30 gpurun_out/m_tests.log; exit 1; }
tail -2 gpurun_out/m_tests.log
for arm in base new; do
  if [ $arm = base ]; then L=$R/abtmp/libmmdx_base.so; else L=$R/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib/libmmdx_hip.so; fi
  timeout -k 10 300 python -u tools/conv_bench.py --lib $L > gpurun_out/m_cb_$arm.log 2>&1 || exit 2
  echo "$arm"; grep TOTAL gpurun_out/m_cb_$arm.log
done
for r in 1 2; do for arm in base new; do
  if [ $arm = base ]; then export MMDX_LIB_PATH=$R/abtmp/libmmdx_base.so; else unset MMDX_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/m_b_${arm}_$r.log 2>&1 || exit 3
  echo "$arm $r $(grep -o '"value": [0-9.]*' gpurun_out/m_b_${arm}_$r.log | head -1)"
done; done
