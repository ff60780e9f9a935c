set -u
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_text_gpu.py tests/test_model_parity_gpu.py tests/test_benched_path_gpu.py tests/test_dp_gpu.py tests/test_inference_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_lab.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lab_pk -o run -- python3 $R/tools/lab/lstm_lab.py > $R/gpurun_out/lab_pk.log 2>&1 || exit 1
cd $R
timeout -k 10 200 python -u tools/step_probe.py --text-only > gpurun_out/probe_t5.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/step_probe.py --image-only > gpurun_out/probe_i5.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/step_probe.py --threads --steps 2 > gpurun_out/probe_a5.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline > gpurun_out/bench_lab.log 2>&1 || exit 1
for m in t2 t3; do
  MMDX_LIB_PATH=$R/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab/libmmdx_$m.so timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "conv_fwd_dgrad or production_m" -x -q --timeout 150 --timeout-method thread > gpurun_out/t_$m.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/conv_bench.py --ops fwd --lib multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab/libmmdx_$m.so > gpurun_out/cb_$m.log 2>&1 || exit 1
done
timeout -k 10 200 python -u tools/conv_bench.py --ops fwd > gpurun_out/cb_base.log 2>&1
