# A/B/C of three library builds (MMDX_LIB_PATH), paired benches, two repetitions
set -u
mkdir -p gpurun_out
L=/root/repo/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib/libmmdx_hip.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py::test_conv_fwd_dgrad_wgrad -q -x --timeout 120 > gpurun_out/t_conv.log 2>&1 || { echo "tests rc=$?"; tail -5 gpurun_out/t_conv.log; exit 1; }
tail -1 gpurun_out/t_conv.log
for rep in 1 2; do
  for arm in /root/repo/abtmp/libmmdx_old.so /root/repo/abtmp/libmmdx_oldnorm.so $L; do
    n=$(basename $arm .so)_$rep
    MMDX_LIB_PATH=$arm timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab3_$n.log 2>&1 || exit 2
    echo $n $(grep -o '"value": [0-9.]*' gpurun_out/ab3_$n.log)
  done
done
MMDX_BENCH_LAUNCH_TABLE=gpurun_out/launch_table_new.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lt_new.log 2>&1
MMDX_LIB_PATH=/root/repo/abtmp/libmmdx_old.so MMDX_BENCH_LAUNCH_TABLE=gpurun_out/launch_table_old.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lt_old.log 2>&1
