# rocprofv3 kernel stats of the C4 bench for three library builds (MMDX_LIB_PATH)
set -u
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$R/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib/libmmdx_hip.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py::test_conv_fwd_dgrad_wgrad tests/test_trunk_launches_gpu.py -q -x --timeout 200 > gpurun_out/t_conv.log 2>&1 || { echo "tests rc=$?"; tail -5 gpurun_out/t_conv.log; exit 1; }
tail -1 gpurun_out/t_conv.log
cd /tmp
for arm in $R/abtmp/libmmdx_old.so $R/abtmp/libmmdx_oldnorm.so $L; do
  n=$(basename $arm .so)
  MMDX_LIB_PATH=$arm timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof3_$n" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof3_$n.log" 2>&1 || exit 2
  echo $n $(grep -o '"value": [0-9.]*' "$R/gpurun_out/prof3_$n.log")
done
cd $R
for rep in 1 2; do
  for arm in $R/abtmp/libmmdx_old.so $R/abtmp/libmmdx_oldnorm.so $L; do
    n=$(basename $arm .so)_$rep
    MMDX_LIB_PATH=$arm timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab3_$n.log 2>&1 || exit 2
    echo $n $(grep -o '"value": [0-9.]*' gpurun_out/ab3_$n.log)
  done
done
