# C4 A/B of the session-start library against the current one (MMDX_LIB_PATH), paired, two
# repetitions; then one C5 line of the current library
set -u
mkdir -p gpurun_out
L=/root/repo/multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib/libmmdx_hip.so
for rep in 1 2; do
  for arm in /root/repo/abtmp/libmmdx_4b.so $L; do
    n=$(basename $arm .so)_$rep
    MMDX_LIB_PATH=$arm timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/abc4_$n.log 2>&1 || exit 2
    echo $n $(grep -o '"value": [0-9.]*' gpurun_out/abc4_$n.log)
  done
done
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abc5_cur.log 2>&1 || exit 3
echo c5 $(grep -o '"value": [0-9.]*' gpurun_out/abc5_cur.log)
