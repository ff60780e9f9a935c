# AdamW: 4 vectors per thread in flight (bit-identical per element) and the chunk size
# (MMDX_ADAMW_CHUNK): optimizer tests, then C5 / C4 paired arms
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "adamw or clip or amp" tests/test_amp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_adamw.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_adamw.log; exit 1; }
tail -1 gpurun_out/t_adamw.log
for cfg in c5 c4; do
  for rep in 1 2; do
    for arm in pre n64 n16 n8; do
      unset MMDX_LIB_PATH MMDX_ADAMW_CHUNK
      case $arm in pre) export MMDX_LIB_PATH=$R/abtmp/libmmdx_pre.so;; n16) export MMDX_ADAMW_CHUNK=16384;; n8) export MMDX_ADAMW_CHUNK=8192;; esac
      timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/adamw_${cfg}_$arm$rep.log 2>&1 || exit 2
      echo ${cfg}_$arm$rep $(grep -o '"value": [0-9.]*' gpurun_out/adamw_${cfg}_$arm$rep.log)
    done
  done
done
