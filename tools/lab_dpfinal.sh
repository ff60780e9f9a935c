# one-rank RCCL rehearsal of the DP step on the final code, paired with the plain step, C4 and C5
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_dp.log 2>&1 || { echo "dp tests rc=$?"; tail -30 gpurun_out/t_dp.log; exit 1; }
tail -1 gpurun_out/t_dp.log
p=29600
for cfg in c4 c5; do
  for arm in plain reh; do
    p=$((p + 1))
    if [ $arm = plain ]; then
      timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dpf_${cfg}_$arm.log 2>&1 || exit 2
    else
      MMDX_DP_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $p bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dpf_${cfg}_$arm.log 2>&1 || exit 3
    fi
    echo ${cfg}_$arm $(grep -o '"value": [0-9.]*' gpurun_out/dpf_${cfg}_$arm.log)
  done
done
