# one-rank RCCL rehearsal of the data-parallel step (comm path, in-place segment all-reduces)
set -u
mkdir -p gpurun_out
for cfg in c4 c5; do
  MMDX_DP_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --config $cfg --steps 20 --warmup 5 \
    --no-cpu-baseline > gpurun_out/rehearse_$cfg.log 2>&1 || { echo "rehearse $cfg rc=$?"; tail -20 gpurun_out/rehearse_$cfg.log; exit 2; }
  echo rehearse_$cfg $(grep -o '"value": [0-9.]*\|"parallelism": "[^"]*"' gpurun_out/rehearse_$cfg.log)
done
