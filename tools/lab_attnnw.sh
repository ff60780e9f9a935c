# flash forward block size: tests, then C5 paired over MMDX_ATTN_FWD_NW (default = 16 for L > 128)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_flash_gpu.py tests/test_stack_plans_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_nw.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_nw.log; exit 1; }
tail -1 gpurun_out/t_nw.log
for rep in 1 2; do
  for nw in 0 8; do
    MMDX_ATTN_FWD_NW=$nw timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/nw_${nw}_$rep.log 2>&1 || exit 2
    echo nw_${nw}_$rep $(grep -o '"value": [0-9.]*' gpurun_out/nw_${nw}_$rep.log)
  done
done
