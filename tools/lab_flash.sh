# flash-style attention: parity tests, stack / ViT / text tests, then C5 A/B (MMDX_ATTN_FLASH)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attention_flash_gpu.py tests/test_stack_plans_gpu.py \
  tests/test_vit_gpu.py tests/test_text_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/t_flash.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/t_flash.log; exit 1; }
tail -2 gpurun_out/t_flash.log
for rep in 1 2; do
  for f in 0 1; do
    n=flash${f}_$rep
    MMDX_ATTN_FLASH=$f timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$n.log 2>&1 || exit 2
    echo $n $(grep -o '"value": [0-9.]*' gpurun_out/ab_$n.log)
  done
done
