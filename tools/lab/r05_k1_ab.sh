# single-K-tile conv variant (MMDX_CONV_K1): parity, isolated 1x1 C64 / K64 shapes, paired C4
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_k1_gpu.py tests/test_conv8_gpu.py > gpurun_out/k1_tests.log 2>&1 || { tail -40 gpurun_out/k1_tests.log; exit 1; }
tail -2 gpurun_out/k1_tests.log
for k in 0 1; do MMDX_CONV_K1=$k timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/k1_cb$k.log 2>&1 || exit 2; echo "k1=$k"; grep -E "1x1/1 .*(C64 |K64 )" gpurun_out/k1_cb$k.log | grep -E "fwd|dgrad"; grep TOTAL gpurun_out/k1_cb$k.log; done
for r in 1 2; do for k in 0 1; do MMDX_CONV_K1=$k timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/k1_b${k}_$r.log 2>&1 || exit 3; echo "k1=$k $r $(grep -o '"value": [0-9.]*' gpurun_out/k1_b${k}_$r.log | head -1)"; done; done
