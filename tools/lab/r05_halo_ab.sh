# halo-band conv A/B: parity tests, isolated layer1 3x3 fwd / dgrad per stage count, C4 step
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_halo_gpu.py > gpurun_out/h2_tests.log 2>&1 || { tail -40 gpurun_out/h2_tests.log; exit 1; }
tail -3 gpurun_out/h2_tests.log
for h in 0 1 3 4; do MMDX_CONV_HALO=$h timeout -k 10 200 python -u tools/conv_bench.py --filter "C64 K64 3x3" --ops fwd,dgrad > gpurun_out/h2_cb$h.log 2>&1 || exit 2; echo "halo=$h"; grep -E "3x3" gpurun_out/h2_cb$h.log; done
for h in 0 1; do MMDX_CONV_HALO=$h timeout -k 10 200 python -u tools/conv_bench.py --batch 64 --filter "C64 K64 3x3" --ops fwd,dgrad > gpurun_out/h2_cb64_$h.log 2>&1 || exit 2; echo "b64 halo=$h"; grep -E "3x3" gpurun_out/h2_cb64_$h.log; done
