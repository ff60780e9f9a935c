# dropout-in-LayerNorm: its kernel test first, then the whole GPU suite, smoke, two C5 benches
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ln_dropout_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_lnd.log 2>&1 || { echo "lnd rc=$?"; tail -30 gpurun_out/t_lnd.log; exit 1; }
tail -1 gpurun_out/t_lnd.log
TS=900 bash tools/gpu_round.sh r04t tests || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r04t.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke_r04t.log; exit 1; }
tail -1 gpurun_out/smoke_r04t.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5_lnd_$rep.log 2>&1 || exit 2
  echo c5_$rep $(grep -o '"value": [0-9.]*' gpurun_out/c5_lnd_$rep.log)
done
