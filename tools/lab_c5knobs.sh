# C5 knob sweep (paired, 2 reps): towers in series vs beside each other, 256x256 forward tiles off
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in "X=1" "MMDX_TEXT_STREAM=main" "MMDX_GEMM256_FWD_MIN=0"; do
    n=$(echo $arm | tr '=' '_')_$rep
    env $arm timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5k_$n.log 2>&1 || exit 2
    echo $n $(grep -o '"value": [0-9.]*' gpurun_out/c5k_$n.log)
  done
done
