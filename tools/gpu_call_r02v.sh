#!/bin/bash
set -u
bash run_gpu.sh tests 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread || exit 1
bash run_gpu.sh bench1 300 python bench.py --steps 40 --no-cpu-baseline || exit 2
bash run_gpu.sh bench2 300 python bench.py --steps 40 --no-cpu-baseline || exit 2
