#!/bin/bash
set -u
bash run_gpu.sh probe 200 python tools/step_probe.py --threads --steps 4 || exit 2
bash run_gpu.sh probe_bt 200 python tools/step_probe.py --threads --bwd-thread --steps 4 || exit 2
bash run_gpu.sh probe_img 200 python tools/step_probe.py --image-only --steps 4 || exit 2
