# round 6: host cProfile of the C2 step on an idle device (where its ~3.2 ms of issue go)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_profile.py --config c2 --steps 20 --idle > $R/gpurun_out/h1_c2.log 2>&1; echo rc=$?
