# full GPU suite and smoke() on the final code
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/full_suite.log 2>&1 || { echo "suite rc=$?"; tail -30 gpurun_out/full_suite.log; exit 1; }
tail -2 gpurun_out/full_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
