# round 6 closing: the full GPU suite and smoke on the last code
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; tail -1 $R/gpurun_out/$label.log | cut -c1-160; [ $rc -le 1 ] || exit $rc; }
run m5_suite 800 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider
run m5_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
