#!/bin/bash
# A/B of alternative library builds on the isolated conv shapes (tools/conv_bench.py --lib),
# arms interleaved twice.
# usage: bash tools/lab/ab_conv.sh <tag> <arm dirs under lib_ab/...>
set -u
tag=$1; shift
R=$(pwd); mkdir -p gpurun_out
P=multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/lib_ab
for rep in 1 2; do
  for arm in "$@"; do
    timeout -k 10 300 python tools/conv_bench.py --lib $P/$arm/libmmdx_hip.so \
      --json gpurun_out/ab_${tag}_${arm}_$rep.json > gpurun_out/ab_${tag}_${arm}_$rep.log 2>&1
    rc=$?; echo "[$arm $rep] rc=$rc"; tail -3 gpurun_out/ab_${tag}_${arm}_$rep.log
    [ $rc -le 1 ] || exit $rc
  done
done
