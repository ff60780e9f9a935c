#!/bin/bash
# usage: run_gpu.sh <label> <timeout-seconds> <cmd...>; continue only on rc 0/1 (test failures)
label=$1; shift; to=$1; shift
timeout -k 10 $to "$@" > gpurun_out/$label.log 2>&1
rc=$?
echo "[$label] rc=$rc"; tail -25 gpurun_out/$label.log
[ $rc -le 1 ]
