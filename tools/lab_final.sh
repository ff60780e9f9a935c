# round-end measurement set: C4 (default bench line, CPU baseline), C5 / C2 / C3 lines, C4 kernel
# trace, C4 PMC passes (HBM traffic, MFMA busy), C5 kernel trace
set -u
bash tools/gpu_round.sh r04z bench,c5,c2,c3,prof,pmc,pmcm 20 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r04z_c5" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config c5 --steps 10 --warmup 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_c5.log" 2>&1 || exit 3
echo c5 prof done
