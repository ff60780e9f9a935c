# HBM traffic (PMC FETCH_SIZE / WRITE_SIZE passes) of the C4 conv family per wgrad split target
set -o pipefail
R=$(pwd); cd /tmp && export TMPDIR=/tmp
for t in 512 384 256; do
  for c in FETCH_SIZE WRITE_SIZE; do
    MMDX_WGRAD_TARGET=$t timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/wtp_${t}_$c -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/wtp_${t}_$c.log 2>&1 || exit 2
  done
  cd $R && python3 tools/pmc_traffic.py gpurun_out/wtp_${t}_FETCH_SIZE gpurun_out/wtp_${t}_WRITE_SIZE --config c4 --batch 128 -o gpurun_out/wtp_$t.json > gpurun_out/wtp_$t.txt 2>&1; echo "target=$t rc=$?"; tail -4 gpurun_out/wtp_$t.txt; cd /tmp
done
