set -o pipefail
PT="tests -m gpu" bash tools/gpu_round.sh r05a tests,convb,bench,c5 20 || exit $?
for f in "28x28 C256 K256 3x3/2" "14x14 C256 K256 3x3/1" "7x7 C512 K512 3x3/1" "56x56 C64 K64 3x3/1"; do
  tag=$(echo "$f" | tr ' /x' '___')
  timeout -k 10 400 bash tools/pmc_conv.sh "w_$tag" "$f" wgrad > gpurun_out/pmcw_$tag.txt 2>&1 || exit $?
done
timeout -k 10 400 bash tools/pmc_conv.sh "f_14" "14x14 C256 K256 3x3/1" fwd > gpurun_out/pmcf_14.txt 2>&1 || exit $?
