#!/bin/bash
# One GPU-box session: parity tests, headline bench, kernel-trace profile, two PMC passes.
# usage (from the repo root, under gpurun): bash tools/gpu_round.sh <tag> <phases> [steps]
#   phases: comma list of tests,abtest,bench,c5,c2,c3,host,rehab,gemmb,convb,convab,benchab,prof,pmc,pmcm
# Every GPU step has its own time limit; the script stops at the first step that faults,
# aborts or times out (rc > 1), so nothing else touches the GPU after a failure.
set -u
tag=${1:-r01}; phases=${2:-tests,bench}; steps=${3:-20}
has() { [[ ",$phases," == *",$1,"* ]]; }
R=$(pwd)
mkdir -p gpurun_out
step() {  # step <label> <timeout> <cmd...>
  local label=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$R/gpurun_out/$label.log" 2>&1
  local rc=$?
  echo "[$label] rc=$rc"; tail -4 "$R/gpurun_out/$label.log"
  [ $rc -le 1 ] || exit $rc
}
export TMPDIR=/tmp
# PT overrides the test selection (e.g. PT="tests/test_amp_gpu.py -x"); TT the per-test limit
has tests && step tests ${TS:-900} python -u -m pytest ${PT:-tests -m gpu -x} -v -s -rA \
  --timeout ${TT:-120} --timeout-method thread
# the test selection PT2 once per arm of an env knob (AB_VAR = AB_A / AB_B)
if has abtest; then
  for arm in "$AB_A" "$AB_B"; do
    step "abtest_$(basename "$arm")" ${TS:-900} env "$AB_VAR=$arm" python -u -m pytest $PT2 -v -s -rA \
      --timeout ${TT:-120} --timeout-method thread
  done
fi
has bench && step bench 600 python bench.py --steps "$steps" --warmup 5 ${BA:-}
has c5 && step c5 600 python bench.py --config c5 --steps "$steps" --warmup 5 --no-cpu-baseline
has c2 && step c2 600 python bench.py --config c2 --steps "$steps" --warmup 5 --no-cpu-baseline
has c3 && step c3 600 python bench.py --config c3 --steps "$steps" --warmup 5 --no-cpu-baseline
has host && step host 300 python tools/host_profile.py --config ${HC:-c4} --steps 5
# the one-rank RCCL rehearsal of the data-parallel step, once per arm of AB_VAR
if has rehab; then
  for rep in 1 2; do
    for arm in "$AB_A" "$AB_B"; do
      step "rehab_$(basename "$arm")_$rep" 300 env "$AB_VAR=$arm" MMDX_DP_REHEARSE=1 \
        python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port $((29500 + rep)) bench.py --steps 30 --warmup 5 --no-cpu-baseline
    done
  done
fi
has gemmb && step gemmb 300 python tools/gemm_bench.py --dtype ${GD:-f16}
has convb && step convb 600 python tools/conv_bench.py --json "gpurun_out/${tag}_conv_shapes.json"
# A/B of an env knob (AB_VAR, arms AB_A / AB_B): conv table per arm, then paired benches
if has convab; then
  for arm in "$AB_A" "$AB_B"; do
    step "convab_$(basename "$arm")" 600 env "$AB_VAR=$arm" python tools/conv_bench.py --ops "${AB_OPS:-fwd,dgrad,wgrad}"
  done
fi
if has benchab; then
  for rep in 1 2; do
    for arm in "$AB_A" "$AB_B"; do
      step "benchab_$(basename "$arm")_$rep" 300 env "$AB_VAR=$arm" python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BA:-}
    done
  done
fi
cd /tmp
has prof && step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" \
  -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline ${PA:-}
has pmc && step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmcf_$tag" \
  -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline
has pmc && step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmcw_$tag" \
  -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline
has pmcm && step pmc_mfma 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d "$R/gpurun_out/pmcm_$tag" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline \
  --config "${PC:-c4}"
cd "$R"
has pmcm && python tools/pmc_mfma.py "gpurun_out/pmcm_$tag" --config "${PC:-c4}" \
  -o "gpurun_out/${tag}_${PC:-c4}_mfma_util.json"
has pmc && python tools/pmc_traffic.py "gpurun_out/pmcf_$tag" "gpurun_out/pmcw_$tag" --config c4 \
  --batch 128 -o "gpurun_out/${tag}_conv_traffic.json"
exit 0
