#!/bin/bash
# PMC passes on one conv shape (tools/conv_bench.py --filter), for main-loop diagnosis.
# usage: bash tools/pmc_conv.sh <tag> "<filter>" <ops>
tag=$1; filt=$2; ops=${3:-fwd}
R=$(pwd); export TMPDIR=/tmp; cd /tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE TA_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_${tag}_$i" -o run -- \
    python3 "$R/tools/conv_bench.py" --filter "$filt" --ops "$ops" --reps 5 > "$R/gpurun_out/pmc_${tag}_$i.log" 2>&1 || exit $?
done
cd "$R"
python3 - "$tag" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/pmc_{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "igemm" not in n and "wgrad_reduce" not in n: continue
        key = n[:90]
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
