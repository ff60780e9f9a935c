#!/usr/bin/env python3
"""MFMA utilisation of the step's kernel families from one rocprofv3 PMC pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d <dir> \
        -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
    python tools/pmc_mfma.py <dir> [-o profiles/<tag>_mfma_util.json]

SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over every SIMD (32 per
v_mfma_f32_32x32x16_bf16, 16 per 16x16x32; MI355X_MICROARCH.md price list); GRBM_GUI_ACTIVE is
the dispatch's busy cycles summed over the 8 XCDs.  Per dispatch
    util = MFMA_BUSY / (1024 SIMDs * GRBM_GUI_ACTIVE / 8),
the fraction of the chip's MFMA issue capacity the dispatch used while it ran (at the clock
it actually ran at, so DVFS does not enter).  Families are summed as cycle-weighted means.
Concurrent dispatches overlap in GRBM_GUI_ACTIVE (the chip is busy for either), so a family's
figure is its share of the MFMA capacity of the time it was resident, not an isolated rate.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

SIMDS = 256 * 4
FAMILIES = [
    ("conv_fwd", re.compile(r"igemm(_dma)?_kernel.*(Im2colK|PointFwdK)")),
    ("conv_dgrad", re.compile(r"igemm(_dma)?_kernel.*(DgradK|DgradPhaseK|PhaseTap)")),
    ("conv_wgrad", re.compile(r"igemm(_dma)?_kernel.*(Im2colR|PointWgradR)")),
    ("lstm", re.compile(r"lstm_")),
    ("gemm", re.compile(r"igemm(_dma)?_kernel|splitk")),
]


def family(name):
    for f, rx in FAMILIES:
        if rx.search(name):
            return f
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("-o", "--out", default="")
    ap.add_argument("--config", default="c4")
    ap.add_argument("--rev", default=os.environ.get("MMDX_GIT_REV", "unstamped"),
                    help="git revision the counters were measured on (the GPU box has no .git)")
    args = ap.parse_args()
    files = glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {args.dir}")
    disp = collections.defaultdict(lambda: {"name": "", "mfma": 0.0, "grbm": 0.0})
    for f in files:
        for row in csv.DictReader(open(f)):
            key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
            d = disp[key]
            d["name"] = row.get("Kernel_Name", d["name"])
            v = float(row["Counter_Value"])
            if row.get("Counter_Name") == "SQ_VALU_MFMA_BUSY_CYCLES":
                d["mfma"] += v
            elif row.get("Counter_Name") == "GRBM_GUI_ACTIVE":
                d["grbm"] += v
    fam = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for d in disp.values():
        if d["grbm"] <= 0:
            continue
        a = fam[family(d["name"])]
        a[0] += d["mfma"]
        a[1] += SIMDS * d["grbm"] / 8.0
        a[2] += 1
    conv = [fam[k] for k in ("conv_fwd", "conv_dgrad", "conv_wgrad")]
    out = {k: {"mfma_util": round(v[0] / v[1], 4) if v[1] else None, "dispatches": v[2]}
           for k, v in sorted(fam.items())}
    cm, cc = sum(v[0] for v in conv), sum(v[1] for v in conv)
    out["conv_all"] = {"mfma_util": round(cm / cc, 4) if cc else None,
                       "dispatches": sum(v[2] for v in conv)}
    out["formula"] = "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8), cycle-weighted"
    out["config"] = args.config
    out["git_rev"] = args.rev
    for k, v in out.items():
        print(f"{k:12s} {v}")
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
