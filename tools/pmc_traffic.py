#!/usr/bin/env python3
"""HBM traffic of the conv kernels (C2-C4) or the dense GEMMs (C5, --family gemm) from two
rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE  --output-format csv -d <dir_f> -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE  --output-format csv -d <dir_w> -- python3 bench.py ...
    python tools/pmc_traffic.py <dir_f> <dir_w> --config c4 --batch 128 -o profiles/r01_conv_traffic.json

FETCH_SIZE / WRITE_SIZE are kilobytes; on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced read (MI355X_MICROARCH.md §HBM), so  bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024.
Conv kernels are the implicit-GEMM instantiations whose operand source is an im2col/dgrad
gather (`Im2colK`, `DgradK`, `Im2colR`) or a pointwise conv's dense operand (`PointFwdK`,
`PointDgradK`, `PointWgradR`) plus the split-K `wgrad_reduce_kernel`; the per-launch
figure divides by the number of conv CALLS (steps x --calls-per-step; steps = AdamW
dispatches), the unit bench.py's `roofline.achieved` times.
"""
import argparse
import csv
import glob
import json
import os
import re

CONV = re.compile(r"igemm(_dma)?_kernel.*(Im2col|Dgrad|PhaseTap|PointFwdK|PointWgradR)")
# C5's family: every implicit-GEMM instantiation (all dense there) + its split-K reduces
GEMM = re.compile(r"igemm(_dma)?_kernel")
GEMM_REDUCE = re.compile(r"splitk_reduce")
STEP = re.compile(r"adamw_kernel")
REDUCE = re.compile(r"wgrad_reduce_kernel")


def load(d, counter, fam=None, red=None):
    fam = fam or CONV
    red = red or REDUCE
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per_dispatch = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
            name = row.get("Kernel_Name", "")
            v = float(row["Counter_Value"])
            prev = per_dispatch.get(key, (name, 0.0))
            per_dispatch[key] = (name, prev[1] + v)
    conv_kb = red_kb = 0.0
    n_conv = n_step = 0
    for name, v in per_dispatch.values():
        if STEP.search(name):
            n_step += 1
        if fam.search(name):
            conv_kb += v
            n_conv += 1
        elif red.search(name):
            red_kb += v
    return conv_kb, red_kb, n_conv, n_step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--config", default="c4")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--calls-per-step", type=int, default=158,
                    help="conv calls per train step (bench.py's conv_launches_per_step)")
    ap.add_argument("--family", choices=("conv", "gemm"), default="conv")
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--rev", default=os.environ.get("MMDX_GIT_REV", "unstamped"),
                    help="git revision the counters were measured on (the GPU box has no .git)")
    a = ap.parse_args()
    fam, red = (GEMM, GEMM_REDUCE) if a.family == "gemm" else (CONV, REDUCE)
    f_conv, f_red, n_f, s_f = load(a.fetch_dir, "FETCH_SIZE", fam, red)
    w_conv, w_red, n_w, s_w = load(a.write_dir, "WRITE_SIZE", fam, red)
    if n_f == 0 or n_f != n_w or s_f == 0 or s_f != s_w:
        raise SystemExit(f"dispatch counts differ or zero: conv {n_f}/{n_w}, steps {s_f}/{s_w}")
    # per conv CALL (the unit bench.py's roofline times: one fwd, dgrad or wgrad call, which
    # may be several dispatches: phase dgrad, split-K wgrad + reduce)
    calls = s_f * a.calls_per_step
    fetch = 2.0 * (f_conv + f_red) * 1024 / calls
    write = (w_conv + w_red) * 1024 / calls
    out = {
        "config": a.config, "per_gpu_batch": a.batch, "git_rev": a.rev,
        "dispatches": n_f, "steps": s_f,
        "calls": calls,
        "family": a.family,
        "kernels": ("igemm(_dma)_kernel (Im2colK/DgradK/DgradPhaseK/Im2colR/PointFwdK/PointDgradK/PointWgradR sources) + wgrad_reduce_kernel"
                    if a.family == "conv" else
                    "igemm(_dma)_kernel (dense GEMM instantiations) + splitk_reduce kernels"),
        "fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(write),
        "traffic_bytes_per_launch": round(fetch + write),
        "reduce_share": round((2 * f_red + w_red) * 1024 / calls / max(1.0, fetch + write), 4),
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)",
    }
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
