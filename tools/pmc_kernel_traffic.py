#!/usr/bin/env python3
"""HBM traffic per kernel instantiation and launch grid from the two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE; gfx950 bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1 KiB), per train step:
where a family's bytes beyond its algorithmic count go.

    python tools/pmc_kernel_traffic.py <fetch_dir> <write_dir> [--steps N] [--top K] [--match RE]
"""
import argparse
import collections
import csv
import glob
import os
import re


def load(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            # the two passes are separate runs of the same command: dispatch ids line up
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            grid = row.get("Grid_Size") or row.get("Grid_Size_X")
            o = out.setdefault(key, [row.get("Kernel_Name", ""), grid,
                                     row.get("Workgroup_Size") or row.get("Workgroup_Size_X"), 0.0])
            o[3] += float(row["Counter_Value"])
    return out


def short(name):
    m = re.search(r"igemm_dma_kernelILi(\d+)ELi(\d+)ENS_\d+Dma(\w+?)ILi\d+ENS_\d+(\w+?)I.*?"
                  r"NS_\d+Dma(\w+?)ILi\d+ENS_\d+(\w+?)I", name)
    if m:
        return f"igemm {m.group(1)}x{m.group(2)} A={m.group(4)} B={m.group(6)}"
    m = re.search(r"igemm_dma_kernelILi(\d+)ELi(\d+)ENS_\d+Dma(\w+?)ILi\d+ENS_\d+(\w+?)I", name)
    if m:
        return f"igemm {m.group(1)}x{m.group(2)} A={m.group(4)} B=same"
    return re.sub(r"^(void )?(_ZN4)?(mmdx::)?", "", name)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--steps", type=int, default=0, help="0: adamw_kernel dispatches")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--match", default=r"igemm|reduce")
    a = ap.parse_args()
    f, w = load(a.fetch_dir, "FETCH_SIZE"), load(a.write_dir, "WRITE_SIZE")
    steps = a.steps or sum(1 for v in f.values() if "adamw_kernel" in v[0]) or 1
    rx = re.compile(a.match)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for k, (name, grid, wg, v) in f.items():
        if not rx.search(name):
            continue
        e = agg[(short(name), grid, wg)]
        e[0] += 1
        e[1] += 2 * v * 1024
        e[2] += (w[k][3] if k in w else 0.0) * 1024
    tot = sum(e[1] + e[2] for e in agg.values())
    print(f"# {len(agg)} (kernel, grid) groups, {tot / steps / 1e9:.2f} GB per step over {steps} steps")
    print("#  MB/step  calls/step  MB/call (fetch)  blocks  kernel")
    for (nm, grid, wg), e in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:a.top]:
        blocks = int(grid) // max(1, int(wg)) if grid and wg else 0
        print(f"{(e[1] + e[2]) / steps / 1e6:10.1f} {e[0] / steps:8.1f} "
              f"{(e[1] + e[2]) / e[0] / 1e6:9.1f} ({e[1] / e[0] / 1e6:6.1f}) {blocks:6d}  {nm}")


if __name__ == "__main__":
    main()
