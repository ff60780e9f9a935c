#!/usr/bin/env python3
"""Which kernels the conv / BN dispatch picks at two batches: reads two rocprofv3
--kernel-trace csvs of tools/trunk_step.py (one per batch) and writes the kernel names with
their launch counts per step side by side, marking those that appear at one batch only or
with a different count (tile shape, stage count, 8-wave variant, split-K operand classes).
    python tools/dispatch_diff.py A_kernel_trace.csv B_kernel_trace.csv --labels 128 256 \
        --reps 2 > profiles/r06_dispatch_b128_vs_b256.txt
"""
import argparse
import collections
import csv
import re


def counts(path, reps):
    c = collections.Counter()
    with open(path) as f:
        for row in csv.DictReader(f):
            c[row["Kernel_Name"]] += 1
    return {k: v / reps for k, v in c.items()}


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("mmdx::", "").replace("_ZN4mmdx", "")
    return n[:160]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--labels", nargs=2, default=["A", "B"])
    ap.add_argument("--reps", type=float, default=2)
    o = ap.parse_args()
    ca, cb = counts(o.a, o.reps), counts(o.b, o.reps)
    keys = sorted(set(ca) | set(cb), key=lambda k: (-(ca.get(k, 0) + cb.get(k, 0)), k))
    la, lb = o.labels
    print(f"# launches per trunk step (fwd + bwd) at batch {la} vs {lb}; '*' = differs")
    print(f"# {'B=' + la:>7s} {'B=' + lb:>7s}  kernel")
    nd = 0
    for k in keys:
        x, y = ca.get(k, 0), cb.get(k, 0)
        mark = "*" if x != y else " "
        nd += x != y
        print(f"{mark} {x:7.1f} {y:7.1f}  {short(k)}")
    print(f"# {nd} of {len(keys)} kernel instantiations differ in launch count")


if __name__ == "__main__":
    main()
