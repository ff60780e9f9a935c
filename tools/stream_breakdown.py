#!/usr/bin/env python3
"""Per-stream, per-category kernel time of one bench step from a rocprofv3 kernel trace
(steps delimited by the AdamW launch).   python tools/stream_breakdown.py <kernel_trace.csv>"""
import collections
import csv
import re
import sys


def cat(n):
    if "lstm" in n:
        return "lstm"
    if "igemm" in n and re.search(r"Im2colR", n):
        return "conv_wgrad"
    if "wgrad_reduce" in n:
        return "conv_wgrad"
    if "igemm" in n and re.search(r"Dgrad|PhaseTap", n):
        return "conv_dgrad"
    if "igemm" in n and "Im2colK" in n:
        return "conv_fwd"
    if "igemm" in n or "splitk" in n:
        return "gemm"
    if "bn_" in n:
        return re.sub(r".*(bn_\w+?)_kernel.*", r"\1", n)
    if "pack_weight" in n:
        return "pack"
    return "other"


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ad = [r for r in rows if "adamw_kernel" in r["Kernel_Name"]]
t0, t1 = int(ad[-2]["End_Timestamp"]), int(ad[-1]["End_Timestamp"])
tot = collections.defaultdict(float)
busy = collections.defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 or e > t1:
        continue
    q = r["Queue_Id"]
    tot[(q, cat(r["Kernel_Name"]))] += (e - s) / 1e6
    busy[q].append((s, e))
print(f"step span {(t1 - t0) / 1e6:.3f} ms")
for q in sorted(busy):
    iv = sorted(busy[q])
    u, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                u += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    u += ce - cs
    print(f"queue {q}: busy {u / 1e6:.3f} ms, {len(iv)} kernels")
    for (qq, c), v in sorted(tot.items(), key=lambda x: -x[1]):
        if qq == q:
            print(f"    {c:16s} {v:7.3f} ms")
