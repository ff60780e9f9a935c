#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 `--kernel-trace` SQLite result (rocpd `*_results.db`),
in the column layout of rocprofv3's `--stats` CSV (Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs, StdDev), so tools/kstats.py and the committed profiles/*.csv read
both.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db -o profiles/<tag>_kernel_stats.csv
"""
import argparse
import csv
import math
import sqlite3
import sys
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("-o", "--out", default="")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    durs = defaultdict(list)
    for name, dur in con.execute("select name, duration from kernels"):
        durs[name].append(float(dur))
    total = sum(sum(v) for v in durs.values()) or 1.0
    rows = []
    for name, v in durs.items():
        n, s = len(v), sum(v)
        mean = s / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        rows.append(dict(Name=name, Calls=n, TotalDurationNs=int(s), AverageNs=round(mean, 1),
                         Percentage=round(100.0 * s / total, 4), MinNs=int(min(v)),
                         MaxNs=int(max(v)), StdDev=round(sd, 1)))
    rows.sort(key=lambda r: -r["TotalDurationNs"])
    out = open(a.out, "w", newline="") if a.out else sys.stdout
    w = csv.DictWriter(out, fieldnames=list(rows[0]))
    w.writeheader()
    w.writerows(rows)


if __name__ == "__main__":
    main()
