#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace run (rocpd .db or *_kernel_stats.csv).

  python tools/prof_summary.py <dir-or-file> [--steps N] [--step-kernel NAME] [--top K] [--grid]
Prints ms/step (total / N), calls/step and the average duration per kernel, sorted by total
time; --grid splits each kernel by its launch grid (one line per (name, grid)).  N defaults to
the call count of a once-per-step kernel (--step-kernel, default the fused AdamW launch), so
warm-up and untimed steps in the trace are counted instead of assumed.
"""
import argparse
import csv
import glob
import os
import sqlite3


def _rows_db(path, by_grid):
    c = sqlite3.connect(path)
    key = "name, grid_x, grid_y, grid_z, workgroup_x" if by_grid else "name"
    q = (f"select {key}, count(*), sum(duration), avg(duration), max(scratch_size) "
         f"from kernels group by {key}")
    out = []
    for r in c.execute(q):
        if by_grid:
            name = f"{r[0]} grid=({r[1]},{r[2]},{r[3]})x{r[4]}"
            r = (name,) + r[5:]
        out.append(dict(name=r[0], calls=int(r[1]), total=float(r[2]), avg=float(r[3]),
                        scratch=int(r[4] or 0)))
    return out


def _rows_csv(path):
    out = []
    for r in csv.DictReader(open(path)):
        out.append(dict(name=r["Name"], calls=int(r["Calls"]), total=float(r["TotalDurationNs"]),
                        avg=float(r["AverageNs"]), scratch=0))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=0,
                    help="divide totals by this many steps (0: the --step-kernel call count)")
    ap.add_argument("--step-kernel", default="adamw_kernel",
                    help="substring of a kernel launched exactly once per step")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--grid", action="store_true")
    ap.add_argument("--width", type=int, default=140)
    a = ap.parse_args()
    p = a.path
    if os.path.isdir(p):
        dbs = glob.glob(os.path.join(p, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)
        p = (dbs or csvs)[0]
    rows = _rows_db(p, a.grid) if p.endswith(".db") else _rows_csv(p)
    if a.steps <= 0:
        once = [r for r in rows if a.step_kernel in r["name"]]
        if not once:
            raise SystemExit(f"no kernel matching {a.step_kernel!r}: pass --steps")
        a.steps = sum(r["calls"] for r in once)
    tot = sum(r["total"] for r in rows)
    print(f"# {p}: {len(rows)} kernels, {tot / 1e6:.2f} ms total, "
          f"{tot / 1e6 / a.steps:.3f} ms per step over {a.steps} steps "
          f"(step count: {'--steps' if a.steps and not any(a.step_kernel in r['name'] for r in rows) else a.step_kernel + ' calls or --steps'})")
    print(f"# {'ms/step':>8} {'%':>5} {'calls/step':>10} {'avg us':>9} {'scratch':>7}  kernel")
    for r in sorted(rows, key=lambda r: -r["total"])[:a.top]:
        print(f"  {r['total'] / 1e6 / a.steps:8.3f} {100 * r['total'] / tot:5.1f} "
              f"{r['calls'] / a.steps:10.1f} {r['avg'] / 1e3:9.1f} {r['scratch']:7d}  "
              f"{r['name'][:a.width]}")


if __name__ == "__main__":
    main()
