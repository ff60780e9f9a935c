#!/usr/bin/env python3
"""Per-stream busy time of the last N bench steps from a rocprofv3 kernel trace.

Steps are delimited by the AdamW kernel (one launch per step).  For each step: wall span
(end of previous adamw -> end of this adamw), busy time per stream (union of kernel
intervals), and the top kernels by time on each stream.
    python tools/timeline.py gpurun_out/prof_X/run_kernel_trace.csv [steps]
"""
import collections
import csv
import re
import sys


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def short(n):
    n = re.sub(r"_ZN4mmdx\d+", "", n)
    return n[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [int(r["End_Timestamp"]) for r in rows if "adamw_kernel" in r["Kernel_Name"]]
    if len(ends) < 2:
        sys.exit("need >= 2 adamw launches")
    ends = ends[-(nsteps + 1):]
    for a, b in zip(ends[:-1], ends[1:]):
        ks = [r for r in rows if a < int(r["End_Timestamp"]) <= b]
        by_stream = collections.defaultdict(list)
        names = collections.defaultdict(lambda: collections.Counter())
        for r in ks:
            st = r["Stream_Id"] + "/" + r["Queue_Id"]
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            by_stream[st].append((s, e))
            names[st][short(r["Kernel_Name"])] += e - s
        print(f"step span {(b - a) / 1e6:.3f} ms, all-stream busy {union([x for v in by_stream.values() for x in v]) / 1e6:.3f} ms")
        for st, iv in sorted(by_stream.items()):
            print(f"  stream {st}: busy {union(iv) / 1e6:.3f} ms, {len(iv)} kernels")
            for n, t in names[st].most_common(6):
                print(f"      {t / 1e6:7.3f} ms  {n}")


if __name__ == "__main__":
    main()


def gaps(path, stream="0/1", top=12):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [int(r["End_Timestamp"]) for r in rows if "adamw_kernel" in r["Kernel_Name"]]
    a, b = ends[-2], ends[-1]
    ks = [r for r in rows if a < int(r["End_Timestamp"]) <= b
          and r["Stream_Id"] + "/" + r["Queue_Id"] == stream]
    g = []
    for p, q in zip(ks[:-1], ks[1:]):
        d = int(q["Start_Timestamp"]) - int(p["End_Timestamp"])
        g.append((d, short(p["Kernel_Name"]), short(q["Kernel_Name"]),
                  (int(p["End_Timestamp"]) - a) / 1e6))
    tot = sum(x[0] for x in g if x[0] > 0)
    small = sum(x[0] for x in g if 0 < x[0] < 20000)
    print(f"stream {stream}: total gap {tot / 1e6:.3f} ms, gaps < 20us sum {small / 1e6:.3f} ms "
          f"over {sum(1 for x in g if 0 < x[0] < 20000)} gaps")
    for d, pn, qn, at in sorted(g, reverse=True)[:top]:
        print(f"  {d / 1e3:8.1f} us at {at:7.3f} ms  after {pn}  before {qn}")
