#!/usr/bin/env python3
"""Instruction mix per conv launch class from one rocprofv3 PMC pass:

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES \
        --output-format csv -d <dir> -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
    python tools/pmc_insts.py <dir> [--rev REV] [-o profiles/<tag>_conv_inst_mix.txt]

Per dispatch the SQ_INSTS_* counters are summed over the chip (wave-instructions).  Each
implicit-GEMM conv dispatch is classed by its operand sources (fwd: Im2colK / PointFwdK,
dgrad: DgradK / DgradPhaseK / PointDgradK, wgrad: Im2colR / PointWgradR) and by its grid
(dispatches with the same class and grid are the same trunk launch); the table gives VALU,
SALU and LDS instructions per MFMA instruction for every class, summed over the pass.
"""
import argparse
import collections
import csv
import os
import re


def klass(name):
    if "igemm" not in name:
        return None
    if re.search(r"Im2colR|PointWgradR", name):
        return "wgrad"
    if re.search(r"Dgrad", name):
        return "dgrad"
    if re.search(r"Im2colK|PointFwdK", name):
        return "fwd"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--rev", default=os.environ.get("MMDX_GIT_REV", "unstamped"))
    ap.add_argument("-o", default=None)
    a = ap.parse_args()
    rows = csv.DictReader(open(os.path.join(a.dir, "run_counter_collection.csv")))
    disp = collections.defaultdict(dict)
    for r in rows:
        k = klass(r["Kernel_Name"])
        if k is None:
            continue
        d = disp[r["Dispatch_Id"]]
        d["k"], d["grid"] = k, int(r["Grid_Size"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    fam = collections.defaultdict(lambda: collections.Counter())
    per = collections.defaultdict(lambda: collections.Counter())
    for d in disp.values():
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS"):
            fam[d["k"]][c] += d.get(c, 0.0)
            per[(d["k"], d["grid"])][c] += d.get(c, 0.0)
        fam[d["k"]]["n"] += 1
        per[(d["k"], d["grid"])]["n"] += 1

    def line(tag, c):
        m = max(c["SQ_INSTS_MFMA"], 1.0)
        return (f"{tag:28s} dispatches {int(c['n']):4d}  MFMA {c['SQ_INSTS_MFMA'] / 1e6:9.2f} M  "
                f"VALU/MFMA {c['SQ_INSTS_VALU'] / m:5.2f}  SALU/MFMA {c['SQ_INSTS_SALU'] / m:5.2f}  "
                f"LDS/MFMA {c['SQ_INSTS_LDS'] / m:5.2f}")
    out = [f"# conv instruction mix per MFMA, PMC SQ_INSTS_* (rev {a.rev}, tools/pmc_insts.py)"]
    for k in ("fwd", "dgrad", "wgrad"):
        out.append(line(k + " (family)", fam[k]))
    tot = collections.Counter()
    for k in fam:
        tot.update(fam[k])
    out.append(line("all convs", tot))
    out.append("# per launch class (class, grid), heaviest 20 by VALU + SALU instructions")
    top = sorted(per.items(), key=lambda kv: -(kv[1]["SQ_INSTS_VALU"] + kv[1]["SQ_INSTS_SALU"]))
    for (k, g), c in top[:20]:
        out.append(line(f"{k} grid {g}", c))
    text = "\n".join(out) + "\n"
    print(text, end="")
    if a.o:
        open(a.o, "w").write(text)


if __name__ == "__main__":
    main()
