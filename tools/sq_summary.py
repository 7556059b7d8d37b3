#!/usr/bin/env python3
"""Per-kernel averages of the SQ counters collected by tools/profile_round.sh.
usage: sq_summary.py DIR   (DIR/p*/**/*counter_collection*.csv)"""
import csv
import glob
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.replace("void ", "").split("(")[0].split("::")[-1][:60]


def main():
    root = sys.argv[1]
    acc = {}
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                d = acc.setdefault(k, {})
                d.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    for k, d in sorted(acc.items()):
        if "SQ_WAVES" in d and max(d["SQ_WAVES"]) < 1000:
            continue
        print(k)
        for c, v in sorted(d.items()):
            print("   %-24s %16.0f  (x%d)" % (c, sum(v) / len(v), len(v)))
        w = d.get("SQ_WAVES")
        if w:
            n = sum(w) / len(w)
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM",
                      "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if c in d:
                    print("   per wave %-18s %10.1f" % (c, sum(d[c]) / len(d[c]) / n))
        wc = d.get("SQ_WAVE_CYCLES")
        if wc:
            t = sum(wc) / len(wc)
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in d:
                    print("   frac %-22s %8.3f" % (c, sum(d[c]) / len(d[c]) / t))


if __name__ == "__main__":
    main()
