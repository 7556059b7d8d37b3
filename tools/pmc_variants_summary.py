#!/usr/bin/env python3
"""Per-kernel HBM bytes per record of tools/pmc_variants.sh's runs (FETCH x2
as calibrated, WRITE x1; DESIGN.md §6 PMC method).
  python tools/pmc_variants_summary.py gpurun_out/pmcvar/c4 33554432 decode"""
import csv
import glob
import sys


def main():
    root, n, pat = sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else ""
    for d in sorted(glob.glob(root + "/v*")):
        v = open(d + "/variant.txt").read().strip()
        out = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            vals = {}
            for f in glob.glob("%s/%s/*counter_collection.csv" % (d, ctr)):
                for r in csv.DictReader(open(f)):
                    k = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
                    if pat in k:
                        vals.setdefault(k, []).append(float(r["Counter_Value"]))
            out[ctr] = vals
        for k in sorted(out["WRITE_SIZE"]):
            f = out["FETCH_SIZE"].get(k, [0.0])
            w = out["WRITE_SIZE"][k]
            print("%-40r %-28s fetch %6.1f  write %6.1f B/record" %
                  (v, k, 2 * 1024 * sum(f) / len(f) / n, 1024 * sum(w) / len(w) / n))


if __name__ == "__main__":
    main()
