#!/usr/bin/env python3
"""Hash of the kernel sources a PMC summary describes: every file under
fbthrift_amd/csrc plus include/thrift_gpu.h, in name order. tools/pmc_summary.py
stamps it into each profiles/**/pmc_*.json, and bench.py's pmc_traffic()
refuses a summary whose stamp differs from the tree being benched (the
counters would describe other kernels).  usage: srchash.py [ROOT]"""
import hashlib
import os
import sys

EXTS = (".hip", ".h", ".cpp", ".py", "Makefile")


def source_hash(root):
    h = hashlib.sha256()
    csrc = os.path.join(root, "fbthrift_amd", "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith(EXTS))
    paths = [os.path.join(csrc, f) for f in files] + [os.path.join(root, "include", "thrift_gpu.h")]
    for p in paths:
        h.update(os.path.relpath(p, root).encode())
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash(sys.argv[1] if len(sys.argv) > 1
                      else os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
