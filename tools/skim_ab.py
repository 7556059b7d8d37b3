#!/usr/bin/env python3
"""A/B timing of the schemaless skim (tgpu_skim_batch) on a bench workload:
full entry tables vs counts only (max_fields=0), to separate the parse cost
from the entry-store cost. Usage: python tools/skim_ab.py [config]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import torch

    import bench

    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS[cfg](bench.WORKLOADS[cfg].default_records if cfg != 5 else 1 << 26,
                              0, dev)
    wl.encode()
    torch.cuda.synchronize()
    offs = wl.offs if hasattr(wl, "offs") else \
        torch.arange(wl.n + 1, dtype=torch.int64, device=dev) * wl.L
    nf = len(wl.gs.schema.structs[0].fields)
    w = wl.wire[: wl.wire_bytes]
    res = {}
    fbuf = torch.empty(nf * wl.n * 16, dtype=torch.uint8, device=dev)
    cbuf = torch.empty(wl.n, dtype=torch.int32, device=dev)
    for rnd in range(5):
        for mf in (nf, 0):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            wl.S.skim(w, offs, wl.n, max_fields=mf, check=False, fields=fbuf, counts=cbuf)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mf, []).append(e0.elapsed_time(e1))
    for mf, t in res.items():
        print("config %d max_fields %d: median %.3f ms min %.3f ms" %
              (cfg, mf, statistics.median(t), min(t)), flush=True)


if __name__ == "__main__":
    main()
