#!/usr/bin/env python3
"""Round-6 A/B of the block rule's packing in config 4's decode (interleaved,
HIP events, median decode call per variant). A variant is "env:NAME=VALUE"
and/or "#define ..." lines for the schema compiler (TGPU_JIT_DEFINES).
  python tools/pack_ab.py "env:TGPU_ARENA_PACK=0" "" "#define TGPU_PACK_GATHER"
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


SET = set()


def apply(v):
    defs = []
    for k in SET:  # (a variant's env settings end with it)
        os.environ.pop(k, None)
    SET.clear()
    for part in v.split(";"):
        if part.startswith("env:"):
            k, _, val = part[4:].partition("=")
            os.environ[k] = val
            SET.add(k)
        elif part:
            defs.append(part)
    os.environ["TGPU_JIT_DEFINES"] = "\n".join(defs)


def main():
    import torch

    import bench

    variants = sys.argv[1:] or [""]
    cfg = int(os.environ.get("AB_CONFIG", "4"))
    dev = torch.device("cuda:0")
    W = bench.WORKLOADS[cfg]
    wl = W(W.default_records, 0, dev)
    dec = {v: [] for v in variants}
    for rnd in range(int(os.environ.get("AB_ROUNDS", "4"))):
        for v in variants:
            apply(v)
            wl.gs.compile(wl.protocol)
            wl.encode()
            for _ in range(4):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                wl.decode()
                ev[1].record()
                torch.cuda.synchronize()
                dec[v].append(ev[0].elapsed_time(ev[1]))
            if rnd == 0:
                wl.check_timed()
        print("round %d done" % rnd, flush=True)
    for v in variants:
        print("config %d %-60r dec %.4f ms (min %.4f)" % (cfg, v, statistics.median(dec[v]),
                                                         min(dec[v])), flush=True)


if __name__ == "__main__":
    main()
