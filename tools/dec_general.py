#!/usr/bin/env python3
"""Records the compiled decode sends to the general reader on a canonical
stream, per call (tgpu_index_stats 'general'): configs 3 and 5 (LDS-DMA
staged decode tiles). Any non-zero count on these streams means a tile's
staged bytes did not parse as the canonical records they are."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import torch

    import bench

    dev = torch.device("cuda:0")
    for cfg in (3, 5):
        W = bench.WORKLOADS[cfg]
        wl = W(W.default_records, 0, dev)
        counts = []
        for r in range(10):
            wl.encode()
            wl.decode()
            torch.cuda.synchronize()
            counts.append(wl.S.context().index_stats()["general"])
        print("config %d: general-reader records per decode call %s" % (cfg, counts), flush=True)
        del wl
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
