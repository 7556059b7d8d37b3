"""Diagnostics (round 6, verdict housekeeping): the LDS-DMA settle in the
fixed-layout plan decode. Run with TGPU_LIB_PATH pointing at a build of the
library with -DTGPU_PLAN_STALE_CHECK (tools/build_variant.sh): every value
word the plan decode takes from its staged LDS tile is decoded a second time
from HBM, and a difference (a staged word that had not landed, whose header
bytes happened to be intact) is counted. Prints the count after K full-size
config-2 decodes (64 Mi records)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import torch

    import bench
    from fbthrift_amd import _lib

    assert "TGPU_LIB_PATH" in os.environ, "run against the diagnostics build"
    L = _lib.lib()
    f = L.tgpu_debug_plan_stale
    f.restype = ctypes.c_ulonglong
    f.argtypes = [ctypes.c_int]
    dev = torch.device("cuda:0")
    wl = bench.Flat8(1 << 26, 0, dev)
    wl.encode()
    torch.cuda.synchronize()
    f(1)
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    for _ in range(K):
        wl.decode()
    wl.verify()
    print("plan decode: %d calls x %d records, stale words %d" % (K, wl.n, f(0)), flush=True)


if __name__ == "__main__":
    main()
