#!/usr/bin/env python3
"""LDS-DMA completion probe (tools/glds_probe.hip): for each mode, the threads
that saw their LDS-staged words change after the staging barrier, over a
buffer of random bytes. usage: glds_probe.py [--gib 4] [--tile 16912] [--reps 10]"""
import argparse
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--tile", type=int, default=16912)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--stride", type=int, default=16384, help="tile starts (< tile: overlap)")
    ap.add_argument("--modes", default="0,1,4")
    ap.add_argument("--refresh", action="store_true",
                    help="rewrite the buffer (device copy) before every launch")
    args = ap.parse_args()
    import torch

    n = int(args.gib * 2**30)
    buf = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    ref = buf.clone() if args.refresh else None
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libglds_probe.so"))
    names = {0: "LDS-DMA", 1: "register staging", 2: "LDS-DMA + read-back before barrier",
             3: "LDS-DMA + s_sleep after barrier", 4: "LDS-DMA + LDS traffic",
             5: "register staging + LDS traffic"}
    for mode in [int(m) for m in args.modes.split(",")]:
        out = (ctypes.c_ulonglong * 3)()
        rc = lib.glds_probe_run(ctypes.c_void_p(buf.data_ptr()), ctypes.c_uint64(n),
                                ctypes.c_uint32(args.tile), ctypes.c_uint32(args.stride), mode,
                                args.reps, ctypes.c_void_p(ref.data_ptr() if ref is not None else 0),
                                out)
        assert rc == 0, rc
        blocks = (n + args.stride - 1) // args.stride
        print("stride %d mode %d %-36s threads: changed after barrier %d, first read != HBM %d, "
              "second read != HBM %d (of %d x %d)" % (args.stride, mode, names[mode], out[0], out[1], out[2],
                                                    blocks * 256, args.reps), flush=True)


if __name__ == "__main__":
    main()
