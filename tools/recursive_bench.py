#!/usr/bin/env python3
"""Indexed decode of the golden recursive streams (tests/golden tree_* /
chain_*: Tree {v, list<Tree> kids, tag}, boxed Node chains), each replicated
to ~1 Mi records, through the unrolled nested program (TGPU_NESTED=1) and
through the general decoder alone (TGPU_NESTED=0). Prints one JSON line per
(case, path): ms per call (device time of the whole decode call, buffers
preallocated), wire GB/s, and how many records the general decoder took;
then the encode of the decoded records the same two ways (the unrolled
writer, deferring deeper records to the general writer, and the general
writer alone). TGPU_DEEP_WIDE=0
in the environment: the general kernels' deep pass without its wide tier.

  python tools/recursive_bench.py [--reps 10] [--copies 5000]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--copies", type=int, default=5000)
    ap.add_argument("--cases", nargs="*", default=["tree_binary", "tree_compact", "chain_binary",
                                                   "chain_compact"])
    args = ap.parse_args()
    import torch

    import nested_helpers as nh
    from fbthrift_amd import _lib
    from fbthrift_amd import serializer as SZ

    os.environ["TGPU_JIT"] = "1"
    dev = torch.device("cuda:0")
    for name in args.cases:
        c = nh.NestedCase(name)
        base = np.frombuffer(c.wire, np.uint8)
        R = args.copies
        wire = torch.from_numpy(np.tile(base, R)).to(dev)
        o = c.offsets.astype(np.int64)
        offs = np.concatenate([o[:-1] + k * len(base) for k in range(R)] + [[R * len(base)]])
        offs = torch.from_numpy(offs).to(dev)
        n = c.n * R
        Ser = {0: SZ.BinarySerializer, 2: SZ.CompactSerializer}[c.protocol]
        gs = SZ.GpuSchema(c.schema)
        gs.compile(c.protocol)
        recs = torch.empty(n * gs.record_size, dtype=torch.uint8, device=dev)
        cap = Ser.arena_bytes(gs, wire.numel())
        arena = torch.empty(cap, dtype=torch.uint8, device=dev)
        lib = _lib.lib()

        def call():
            st = _lib.Status()
            nd, cons = ctypes.c_uint64(), ctypes.c_uint64()
            lib.tgpu_decode_batch(Ser.context().handle, gs.handle, Ser.protocol,
                                  ctypes.c_void_p(wire.data_ptr()), wire.numel(),
                                  ctypes.c_void_p(offs.data_ptr()), n,
                                  ctypes.c_void_p(recs.data_ptr()),
                                  ctypes.c_void_p(arena.data_ptr()), cap, None, None,
                                  ctypes.byref(st), ctypes.byref(nd), ctypes.byref(cons))
            assert st.code == 0 and nd.value == n, st.as_tuple()

        def timed(fn, reps):
            fn()  # warm-up (and the first-call compile)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t) * 1e3 / reps

        for nested in ("1", "0"):
            os.environ["TGPU_NESTED"] = nested
            ms = timed(call, args.reps)
            print(json.dumps({"case": name, "op": "decode",
                              "path": "nested" if nested == "1" else "general",
                              "deep_tiers": 1 if os.environ.get("TGPU_DEEP_WIDE") == "0" else 2,
                              "records": n, "wire_bytes": wire.numel(), "ms": round(ms, 3),
                              "wire_GBps": round(wire.numel() / ms / 1e6, 1),
                              "general_records": Ser.context().index_stats()["general"]}),
                  flush=True)
        # encode: the unrolled nested writer (round 5; records nesting past
        # its levels go to the general writer's deep pass) and the general
        # writer alone
        out = torch.empty(wire.numel(), dtype=torch.uint8, device=dev)
        woffs = torch.empty(n + 1, dtype=torch.int64, device=dev)

        def enc():
            got, _ = Ser.serialize(gs, recs, n, wire, arena, out=out, offsets=woffs)
            assert got.numel() == wire.numel()

        for nested in ("1", "0"):
            os.environ["TGPU_NESTED"] = nested
            out.zero_()
            ms = timed(enc, args.reps)
            assert torch.equal(out, wire)
            print(json.dumps({"case": name, "op": "encode",
                              "path": "nested" if nested == "1" else "general",
                              "deep_tiers": 1 if os.environ.get("TGPU_DEEP_WIDE") == "0" else 2,
                              "records": n, "wire_bytes": wire.numel(), "ms": round(ms, 3),
                              "wire_GBps": round(wire.numel() / ms / 1e6, 1),
                              "general_records": Ser.context().index_stats()["general"]}),
                  flush=True)


if __name__ == "__main__":
    main()
