#!/usr/bin/env python3
"""CompactV1 against Compact on config 4's schema (i64, list<i32>, a struct of
three doubles): since round 5 a V1 schema with doubles has its own compiled
programs (little-endian FIXED ops), so its encode and indexed decode should
run at Compact's speed. Records generated on the device (the bench's
generator), encoded by each protocol's compiled encoder, then timed: best of
--reps calls, device-synchronised wall time. Also checks that the V1 decode
returns the records it was given. GPU only.

  python tools/v1_time.py [--records 8388608] [--reps 10]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 23)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    import datagen
    from fbthrift_amd import serializer as SZ
    from fbthrift_amd.schema import Schema

    n = args.records
    schema = Schema.from_table(datagen.SCHEMAS["nested"])
    rs = schema.record_size
    dev = torch.device("cuda:0")
    recs = torch.empty(n * rs, dtype=torch.uint8, device=dev)
    side = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libtgpu_datagen.so"))
    assert lib.tgpu_gen_nested_packed(ctypes.c_uint64(datagen.SEED), ctypes.c_uint64(0),
                                      ctypes.c_uint64(n), ctypes.c_void_p(recs.data_ptr()),
                                      ctypes.c_void_p(side.data_ptr()), None) == 0
    gs = SZ.GpuSchema(schema)

    def best(fn):
        fn()
        torch.cuda.synchronize()
        b = 1e9
        for _ in range(args.reps):
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            b = min(b, time.perf_counter() - t)
        return b * 1e3

    for name, S in (("compact", SZ.CompactSerializer), ("compact_v1", SZ.CompactV1Serializer)):
        gs.compile(S.protocol)
        wire, offs = S.serialize(gs, recs, n, list_base=side)
        torch.cuda.synchronize()
        out = torch.empty_like(wire)
        oo = torch.empty_like(offs)
        enc_ms = best(lambda: S.serialize(gs, recs, n, list_base=side, out=out, offsets=oo))
        got = {}

        def dec():
            got["r"] = S.deserialize_status(gs, wire, n, offs)

        dec_ms = best(dec)
        grec, garena, st, nd, cons = got["r"]
        assert st.code == 0 and nd == n, st.as_tuple()
        # the records' scalar members round-trip (list spans point into the
        # decode's own arena, so compare the re-encoded stream instead)
        back, _ = S.serialize(gs, grec, n, list_base=garena)
        assert torch.equal(back, wire), name
        print(json.dumps({"protocol": name, "records": n, "wire_bytes": wire.numel(),
                          "encode_ms": round(enc_ms, 3), "decode_indexed_ms": round(dec_ms, 3),
                          "general_records": S.context().index_stats()["general"]}), flush=True)


if __name__ == "__main__":
    main()
