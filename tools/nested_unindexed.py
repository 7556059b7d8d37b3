"""Times the nested leg's stream decoded without an index (the file loop over
a nested schema): tgpu_decode_batch with offsets = None builds the record
index on the device first. Prints one JSON line (best of reps, HIP events)."""
import json
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from fbthrift_amd import serializer as SZ  # noqa: E402


def main(n=1 << 22, reps=3):
    dev = torch.device("cuda:0")
    schema, recs, lbase, *_ = bench.nested_batch(dev, n)
    gs = SZ.GpuSchema(schema)
    Ser = SZ.BinarySerializer
    Ser.context().reserve(n)
    gs.compile(0)
    wire, offs = Ser.serialize(gs, recs, n, list_base=lbase)
    arena = torch.empty(Ser.arena_bytes(gs, wire.numel()) + 16, dtype=torch.uint8, device=dev)
    back = torch.empty(n * schema.size[0], dtype=torch.uint8, device=dev)
    out = {"records": n, "wire_bytes": wire.numel()}
    for name, o in (("indexed", offs), ("unindexed", None)):
        t = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            Ser.deserialize(gs, wire, n, offsets=o, records=back, arena=arena, sync=False)
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1))
        st, nd, cons = Ser.context().wait()
        assert st.code == 0 and nd == n, st.as_tuple()
        out[name + "_ms"] = round(min(t[1:]), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
