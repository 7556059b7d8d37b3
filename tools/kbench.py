#!/usr/bin/env python3
"""Interleaved A/B timing of fixed-layout kernel variants in one process
(cdna_hip_programming.md §5.4 rule 24). Usage:
  python tools/kbench.py --dec 256,0,0,0 256,1,0,0 ... --enc 256,0 256,1 ...
Prints median/min decode and encode call times per variant (ms) and GB/s of
algorithmic bytes (decode 161 B/record, encode 153 B/record)."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dec", nargs="*", default=["256,0,0,0"])
    ap.add_argument("--enc", nargs="*", default=["256,0"])
    ap.add_argument("--records", type=int, default=1 << 26)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    import torch
    import bench
    import datagen
    from fbthrift_amd.schema import Schema
    from fbthrift_amd.serializer import BinarySerializer as BS, GpuSchema

    dev = torch.device("cuda:0")
    n = args.records
    gs = GpuSchema(Schema.from_table(datagen.SCHEMAS["flat8"]))
    recs = bench.gen_flat8_device(n, 0, dev)
    BS.context().reserve(n)
    wire = torch.empty(n * 89, dtype=torch.uint8, device=dev)
    back = torch.empty(n * 72, dtype=torch.uint8, device=dev)
    res = {("dec", v): [] for v in args.dec}
    res.update({("enc", v): [] for v in args.enc})
    os.environ["TGPU_PLAN_ENCODE"] = args.enc[0]
    BS.serialize(gs, recs, n, out=wire, offsets=None, sync=False)
    torch.cuda.synchronize()
    want = wire.clone()
    for rnd in range(args.rounds):
        for kind, v in list(res):
            os.environ["TGPU_PLAN_DECODE" if kind == "dec" else "TGPU_PLAN_ENCODE"] = v
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if kind == "dec":
                    BS.deserialize(gs, wire, n, records=back, sync=False)
                else:
                    BS.serialize(gs, recs, n, out=wire, offsets=None, sync=False)
                e1.record()
                torch.cuda.synchronize()
                res[(kind, v)].append(e0.elapsed_time(e1))
            if rnd == 0:
                ok = torch.equal(back, recs) if kind == "dec" else torch.equal(wire, want)
                if not ok:
                    print("MISMATCH", kind, v, flush=True)
    out = {}
    for (kind, v), ts in res.items():
        med = statistics.median(ts)
        alg = n * (161 if kind == "dec" else 153)
        out["%s %s" % (kind, v)] = {"median_ms": round(med, 4), "min_ms": round(min(ts), 4),
                                    "GBps": round(alg / med / 1e6, 1)}
        print(kind, v, out["%s %s" % (kind, v)], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
