#!/usr/bin/env python3
"""Transcoder timing on a bench workload (config 3 / 4): the fused
wire-to-wire form (TGPU_XCODE=1) and the composed decode + encode
(TGPU_XCODE=0), indexed (the workload's offsets) or not, HIP events on the
launch stream around each call (no host status: the calls are stream-ordered
so the events time the kernels alone). Meant to run under
rocprofv3 --kernel-trace --stats for the per-kernel split.
  python tools/xc_time.py --config 3 --reps 5"""
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
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--records", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--forms", nargs="*", default=["1", "0"])
    ap.add_argument("--unindexed", action="store_true")
    args = ap.parse_args()
    import ctypes

    import torch

    import bench
    from fbthrift_amd import _lib
    from fbthrift_amd import serializer as S

    dev = torch.device("cuda:0")
    n = args.records or bench.WORKLOADS[args.config].default_records
    wl = bench.WORKLOADS[args.config](n, 0, dev)
    wl.encode()
    torch.cuda.synchronize()
    src = wl.S
    to = 2 if src.protocol == 0 else 0
    w = wl.wire[: wl.wire_bytes]
    out = torch.empty(8 * wl.wire_bytes + 16, dtype=torch.uint8, device=dev)
    offs = None if args.unindexed else wl.offs
    ctx = src.context()
    s = torch.cuda.current_stream()
    res = {}
    ref = None
    for f in args.forms:
        os.environ["TGPU_XCODE"] = f
        # first call blocking (compiles, checks), then stream-ordered calls
        _, _, st, done, size = src.transcode(wl.gs, w, wl.n, to, offsets=offs, out=out,
                                             want_offsets=False)
        assert st.code == 0 and done == wl.n, st.as_tuple()
        got = out[:size].clone()
        if ref is None:
            ref = got
        assert torch.equal(ref, got), "forms disagree"
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            _lib.lib().tgpu_transcode_batch(
                ctx.handle, wl.gs.handle, src.protocol, to, ctypes.c_void_p(w.data_ptr()),
                w.numel(), ctypes.c_void_p(offs.data_ptr()) if offs is not None else None, wl.n,
                ctypes.c_void_p(out.data_ptr()), out.numel(), None, None,
                ctypes.c_void_p(s.cuda_stream), None, None, None)
            e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res["xcode=%s" % f] = {"median_ms": round(statistics.median(ts), 4),
                               "min_ms": round(min(ts), 4)}
        print(f, res["xcode=%s" % f], flush=True)
    print(json.dumps({"config": args.config, "records": wl.n, "indexed": offs is not None,
                      "wire_bytes": wl.wire_bytes, "out_bytes": int(ref.numel()), **res}))


if __name__ == "__main__":
    main()
