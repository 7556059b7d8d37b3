#!/usr/bin/env python3
"""Single-pass vs two-pass stream index + decode on config 3's stream (the
config-5 data): decode_stream timing per mode (TGPU_INDEX_ONEPASS), results
compared, and the single pass's look-back statistics (TGPU_ONEPASS_STATS).
  python tools/onepass_diag.py [records_log2]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import torch

    import bench

    n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
    dev = torch.device("cuda:0")
    wl = bench.Mixed(n, 0, dev)
    wl.encode()
    torch.cuda.synchronize()
    w = wl.wire[: wl.wire_bytes]
    S = wl.S
    os.environ["TGPU_ONEPASS_STATS"] = "1"
    stats = len(sys.argv) > 2
    if stats:  # look-back counters compiled in (slower: atomics on one address)
        os.environ["TGPU_JIT_DEFINES"] = "#define TGPU_ONEPASS_STATS"
        wl.gs.compile(wl.protocol)
    res = {}
    variants = os.environ.get("ONEPASS_VARIANTS", "")
    modes = ["0", "1", "0", "1"] + [v for v in variants.split(";") if v]
    for mode in modes:
        if mode not in ("0", "1"):  # a JIT define variant of the single pass (timing only)
            os.environ["TGPU_JIT_DEFINES"] = mode
            os.environ["TGPU_INDEX_ONEPASS"] = "1"
        else:
            os.environ["TGPU_INDEX_ONEPASS"] = mode
        rec = torch.zeros(n * wl.gs.record_size, dtype=torch.uint8, device=dev)
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = S.decode_stream(wl.gs, w, max_records=n, offsets=offs, records=rec)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        st = out[-1]
        print("mode %s: %.3f ms n=%d first=%d last=%d status=%s" % (
            mode, dt * 1e3, out[3], out[4], out[5], st.as_tuple()), flush=True)
        res[mode] = (rec, offs)
        if mode not in ("0", "1"):
            os.environ.pop("TGPU_JIT_DEFINES", None)
            continue
    a, b = res["0"], res["1"]
    print("records equal", torch.equal(a[0], b[0]), "offsets equal", torch.equal(a[1], b[1]))


if __name__ == "__main__":
    main()
