#!/usr/bin/env python3
"""Per-call timing of the config-5 decode (tgpu_decode_stream at N=1): wall
clock around each call (synchronized before and after) and HIP events on
the launch stream, for the index variants given as TGPU_INDEX_STARTS values.
  python tools/c5_time.py --records 67108864 --variants 1 0"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 26)
    ap.add_argument("--variants", nargs="*", default=["1", "0"])
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--no-check", action="store_true",
                    help="timing ablations (TGPU_ABL_*): skip the result check")
    ap.add_argument("--stats", action="store_true",
                    help="print each call's time and index repair counters (tgpu_index_stats)")
    ap.add_argument("--sync-before", action="store_true",
                    help="synchronize after the encode (decode starts on an idle GPU)")
    args = ap.parse_args()
    import torch

    import bench

    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS[5](args.records, 0, dev)
    wl.encode()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    for v in args.variants:
        os.environ["TGPU_INDEX_STARTS"] = v
        wall, evt, enc = [], [], []
        for r in range(args.reps + 2):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            torch.cuda.synchronize()
            e[0].record(s)
            wl.encode()
            if args.sync_before:
                torch.cuda.synchronize()
            e[1].record(s)
            t0 = time.perf_counter()
            wl.decode()
            t1 = time.perf_counter()
            e[2].record(s)
            torch.cuda.synchronize()
            if r >= 2:
                wall.append((t1 - t0) * 1e3)
                evt.append(e[1].elapsed_time(e[2]))
                enc.append(e[0].elapsed_time(e[1]))
            if args.stats:
                w = wl.wire[: wl.wire_bytes // 4 * 4].view(torch.int32)
                print("  rep %d: decode events %.3f ms, index repairs %s, wire sum %d" % (
                    r, e[1].elapsed_time(e[2]), wl.S.context().index_stats(),
                    int(w.sum(dtype=torch.int64))), flush=True)
        if not args.no_check:
            wl.check_timed()
        print("TGPU_INDEX_STARTS=%s decode wall %.3f ms  events %.3f ms  (encode events %.3f)"
              % (v, statistics.median(wall), statistics.median(evt), statistics.median(enc)))


if __name__ == "__main__":
    main()
