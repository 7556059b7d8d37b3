#!/usr/bin/env python3
"""Interleaved A/B timing of compiled-program decode variants on the bench's
config 3 / 4 batches (env TGPU_PROG_DECODE="sprog,capmode").
  python tools/kbench_prog.py --config 3 --dec 0,0 1,0 1,1
Each variant's decoded records must equal the first variant's."""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--dec", nargs="*", default=["0,0"])
    ap.add_argument("--records", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    import bench

    dev = torch.device("cuda:0")
    W = bench.WORKLOADS[args.config]
    wl = W(args.records or W.default_records, 0, dev)
    wl.encode()
    torch.cuda.synchronize()
    ref = None
    times = {v: [] for v in args.dec}
    enc = []
    for rnd in range(args.rounds):
        for v in args.dec:
            os.environ["TGPU_PROG_DECODE"] = v
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                wl.decode()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1))
            if rnd == 0:
                st, nd, consumed = wl.S.context().wait()
                assert st.code == 0 and consumed == wl.wire_bytes, (v, st.as_tuple())
                if ref is None:
                    ref = wl.back.clone()
                elif not torch.equal(ref, wl.back):
                    raise SystemExit("variant %s decodes differently" % v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        wl.encode()
        e1.record()
        torch.cuda.synchronize()
        enc.append(e0.elapsed_time(e1))
    dec_alg, enc_alg = wl.algorithmic()
    for v, t in times.items():
        med = statistics.median(t)
        print("config %d dec %-8s median %.4f ms min %.4f ms  %.1f GB/s" %
              (args.config, v, med, min(t), dec_alg / med / 1e6))
    med = statistics.median(enc)
    print("config %d enc median %.4f ms  %.1f GB/s" % (args.config, med, enc_alg / med / 1e6))


if __name__ == "__main__":
    main()
