#!/usr/bin/env python3
"""Interleaved A/B timing of schema-compiler variants (TGPU_JIT_DEFINES: lines
prepended to the generated unit, e.g. "#define TGPU_LDS_BYTE_SINK") on the
bench's config 3 / 4 batch: encode and decode times per variant; every
variant's wire stream and decoded records must equal the first's.
  python tools/kbench_jit.py --config 4 --var "" "#define TGPU_LDS_BYTE_SINK\""""
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
    ap.add_argument("--var", nargs="*", default=[""])
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--no-check", action="store_true",
                    help="timing-only variants (e.g. TGPU_NO_ELEM_LOAD) change the output")
    args = ap.parse_args()
    import torch

    import bench

    dev = torch.device("cuda:0")
    W = bench.WORKLOADS[args.config]
    wl = W(W.default_records, 0, dev)
    enc = {v: [] for v in args.var}
    dec = {v: [] for v in args.var}
    ref = None
    for rnd in range(args.rounds):
        for v in args.var:
            os.environ["TGPU_JIT_DEFINES"] = v
            wl.gs.compile(wl.protocol)
            for _ in range(3):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                wl.timed_step(ev)
                torch.cuda.synchronize()
                enc[v].append(ev[0].elapsed_time(ev[1]))
                dec[v].append(ev[1].elapsed_time(ev[2]))
            if rnd == 0 and not args.no_check:
                wl.check_timed()
                got = (wl.wire.clone(), wl.back.clone())
                if ref is None:
                    ref = got
                elif not (torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])):
                    raise SystemExit("variant %r differs" % v)
    for v in args.var:
        print("config %d %-40r enc %.4f ms  dec %.4f ms" % (
            args.config, v, statistics.median(enc[v]), statistics.median(dec[v])))


if __name__ == "__main__":
    main()
