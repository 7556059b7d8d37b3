#!/usr/bin/env python3
"""Interleaved A/B timing of an environment switch of libtgpu (read at each
call, e.g. TGPU_FIXED_PATH=plan|jit) on a bench config: encode and decode
times per value; every variant's wire stream and decoded records must equal
the first's.
  python tools/kbench_env.py --config 2 --env TGPU_FIXED_PATH --vals plan jit"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--env", required=True)
    ap.add_argument("--vals", nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=4)
    args = ap.parse_args()
    import torch

    import bench

    dev = torch.device("cuda:0")
    W = bench.WORKLOADS[args.config]
    wl = W(W.default_records, 0, dev)
    enc = {v: [] for v in args.vals}
    dec = {v: [] for v in args.vals}
    ref = None
    for rnd in range(args.rounds):
        for v in args.vals:
            os.environ[args.env] = v
            for _ in range(3):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                wl.timed_step(ev)
                torch.cuda.synchronize()
                enc[v].append(ev[0].elapsed_time(ev[1]))
                dec[v].append(ev[1].elapsed_time(ev[2]))
            if rnd == 0:
                wl.check_timed()
                got = (wl.wire.clone(), wl.back.clone())
                if ref is None:
                    ref = got
                elif not (torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])):
                    raise SystemExit("variant %s=%s differs" % (args.env, v))
    for v in args.vals:
        print("config %d %s=%-10s enc %.4f ms  dec %.4f ms" % (
            args.config, args.env, v, statistics.median(enc[v]), statistics.median(dec[v])))


if __name__ == "__main__":
    main()
