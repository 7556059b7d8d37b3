#!/usr/bin/env python3
"""Prints BASELINE.md §4's results table from bench.py JSON lines
(profiles/<round>/c{1..5}.json): encode / decode GiB/s of wire bytes per
direction (HIP events around each call), the decode roofline fraction, and
the CPU baseline (all usable host cores, and one core)."""
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "profiles/r02"


def load(c):
    p = os.path.join(d, "c%d.json" % c)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.loads(f.read().strip().splitlines()[-1])


rows = ["| Config | GPUs | Encode GiB/s | Decode GiB/s | Roofline fraction (decode) | "
        "CPU GiB/s (cores) | CPU 1 core |", "|---|---|---|---|---|---|---|"]
c1 = load(1)
if c1:
    g = c1.get("gpu_plumbing", {})
    rows.append("| 1 | 0 (+1 plumbing) | — | — | — | %.2f ns/record round trip (1 core) | "
                "GPU 1k-record round trip %s µs |" % (c1["value"], g.get("us_per_round_trip_call", "—")))
for c in (2, 3, 4, 5):
    j = load(c)
    if not j:
        continue
    w = j["config"]["wire_bytes_per_gpu"]
    r = j["roofline"]
    dec = w / (r["avg_launch_ms"] * 1e-3) / 2**30
    enc = w / (r["encode"]["avg_launch_ms"] * 1e-3) / 2**30
    cb = j.get("cpu_baseline", {})
    rows.append("| %d | %d | %.0f | %.0f | %.3f (%s) | %s (%s) | %s |" % (
        c, j["n_gpus"], enc, dec, r["frac"], r["kernel"], cb.get("value", "—"), cb.get("cores", "—"),
        cb.get("single_core", {}).get("value", "—")))
print("\n".join(rows))
