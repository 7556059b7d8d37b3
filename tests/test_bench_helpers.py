"""bench.py's reporting helpers on CPU: the roofline's PMC traffic of a call
made of several kernels (config 5: index speculation + starts copy +
indexed decode, named joined by '+') is the sum of their committed
per-record HBM bytes (profiles/pmc_c5.json, tools/pmc_summary.py); a kernel
without a summary gives None (reported as null, never guessed)."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pmc_traffic_sums_the_calls_kernels():
    with open(os.path.join(ROOT, "profiles", "pmc_c5.json")) as f:
        d = json.load(f)
    ks = ["tgpu_jit_index_spec", "index_starts_copy_kernel", "tgpu_jit_decode"]
    n = 1 << 20
    want = int(sum(d[k]["hbm_bytes_per_record"] for k in ks) * n)
    assert bench.pmc_traffic("+".join(ks), n, 5) == want
    assert bench.pmc_traffic(ks[0], n, 5) == int(d[ks[0]]["hbm_bytes_per_record"] * n)


def test_pmc_traffic_unknown_kernel_is_none():
    assert bench.pmc_traffic("no_such_kernel", 1 << 20, 5) is None
    assert bench.pmc_traffic("tgpu_jit_index_spec+no_such_kernel", 1 << 20, 5) is None
