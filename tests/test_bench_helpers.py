"""bench.py's reporting helpers on CPU: the roofline's PMC traffic of a call
made of several kernels (config 5: index speculation + indexed decode, named
joined by '+') is the sum of their committed per-record HBM bytes
(profiles/r<NN>/pmc/pmc_c5.json, tools/pmc_summary.py); a summary stamped
with other kernel sources than the tree's (tools/srchash.py) is refused, and
a kernel without counters gives None (reported as null, never guessed)."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tree(tmp_path, summaries):
    """A repo root sharing this tree's kernel sources, with the given
    {round: summary} PMC files."""
    os.symlink(os.path.join(ROOT, "fbthrift_amd"), tmp_path / "fbthrift_amd")
    os.symlink(os.path.join(ROOT, "include"), tmp_path / "include")
    for rnd, d in summaries.items():
        p = tmp_path / "profiles" / rnd / "pmc"
        p.mkdir(parents=True)
        (p / "pmc_c5.json").write_text(json.dumps(d))
    return str(tmp_path)


def _summary(h):
    return {"config": 5, "source_hash": h,
            "tgpu_jit_index_spec": {"hbm_bytes_per_record": 70.5},
            "tgpu_jit_decode": {"hbm_bytes_per_record": 119.0}}


def test_pmc_traffic_sums_the_calls_kernels(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from srchash import source_hash

    root = _tree(tmp_path, {"r04": _summary(source_hash(ROOT)), "r05": _summary("0" * 16)})
    n = 1 << 20
    t, src = bench.pmc_traffic("tgpu_jit_index_spec+tgpu_jit_decode", n, 5, root=root)
    assert t == int((70.5 + 119.0) * n) and src == "profiles/r04/pmc/pmc_c5.json"
    assert bench.pmc_traffic("tgpu_jit_decode", n, 5, root=root)[0] == int(119.0 * n)
    assert bench.pmc_traffic("no_such_kernel", n, 5, root=root)[0] is None
    assert bench.pmc_traffic("tgpu_jit_index_spec+no_such_kernel", n, 5, root=root)[0] is None


def test_pmc_traffic_refuses_stale_sources(tmp_path):
    root = _tree(tmp_path, {"r04": _summary("0123456789abcdef")})
    t, why = bench.pmc_traffic("tgpu_jit_decode", 1 << 20, 5, root=root)
    assert t is None and "stale" in why and "r04" in why
