#!/usr/bin/env python3
"""Headline benchmark: device-resident Binary-protocol encode+decode of flat
{1..8: i64} records (BASELINE.json configs[1]: 64M records per MI355X).

One step = encode the resident record batch to the Binary wire stream, then
decode that stream back into records (tgpu_encode_batch + tgpu_decode_batch,
both HBM-resident, no host sync inside the step). `value` = 2 x wire bytes x
steps x GPUs / max-over-ranks elapsed, in GiB/s.

Multi-GPU (torchrun): every rank owns an independent shard of 64M records
(weak scaling, no data-path collective); a barrier + synchronize bracket the
timed steps and the elapsed time is the max over ranks.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

METRIC = "device-resident GiB/s encode+decode, 64M flat records, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
GOLDEN = 0x9E3779B97F4A7C15
SEED = 0x1729


def gen_flat8_device(n, first, dev):
    """Config 1/2 records in the 72-byte layout, generated on the GPU with the
    counter-based splitmix64 spec of tests/golden/datagen.py (int64 torch ops;
    wrapping multiply, logical shifts emulated with masks)."""
    import torch

    def m64(x):
        return x

    def srl(x, k):
        return (x >> k) & ((1 << (64 - k)) - 1)

    def s64(v):
        return v - (1 << 64) if v >= (1 << 63) else v

    out = torch.empty((n, 9), dtype=torch.int64, device=dev)
    chunk = 1 << 22
    edges = torch.tensor([0, -1, 1, -(1 << 63), (1 << 63) - 1], dtype=torch.int64, device=dev)
    for b in range(0, n, chunk):
        e = min(n, b + chunk)
        i = torch.arange(first + b, first + e, dtype=torch.int64, device=dev)
        idx = (i.unsqueeze(1) * 8 + torch.arange(8, dtype=torch.int64, device=dev)) + 1
        z = idx * s64(GOLDEN) + SEED
        z = (z ^ srl(z, 30)) * s64(0xBF58476D1CE4E5B9)
        z = (z ^ srl(z, 27)) * s64(0x94D049BB133111EB)
        z = z ^ srl(z, 31)
        r = i % 997
        edge_rows = r < 5
        if bool(edge_rows.any()):
            k = (r.unsqueeze(1) + torch.arange(8, device=dev)) % 5
            z = torch.where(edge_rows.unsqueeze(1), edges[k], z)
        out[b:e, :8] = z
    out[:, 8] = 0x0101010101010101  # isset bytes
    return out.view(torch.uint8).reshape(-1)


def cpu_baseline(seconds=12.0):
    """The oracle's codegen-equivalent Binary encode+decode (the reference's
    generated T::write / T::readNoXfer restated, -O3 -march=native) on this
    host's cores, over a bounded sample, same metric."""
    import numpy as np

    from oracle import oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    n = 1 << 22
    recs = np.zeros(n * 72, np.uint8)
    oracle.lib().oracle_gen_flat8(SEED, 0, n, recs.ctypes.data)
    wire = np.zeros(n * 89, np.uint8)
    back = np.zeros(n * 72, np.uint8)
    L = oracle.lib()
    reps, t0 = 0, time.perf_counter()
    while True:
        L.oracle_flat8_binary_encode(recs.ctypes.data, n, wire.ctypes.data, threads)
        rc = L.oracle_flat8_binary_decode(wire.ctypes.data, n, back.ctypes.data, threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    assert rc == 0 and np.array_equal(back, recs)
    gib = 2.0 * n * 89 * reps / el / 2**30
    return {"value": round(gib, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": "%d x encode+decode of 4Mi config-2 records (%.1f s wall)" % (reps, el)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--records", type=int, default=1 << 26)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-copy-ceiling", action="store_true")
    ap.add_argument("--host-start", action="store_true",
                    help="also time pinned-host -> decode -> host and host -> encode -> host")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from fbthrift_amd.schema import Schema
    from fbthrift_amd.serializer import BinarySerializer as BS, GpuSchema, TgpuError
    import datagen

    n = args.records
    schema = Schema.from_table(datagen.SCHEMAS["flat8"])
    gs = GpuSchema(schema)
    L = gs.fixed_wire_size(0)
    assert L == 89 and schema.record_size == 72
    ctx = BS.context()
    ctx.reserve(n)

    recs = gen_flat8_device(n, rank * n, dev)  # shard `rank` of the record space
    wire = torch.empty(n * L, dtype=torch.uint8, device=dev)
    back = torch.empty(n * 72, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        BS.serialize(gs, recs, n, out=wire, offsets=None, sync=False)
        if ev:
            ev[1].record(stream)
        BS.deserialize(gs, wire, n, records=back, sync=False)
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    st, nd, consumed = ctx.wait()
    if st.code or consumed != n * L:
        raise TgpuError("warmup decode failed: %s" % (st.as_tuple(),))
    if not torch.equal(back, recs):
        raise RuntimeError("round trip mismatch")

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st, nd, consumed = ctx.wait()
    assert st.code == 0 and consumed == n * L
    enc_ms = sorted(e[0].elapsed_time(e[1]) for e in evs)
    dec_ms = sorted(e[1].elapsed_time(e[2]) for e in evs)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    wire_bytes = n * L
    value = 2.0 * wire_bytes * args.steps * world / elapsed / 2**30
    dec_avg = sum(dec_ms) / len(dec_ms) / 1e3
    enc_avg = sum(enc_ms) / len(enc_ms) / 1e3
    dec_alg = n * (89 + 72)  # read 89 wire + write 64 values + 8 isset
    enc_alg = n * (64 + 89)  # read 64 values + write 89 wire
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: splitmix64(seed 0x1729) int64 values + edge values, generated on device",
        "config": {"workload": "config 2: Binary protocol, flat {1..8: i64} records, encode+decode",
                   "records_per_gpu": n, "wire_bytes_per_gpu": wire_bytes,
                   "record_bytes": 72, "wire_bytes_per_record": L,
                   "parallelism": "dp%d (independent record shards, no collective)" % world},
        "roofline": {"bound": "hbm", "kernel": "plan_binary_decode_kernel",
                     "achieved": round(dec_alg / dec_avg / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(dec_alg / dec_avg / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": pmc_traffic("plan_binary_decode_kernel", n),
                     "algorithmic_bytes_per_launch": dec_alg,
                     "avg_launch_ms": round(dec_avg * 1e3, 4),
                     "timing": "HIP events on the launch stream around the decode call "
                               "(main kernel + 4 tiny bookkeeping kernels)",
                     "copy_ceiling": None if args.no_copy_ceiling else copy_ceiling(dev),
                     "encode": {"kernel": "plan_binary_encode_kernel",
                                "achieved": round(enc_alg / enc_avg / 1e9, 1),
                                "frac": round(enc_alg / enc_avg / 1e9 / HBM_PEAK_GBS, 4),
                                "avg_launch_ms": round(enc_avg * 1e3, 4)}},
    }
    if args.host_start and rank == 0:
        line["host_start"] = host_start(gs, recs, wire, back, n, L, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def copy_ceiling(dev, nbytes=4 << 30):
    """Measured HBM copy ceiling on this GPU: the best of the 16-byte-lane copy
    shapes in tools/copy_ceiling.hip over 4 GiB, read + write bytes / time;
    falls back to torch's device copy when that helper is not
    built. Reported beside the 8 TB/s spec `peak`."""
    import ctypes

    import torch

    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    lib_path = os.path.join(ROOT, "tools", "build", "libcopyceil.so")
    if os.path.exists(lib_path):
        lib = ctypes.CDLL(lib_path)
        ms = ctypes.c_float()
        torch.cuda.synchronize()
        best = None
        for variant in range(8):
            rc = lib.copy_ceiling_run(variant, ctypes.c_void_p(a.data_ptr()),
                                      ctypes.c_void_p(b.data_ptr()), ctypes.c_uint64(nbytes), 5,
                                      ctypes.byref(ms))
            if rc != 0:
                raise RuntimeError("copy ceiling kernel failed")
            if best is None or ms.value < best[0]:
                best = (ms.value, variant)
        t, how = best[0] / 1e3, "hip copy variant %d (best of 8)" % best[1]
    else:
        b.copy_(a)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        t, how = e0.elapsed_time(e1) / 5 / 1e3, "torch_copy"
    del a, b
    return {"GBps": round(2 * nbytes / t / 1e9, 1), "how": how}


def pmc_traffic(kernel, n):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (profiles/pmc_latest.json, written by tools/pmc_summary.py from
    separate --pmc passes, gfx950 FETCH_SIZE x2 correction applied), scaled to
    this launch's record count; None when no summary exists."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(path) as f:
            d = json.load(f)[kernel]
        return int(d["hbm_bytes_per_record"] * n)
    except (OSError, KeyError, ValueError):
        return None


def host_start(gs, recs, wire, back, n, L, dev):
    """Host-memory start/end rates (pinned buffers, PCIe-inclusive): decode =
    H2D(wire) + kernels + D2H(records); encode = H2D(records) + kernels +
    D2H(wire). Reported for DESIGN.md, never as `value`."""
    import torch

    from fbthrift_amd.serializer import BinarySerializer as BS

    h_wire = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    h_recs = torch.empty(n * 72, dtype=torch.uint8, pin_memory=True)
    h_wire.copy_(wire)
    h_recs.copy_(recs)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("decode", lambda: (wire.copy_(h_wire, non_blocking=True),
                                        BS.deserialize(gs, wire, n, records=back, sync=False),
                                        h_recs.copy_(back, non_blocking=True))),
                     ("encode", lambda: (recs.copy_(h_recs, non_blocking=True),
                                        BS.serialize(gs, recs, n, out=wire, offsets=None,
                                                     sync=False),
                                        h_wire.copy_(wire, non_blocking=True)))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / 3
        res[name + "_gibps"] = round(n * L / el / 2**30, 3)
    return res


if __name__ == "__main__":
    main()
