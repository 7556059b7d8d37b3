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
TRACE_MARKS = os.environ.get("BENCH_TRACE_MARKS", "") == "1"
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


def cpu_threads():
    """Host cores this process can run on: its CPU affinity, capped by the
    cgroup's CPU quota (a GPU box shares a larger machine: nproc shows all of
    its CPUs, the quota is this job's share). Returns (threads, detail)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return threads, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_cpu_quota": quota}


def _timed(fn, seconds):
    """Runs fn() until `seconds` have passed (at least twice); returns the
    mean seconds per call and the call count."""
    fn()
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return el / reps, reps


def cpu_baseline(wl, seconds=8.0):
    """The oracle's codegen-equivalent encode+decode of the workload's schema
    (the reference's generated T::write / T::readNoXfer restated for it,
    -O3 -march=native, oracle/thrift_oracle.cpp) on this host's cores over a
    bounded sample of the same records, same metric (2 x wire bytes / (encode
    + decode time)); also on one core. Output formats equal the device's
    (string spans = SHARE views, list elements into an arena). Config 5
    decodes the way the reference reads a file: one cursor, record after
    record (Serializer.h:97-100)."""
    import numpy as np

    from oracle import oracle

    L = oracle.lib()
    threads, detail = cpu_threads()
    cfg = wl.config_id
    if cfg == 2:
        n = 1 << 22
        recs = np.zeros(n * 72, np.uint8)
        L.oracle_gen_flat8(SEED, 0, n, recs.ctypes.data)
        wire = np.zeros(n * 89, np.uint8)
        back = np.zeros(n * 72, np.uint8)

        def step(t):
            L.oracle_flat8_binary_encode(recs.ctypes.data, n, wire.ctypes.data, t)
            assert L.oracle_flat8_binary_decode(wire.ctypes.data, n, back.ctypes.data, t) == 0

        def check():
            assert np.array_equal(back, recs)
        wire_bytes = n * 89
    else:
        n = min(wl.n, 1 << 22)
        rs = wl.record_bytes
        recs = wl.recs[: n * rs].cpu().numpy()
        side = wl.side[: n * 64].cpu().numpy()
        sizes = np.zeros(n, np.uint64)
        offs = np.zeros(n + 1, np.uint64)
        back = np.zeros(n * rs, np.uint8)
        size_fn = L.oracle_mixed_compact_size if wl.schema == "mixed" else \
            L.oracle_nested_binary_size
        size_fn(recs.ctypes.data, n, sizes.ctypes.data, threads)
        np.cumsum(sizes, out=offs[1:])
        wire_bytes = int(offs[-1])
        wire = np.zeros(wire_bytes + 16, np.uint8)
        arena = np.zeros(wire_bytes + 16, np.uint8)
        starts = np.zeros(n + 1, np.uint64)

        def step(t):
            # serializedSize pass + scan + write (one contiguous stream), then
            # the decode
            size_fn(recs.ctypes.data, n, sizes.ctypes.data, t)
            np.cumsum(sizes, out=offs[1:])
            if wl.schema == "mixed":
                L.oracle_mixed_compact_encode(recs.ctypes.data, n, side.ctypes.data,
                                              wire.ctypes.data, offs.ctypes.data, t)
                if cfg == 5:
                    got = L.oracle_mixed_compact_read_file(wire.ctypes.data, wire_bytes, n,
                                                           back.ctypes.data, starts.ctypes.data)
                    assert got == n
                else:
                    assert L.oracle_mixed_compact_decode(wire.ctypes.data, offs.ctypes.data, n,
                                                         back.ctypes.data, t) == 0
            else:
                L.oracle_nested_binary_encode(recs.ctypes.data, n, side.ctypes.data,
                                              wire.ctypes.data, offs.ctypes.data, t)
                assert L.oracle_nested_binary_decode(wire.ctypes.data, offs.ctypes.data, n,
                                                     back.ctypes.data, arena.ctypes.data, t) == 0

        def check():
            a, b = recs.reshape(n, rs), back.reshape(n, rs)
            for lo, hi in wl.fixed_ranges:
                assert np.array_equal(a[:, lo:hi], b[:, lo:hi])
            g = wl.wire[: wire_bytes].cpu().numpy() if cfg != 5 else None
            if g is not None:
                assert np.array_equal(wire[:wire_bytes], g)  # same bytes as the GPU's
    t_all, reps = _timed(lambda: step(threads), seconds)
    check()
    t_one, reps1 = _timed(lambda: step(1), seconds / 2)
    gib = lambda t: round(2.0 * wire_bytes / t / 2**30, 3)
    return {"value": gib(t_all), "unit": "GiB/s", "cores": threads, "kind": "port",
            "single_core": {"value": gib(t_one), "unit": "GiB/s", "cores": 1},
            "host": detail,
            "ns_per_record_1core": round(t_one / n * 1e9, 2),
            "sample": "%d x encode+decode of %d config-%d records (%d + %d reps, %.1f s)" % (
                reps + reps1, n, cfg, reps, reps1, t_all * reps + t_one * reps1)}


class Workload:
    """One BASELINE config: resident inputs, one encode+decode step, checks."""
    total_wire_bytes = None  # whole-job bytes per direction (default: per rank x world)
    parallelism = "dp%d (independent record shards, no collective)"

    def timed_step(self, ev):
        mark = TRACE_MARKS and self.trace_mark
        if mark:
            mark()
        ev[0].record(self.stream)
        self.encode()
        ev[1].record(self.stream)
        if mark:
            # (BENCH_TRACE_MARKS=1, profiling runs only: one tiny torch kernel
            # before each timed call and after the last, outside the events, so
            # tools/stats_check.py can cut the kernel trace into the timed
            # calls; the decode is then timed from a second event after it)
            mark()
            ev[3].record(self.stream)
        self.decode()
        ev[2].record(self.stream)
        if mark:
            mark()

    def trace_mark(self):
        import torch

        torch.cuda._sleep(64)  # (at::cuda spin_kernel: a name nothing else launches)

    def check_timed(self):
        st, nd, consumed = self.S.context().wait()
        if st.code or consumed != self.wire_bytes:
            raise RuntimeError("timed decode failed: %s" % (st.as_tuple(),))


class Flat8(Workload):
    """Config 2: Binary, flat {1..8: i64} (72-byte records, 89-byte wire)."""
    config_id = 2
    name = "config 2: Binary protocol, flat {1..8: i64} records, encode+decode"
    default_records = 1 << 26
    # (the lane-stationary plan kernels, k_plan_binary.hip, default since round 5)
    dec_kernel, enc_kernel = "plan_binary_decode_ls_kernel", "plan_binary_encode_ls_kernel"

    def __init__(self, n, rank, dev):
        import torch

        from fbthrift_amd.schema import Schema
        from fbthrift_amd.serializer import BinarySerializer, GpuSchema
        import datagen

        self.S = BinarySerializer
        self.gs = GpuSchema(Schema.from_table(datagen.SCHEMAS["flat8"]))
        self.L = self.gs.fixed_wire_size(0)
        assert self.L == 89 and self.gs.record_size == 72
        self.n = n
        self.S.context().reserve(n)
        self.recs = gen_flat8_device(n, rank * n, dev)  # shard `rank` of the record space
        self.wire = torch.empty(n * self.L, dtype=torch.uint8, device=dev)
        self.back = torch.empty(n * 72, dtype=torch.uint8, device=dev)
        self.stream = torch.cuda.current_stream()
        self.wire_bytes = n * self.L
        self.record_bytes = 72

    def encode(self):
        self.S.serialize(self.gs, self.recs, self.n, out=self.wire, offsets=None, sync=False)

    def decode(self):
        self.S.deserialize(self.gs, self.wire, self.n, records=self.back, sync=False)

    def verify(self):
        import torch

        st, nd, consumed = self.S.context().wait()
        if st.code or consumed != self.wire_bytes:
            raise RuntimeError("decode failed: %s" % (st.as_tuple(),))
        if not torch.equal(self.back, self.recs):
            raise RuntimeError("round trip mismatch")

    def algorithmic(self):
        # decode reads 89 wire + writes 64 values + 8 isset;
        # encode reads 64 values + writes 89 wire.
        return self.n * (89 + 72), self.n * (64 + 89)


class VarLen(Workload):
    """Configs 3 / 4: variable-length records. The encode writes the record
    index (n+1 offsets) the decode then uses; the round trip is checked by
    comparing the fixed members and re-encoding the decoded batch, which must
    reproduce the wire stream byte for byte."""
    jit_decode = "tgpu_jit_decode"

    def __init__(self, n, rank, dev):
        import ctypes

        import torch

        from fbthrift_amd.schema import Schema
        from fbthrift_amd.serializer import BinarySerializer, CompactSerializer, GpuSchema
        import datagen

        self.S = CompactSerializer if self.protocol == 2 else BinarySerializer
        schema = Schema.from_table(datagen.SCHEMAS[self.schema])
        self.gs = GpuSchema(schema)
        # the schema compiler's kernels (tgpu_jit.cpp), compiled up front like
        # the reference's generated code; TGPU_JIT=0 keeps the interpreter
        if os.environ.get("TGPU_JIT", "") != "0" and self.gs.compile(self.protocol):
            self.dec_kernel, self.enc_kernel = self.jit_decode, "tgpu_jit_write"
            self.index_kernel = "tgpu_jit_index_spec"
        self.n = n
        self.record_bytes = rs = schema.record_size
        self.S.context().reserve(n)
        self.stream = torch.cuda.current_stream()
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libtgpu_datagen.so"))
        self.recs = torch.empty(n * rs, dtype=torch.uint8, device=dev)
        self.side = torch.empty(n * 64, dtype=torch.uint8, device=dev)  # string / list payloads
        # payload bytes (strings / list elements) packed back to back in record
        # order (tools/datagen.hip: the columnar layout a caller hands over)
        gen = lib.tgpu_gen_mixed_packed if self.schema == "mixed" else lib.tgpu_gen_nested_packed
        if gen(ctypes.c_uint64(datagen.SEED), ctypes.c_uint64(rank * n), ctypes.c_uint64(n),
               ctypes.c_void_p(self.recs.data_ptr()), ctypes.c_void_p(self.side.data_ptr()),
               ctypes.c_void_p(self.stream.cuda_stream)):
            raise RuntimeError("device record generator failed")
        self.sbase = self.side if self.schema == "mixed" else None
        self.lbase = self.side if self.schema == "nested" else None
        self.offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        _, total = self.S.encoded_size(self.gs, self.recs, n, self.offs, list_base=self.lbase)
        self.wire_bytes = total
        self.wire = torch.empty(total, dtype=torch.uint8, device=dev)
        self.back = torch.empty(n * rs, dtype=torch.uint8, device=dev)
        cap = self.S.arena_bytes(self.gs, total)
        self.arena = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev) if cap else None
        # payload bytes behind the spans: string bytes (config 3) or list
        # elements, 4 bytes each (config 4)
        v = self.recs.view(n, rs)
        lens = [v[:, o:o + 16].contiguous().view(torch.int64)[:, 1] & 0xFFFFFFFF
                for o in self.span_offsets]
        self.side_bytes = int(sum(int(x.sum().item()) for x in lens)) * self.elem_width

    def encode(self):
        self.S.serialize(self.gs, self.recs, self.n, string_base=self.sbase,
                         list_base=self.lbase, out=self.wire, offsets=self.offs, sync=False)

    def decode(self):
        self.S.deserialize(self.gs, self.wire, self.n, offsets=self.offs, records=self.back,
                           arena=self.arena, sync=False)

    def verify(self):
        import torch

        st, nd, consumed = self.S.context().wait()
        if st.code or consumed != self.wire_bytes or nd != self.n:
            raise RuntimeError("decode failed: %s" % (st.as_tuple(),))
        rs = self.record_bytes
        a, b = self.recs.view(self.n, rs), self.back.view(self.n, rs)
        for lo, hi in self.fixed_ranges:
            if not torch.equal(a[:, lo:hi], b[:, lo:hi]):
                raise RuntimeError("round trip mismatch in bytes %d..%d" % (lo, hi))
        # decoded strings are views into the wire; decoded list elements live
        # in the arena: re-encoding from those must give the same stream
        again = torch.empty_like(self.wire)
        offs2 = torch.empty_like(self.offs)
        self.S.serialize(self.gs, self.back, self.n,
                         string_base=self.wire if self.schema == "mixed" else None,
                         list_base=self.arena if self.schema == "nested" else None,
                         out=again, offsets=offs2, sync=True)
        if not torch.equal(again, self.wire) or not torch.equal(offs2, self.offs):
            raise RuntimeError("re-encode of the decoded batch differs from the wire stream")
        del again, offs2

    def algorithmic(self):
        # decode: read the wire + write the records (+ list elements to the
        # arena; strings are views into the wire); encode: read the records
        # and the string/list payloads + write the wire. The record index
        # (8 B/record) is bookkeeping, not counted.
        arena = self.side_bytes if self.schema == "nested" else 0
        return (self.wire_bytes + self.n * self.record_bytes + arena,
                self.n * self.record_bytes + self.side_bytes + self.wire_bytes)


class Mixed(VarLen):
    config_id = 3
    name = "config 3: Compact protocol, {4 x i32, 2 x string[0..32]} records, indexed encode+decode"
    schema, protocol = "mixed", 2
    default_records = 1 << 26
    dec_kernel, enc_kernel = "program_decode_kernel", "program_write_kernel"
    jit_decode = "tgpu_jit_decode"
    index_kernel = "index_tile_spec_kernel"
    fixed_ranges = [(0, 16), (48, 54)]
    span_offsets, elem_width = (16, 32), 1


class Nested(VarLen):
    config_id = 4
    name = "config 4: Binary protocol, {i64, list<i32>[0..16], inner{3 x double}}, indexed encode+decode"
    schema, protocol = "nested", 0
    default_records = 1 << 25
    dec_kernel, enc_kernel = "program_decode_kernel", "program_write_kernel"
    # records built in registers: the LDS record tile would hold its tiles
    # to 3 workgroups per CU (k_program.hip launch_program_decode)
    jit_decode = "tgpu_jit_decode_rr"
    fixed_ranges = [(0, 8), (24, 51), (56, 59)]
    span_offsets, elem_width = (8,), 4


class FileShards(Mixed):
    """Config 5: one Compact file of {4 x i32, 2 x string} records, split by
    BYTES across the ranks (64 Mi records encoded per rank, weak scaling).

    Step: every rank encodes its 64 Mi records (its part of the file, in file
    order); the file's byte ranges are redistributed so rank k holds
    [B_k, B_{k+1} + overlap) (all_to_all over RCCL; nothing at N=1); rank k
    indexes and decodes its range in one call (tgpu_decode_stream,
    speculative: rank 0 from the file's first byte) and confirms its first
    record start against rank k-1's last end (fbthrift_amd/shard.py:
    all-gather of 5 int64 per rank, redone on disagreement). Checked after warm-up: per-rank record counts sum to the file's,
    every decoded record equals the generator's record of the same global
    index, and re-encoding the decoded records reproduces the range's bytes.
    """
    config_id = 5
    parallelism = ("dp%d (one file split by bytes: all_to_all_single of the byte ranges + "
                   "all_gather of the range boundaries)")
    name = ("config 5: Compact protocol, {4 x i32, 2 x string[0..32]} file split by bytes "
            "across GPUs, encode + boundary discovery + decode")
    # bytes of the next rank's range each rank also holds: the longest record
    # of the file (a record starting before B_{k+1} ends by B_{k+1} + it),
    # found at setup from every rank's record index, at least min_overlap
    min_overlap = 4096

    def __init__(self, n, rank, dev):
        super().__init__(n, rank, dev)
        # the decode call (tgpu_decode_stream): round 6, one pass — the
        # speculation, the look-back and the record decode in one kernel
        # (tgpu_jit_index_onepass_rr); TGPU_INDEX_ONEPASS=0 keeps the two
        # passes (the index speculation, the copy of its stored record starts,
        # the indexed program decode)
        two = os.environ.get("TGPU_INDEX_ONEPASS", "") in ("0", "1")
        self.dec_kernel = ("tgpu_jit_index_onepass_rr" if not two and
                           self.dec_kernel.startswith("tgpu_jit")
                           else "tgpu_jit_index_spec+index_starts_copy_kernel+tgpu_jit_decode"
                           if self.dec_kernel.startswith("tgpu_jit")
                           else "index_tile_spec_kernel+index_starts_copy_kernel+"
                                "program_decode_kernel")
        self.setup_file(rank, dev)

    def setup_file(self, rank, dev):
        """The file layout every rank agrees on: each rank's encode output is
        the file's next `wire_bytes` bytes (ranks in order); rank k owns the
        bytes [B_k, B_k+1) and holds need_range(k) after the redistribution."""
        import torch

        from fbthrift_amd import shard

        self.rank, self.dev = rank, dev
        self.world = self.world_size()
        self.enc = self.wire  # this rank's part of the file (in file order)
        self.enc_offs = self.offs
        longest = self.longest_record()
        sizes = self._gather([self.wire_bytes, longest])
        self.overlap = max(self.min_overlap, max(r[1] for r in sizes))
        self.file_off = sum(r[0] for r in sizes[:rank])
        self.file_len = sum(r[0] for r in sizes)
        self.total_wire_bytes = self.file_len
        self.ranges = shard.byte_ranges(self.file_len, self.world)
        self.enc_ranges = []
        off = 0
        for r in sizes:
            self.enc_ranges.append((off, off + r[0]))
            off += r[0]
        self.need = shard.need_range(self.ranges, self.overlap, self.file_len, rank)
        # N=1: the file is this rank's encode output itself
        self.buf = self.wire if self.world == 1 else torch.empty(
            self.need[1] - self.need[0] + 16, dtype=torch.uint8, device=dev)
        self.idx = torch.empty(self.n * 2 + 2, dtype=torch.int64, device=dev)
        self.back = torch.empty(self.n * 2 * self.record_bytes, dtype=torch.uint8, device=dev)
        self.n_local = 0

    def longest_record(self):
        """Longest record of this rank's encode output (its record index)."""
        o = self.enc_offs if getattr(self, "enc_offs", None) is not None else self.offs
        return int((o[1:] - o[:-1]).max().item()) if self.n else 0

    def index_range(self, local, begin, end, speculative):
        """Record starts + records of the records that start in
        [begin, end) of `local` (this rank's held bytes): one
        tgpu_decode_stream call. Returns (n, first, last, status)."""
        recs, _, _, n, first, last, st = self.S.decode_stream(
            self.gs, local, begin=begin, end=end, speculative=speculative,
            max_records=self.idx.numel() - 1, offsets=self.idx, records=self.back)
        return n, first, last, st

    def expected_records(self, base, n):
        """The generator's records [base, base + n) in the record layout (for
        verify)."""
        import ctypes

        import torch

        import datagen

        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libtgpu_datagen.so"))
        want = torch.empty(n * self.record_bytes, dtype=torch.uint8, device=self.dev)
        side = torch.empty(n * 64, dtype=torch.uint8, device=self.dev)
        if lib.tgpu_gen_mixed(ctypes.c_uint64(datagen.SEED), ctypes.c_uint64(base),
                              ctypes.c_uint64(n), ctypes.c_void_p(want.data_ptr()),
                              ctypes.c_void_p(side.data_ptr()),
                              ctypes.c_void_p(self.stream.cuda_stream)):
            raise RuntimeError("generator failed")
        return want

    def reencode(self, records, n, local):
        """Re-encodes decoded records whose strings view `local`."""
        again, _ = self.S.serialize(self.gs, records, n, string_base=local)
        return again

    # ---- collectives ---------------------------------------------------------
    def _gather(self, vals):
        import torch.distributed as dist

        from fbthrift_amd import shard

        return shard.tensor_gather(dist.all_gather, self.dev, self.world_size())(vals)

    @staticmethod
    def world_size():
        import torch.distributed as dist

        return dist.get_world_size() if dist.is_initialized() else 1

    def redistribute(self):
        """File bytes [need) of every rank from the ranks that encoded them."""
        import torch.distributed as dist

        from fbthrift_amd import shard

        if self.world == 1:
            return
        shard.redistribute(self.wire, self.enc_ranges, self.ranges, self.overlap, self.file_len,
                           self.rank, self.buf, dist.all_to_all_single)

    def decode(self):
        from fbthrift_amd import shard

        self.redistribute()
        lo, hi = self.need
        b, e = self.ranges[self.rank]
        local = self.buf[: hi - lo]
        cap = self.idx.numel() - 1
        self.status = None

        def index_fn(begin, speculative):
            # index + decode of the records that start in [begin, e); a re-run
            # after the exchange replaces them
            n, first, last, st = self.index_range(local, begin - lo, e - lo, speculative)
            self.status = st
            if n == 0:
                return 0, shard.NONE, shard.NONE
            return n, first + lo, last + lo

        n, first, last, base, rounds = shard.exchange_boundaries(
            index_fn, self.rank, self.world, b, e, self._gather)
        self.n_local, self.first, self.last, self.base, self.rounds = n, first, last, base, rounds

    def check_timed(self):
        if self.n_local and (self.status is None or self.status.code):
            raise RuntimeError("timed decode failed: %s" % (
                self.status.as_tuple() if self.status is not None else None,))

    def verify(self):
        import torch

        self.check_timed()
        counts = self._gather([self.n_local])
        total = sum(c[0] for c in counts)
        if total != self.n * self.world:
            raise RuntimeError("records found %d != %d" % (total, self.n * self.world))
        n, rs = self.n_local, self.record_bytes
        if n == 0:
            return
        want = self.expected_records(self.base, n)
        a, b = want.view(n, rs), self.back[: n * rs].view(n, rs)
        for lo, hi in self.fixed_ranges:
            if not torch.equal(a[:, lo:hi], b[:, lo:hi]):
                raise RuntimeError("decoded records differ from the generator's")
        lo = self.need[0]
        local = self.buf[: self.need[1] - lo]
        again = self.reencode(self.back[: n * rs], n, local)
        if not torch.equal(again, local[self.first - lo: self.last - lo]):
            raise RuntimeError("re-encoded records differ from the file's bytes")
        del want, again

    def algorithmic(self):
        # per rank, per step: encode as config 3; decode (index + records in
        # one call) must read its range once and write the records (the
        # speculation pass's second read is overhead, not algorithmic)
        dec_bytes = (self.last - self.first) + self.n_local * self.record_bytes
        return dec_bytes, self.n * self.record_bytes + self.side_bytes + self.wire_bytes


WORKLOADS = {2: Flat8, 3: Mixed, 4: Nested, 5: FileShards}


class CudaRuntime:
    """Where the ranks run: one process per MI355X, RCCL (torch's "nccl"
    backend) for the barrier, the max-over-ranks timing and config 5's
    exchange; HIP events on the launch stream."""
    backend = "nccl"

    def setup(self, local):
        import torch

        # ranks beyond the visible GPUs share them round-robin (only with
        # --backend gloo: a one-GPU rehearsal of the multi-rank path)
        local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        return torch.device("cuda", local)

    def init_group(self, dev):
        import torch.distributed as dist

        if self.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(self.backend)

    def sync(self):
        import torch

        torch.cuda.synchronize()

    def event(self):
        import torch

        return torch.cuda.Event(enable_timing=True)


RUNTIME = CudaRuntime()


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`--gpus N` without a launcher: start N ranks (one per GPU) with
    torch.distributed.run on 127.0.0.1 as a CHILD process, re-running this
    same script (sys.argv[0]) with the same arguments, and return its exit
    code. Called before anything touches the GPU; the parent never does."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % n, "--master-addr=127.0.0.1",
           "--master-port=%d" % _free_port(), os.path.abspath(sys.argv[0])] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def resolve_world(gpus):
    """(world, rank, local_rank) from the launcher's environment, checked
    against --gpus; (None, None, None) when this process must launch the
    ranks itself."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if gpus is not None and gpus > 1:
            return None, None, None
        return 1, 0, 0
    world = int(env_world)
    if gpus is not None and gpus != world:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (gpus, world))
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher (no WORLD_SIZE) N > 1 "
                         "starts N ranks with torch.distributed.run")
    ap.add_argument("--backend", default=None, choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (default nccl = RCCL over xGMI; "
                         "gloo lets N ranks share one GPU to rehearse the multi-rank path)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=[1] + sorted(WORKLOADS))
    ap.add_argument("--records", type=int, default=0, help="records per GPU (default: config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-copy-ceiling", action="store_true")
    ap.add_argument("--host-start", action="store_true",
                    help="also time pinned-host -> decode -> host and host -> encode -> host")
    ap.add_argument("--skim", action="store_true",
                    help="also time the schemaless skim of the workload's indexed stream "
                         "(tgpu_skim_batch)")
    ap.add_argument("--irregular", action="store_true",
                    help="config 2 only: also time decodes of streams that leave the canonical "
                         "form (first record reordered; every record with an extra unknown "
                         "field) against the indexed program decode")
    ap.add_argument("--nested", action="store_true",
                    help="also time a nested-container workload (list<struct>, "
                         "list<list<i32>>; Binary; general kernels) encode + decode")
    ap.add_argument("--transcode", action="store_true",
                    help="also time device transcoding of the workload's stream into the "
                         "other protocol (tgpu_transcode_batch)")
    ap.add_argument("--host-batch", action="store_true",
                    help="also time the IOBuf batch API (deserializeBatch / serializeBatch "
                         "into std:: objects, tests/cpp/host_batch_bench) for configs 3/4")
    args = ap.parse_args(argv)
    if args.config == 1:
        print(json.dumps(config1()), flush=True)
        return 0

    world, rank, local = resolve_world(args.gpus)
    if world is None:
        return launch_ranks(args.gpus)

    import torch
    import torch.distributed as dist

    rt = RUNTIME
    if args.backend:
        rt.backend = args.backend
    dev = rt.setup(local)
    if world > 1:
        rt.init_group(dev)

    W = WORKLOADS[args.config]
    n = args.records or W.default_records
    wl = W(n, rank, dev)

    for _ in range(args.warmup):
        wl.encode()
        wl.decode()
    rt.sync()
    wl.verify()

    evs = [[rt.event() for _ in range(4)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    rt.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        wl.timed_step(evs[k])
    rt.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    wl.check_timed()
    enc_ms = [e[0].elapsed_time(e[1]) for e in evs]
    dec_ms = [e[3 if TRACE_MARKS else 1].elapsed_time(e[2]) for e in evs]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    job_bytes = wl.total_wire_bytes or wl.wire_bytes * world
    value = 2.0 * job_bytes * args.steps / elapsed / 2**30
    dec_avg = sum(dec_ms) / len(dec_ms) / 1e3
    enc_avg = sum(enc_ms) / len(enc_ms) / 1e3
    dec_alg, enc_alg = wl.algorithmic()
    traffic, traffic_src = pmc_traffic(wl.dec_kernel, n, args.config)
    enc_traffic, _ = pmc_traffic(wl.enc_kernel, n, args.config)
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: splitmix64(seed 0x1729) records per tests/golden/datagen.py, "
                "generated on device",
        "config": {"workload": wl.name, "records_per_gpu": n, "records_total": n * world, "wire_bytes_per_gpu": wl.wire_bytes,
                   "record_bytes": wl.record_bytes,
                   "wire_bytes_per_record": round(wl.wire_bytes / n, 3),
                   "parallelism": wl.parallelism % world,
                   **({"overlap_bytes": wl.overlap} if hasattr(wl, "overlap") else {})},
        "roofline": {"bound": "hbm", "kernel": wl.dec_kernel,
                     "achieved": round(dec_alg / dec_avg / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(dec_alg / dec_avg / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": dec_alg,
                     "avg_launch_ms": round(dec_avg * 1e3, 4),
                     "timing": "HIP events on the launch stream around the whole decode call "
                               "(main kernel + small bookkeeping kernels)",
                     "copy_ceiling": None if args.no_copy_ceiling else copy_ceiling(dev),
                     "encode": {"kernel": wl.enc_kernel,
                                "achieved": round(enc_alg / enc_avg / 1e9, 1),
                                "frac": round(enc_alg / enc_avg / 1e9 / HBM_PEAK_GBS, 4),
                                "algorithmic_bytes_per_launch": enc_alg,
                                "traffic": enc_traffic,
                                "avg_launch_ms": round(enc_avg * 1e3, 4)}},
    }
    if args.host_start and rank == 0:
        line["host_start"] = host_start(wl, dev)
    if args.transcode and rank == 0:
        line["transcode"] = transcode(wl, dev)
    if args.skim and rank == 0:
        line["skim"] = skim(wl, dev)
    if args.irregular and rank == 0 and args.config == 2:
        line["irregular"] = irregular(wl, dev)
    if args.nested and rank == 0:
        del wl
        torch.cuda.empty_cache()
        line["nested"] = nested(dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(wl)
    if args.host_batch and rank == 0:
        line["host_batch"] = host_batch(wl)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


# Config 4's shape with containers of structs and of containers (the nested
# golden cases' types, tests/golden/nestgen.py): Record {1: i64 id;
# 2: list<Item> items[0..8]; 3: list<list<i32>> grid[0..3][0..7]},
# Item {1: i32 a; 2: i64 b; 3: double c}.
T_I32_, T_I64_, T_DOUBLE_, T_LIST_, T_STRUCT_ = 8, 10, 4, 15, 12
NESTED_TABLE = [
    [[1, T_I64_, 0, 0, -1], [2, T_LIST_, T_STRUCT_, 0, 1],
     [3, T_LIST_, T_LIST_, 0, -1, 0, [T_LIST_, T_I32_, 0, -1]]],
    [[1, T_I32_, 0, 0, -1], [2, T_I64_, 0, 0, -1], [3, T_DOUBLE_, 0, 0, -1]],
]


def nested_batch(dev, n, seed=0x1729):
    """n records of NESTED_TABLE generated on the device (torch, seeded):
    (schema, records, list base, items, grid rows, i32 elements). The list
    base holds the Item arrays, the grid's row spans and the rows' i32
    arrays."""
    import torch

    from fbthrift_amd.schema import Schema

    schema = Schema.from_table(NESTED_TABLE)
    by_name = {st.name: k for k, st in enumerate(schema.structs)}
    r0, r1 = by_name["S0"], by_name["S1"]
    S, IS = schema.size[r0], schema.size[r1]
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    ni = torch.randint(0, 9, (n,), device=dev, generator=g)
    ng = torch.randint(0, 4, (n,), device=dev, generator=g)
    rows = int(ng.sum().item())
    rl = torch.randint(0, 8, (rows,), device=dev, generator=g)
    items = int(ni.sum().item())

    def excl(x):
        c = torch.cumsum(x, 0)
        return c - x

    rl8 = (rl * 4 + 7) // 8 * 8  # each row's i32 array 8-byte aligned
    items_base = 0
    outer_base = (items * IS + 15) // 16 * 16
    inner_base = outer_base + rows * 16
    total = inner_base + int(rl8.sum().item()) + 16
    lbase = torch.zeros(total, dtype=torch.uint8, device=dev)
    # Items
    it = lbase[: items * IS].view(items, IS)
    mo = lambda si, k: schema.member[(si, k)]
    io = lambda si, k: schema.isset[(si, k)]
    it.view(torch.int32).view(items, IS // 4)[:, mo(r1, 0) // 4] = torch.randint(
        -2**31, 2**31 - 1, (items,), device=dev, generator=g, dtype=torch.int32)
    it.view(torch.int64).view(items, IS // 8)[:, mo(r1, 1) // 8] = torch.randint(
        -2**62, 2**62, (items,), device=dev, generator=g, dtype=torch.int64)
    it.view(torch.float64).view(items, IS // 8)[:, mo(r1, 2) // 8] = torch.randn(
        items, device=dev, generator=g, dtype=torch.float64)
    for k in range(3):
        it[:, io(r1, k)] = 1
    # grid rows: spans into the i32 arrays
    outer = lbase[outer_base: outer_base + rows * 16].view(torch.int64).view(rows, 2)
    outer[:, 0] = inner_base + excl(rl8)
    outer[:, 1] = rl
    nints = int(rl8.sum().item()) // 4
    lbase[inner_base: inner_base + nints * 4].view(torch.int32)[:] = torch.randint(
        -2**31, 2**31 - 1, (nints,), device=dev, generator=g, dtype=torch.int32)
    # records
    recs = torch.zeros(n * S, dtype=torch.uint8, device=dev)
    rv = recs.view(n, S)
    rv.view(torch.int64).view(n, S // 8)[:, mo(r0, 0) // 8] = torch.arange(n, device=dev) * 7919
    sp = rv.view(torch.int64).view(n, S // 8)
    sp[:, mo(r0, 1) // 8] = items_base + excl(ni) * IS
    sp[:, mo(r0, 1) // 8 + 1] = ni
    sp[:, mo(r0, 2) // 8] = outer_base + excl(ng) * 16
    sp[:, mo(r0, 2) // 8 + 1] = ng
    for k in range(3):
        rv[:, io(r0, k)] = 1
    return schema, recs, lbase, items, rows, int(rl.sum().item())


def nested(dev, n=1 << 24, reps=5, seed=0x1729):
    """Nested containers on the device (the general reader / writer's frame
    machines, per-record arena regions): n records generated on the device
    (torch, seeded), encoded from a list base holding the Item arrays, the
    grid's row spans and the rows' i32 arrays, then decoded from the indexed
    stream. Timed with HIP events around each call (best of `reps`); checked
    by re-encoding the decoded records (their spans now index the decode's
    arena) to the same bytes. Rates are wire GiB/s; the rooflines price the
    algorithmic bytes (wire + records + element arrays) against HBM."""
    import torch

    from fbthrift_amd import serializer as SZ

    schema, recs, lbase, items, rows, nints = nested_batch(dev, n, seed)
    S, IS = schema.size[0], schema.size[1]
    gs = SZ.GpuSchema(schema)
    Ser = SZ.BinarySerializer
    Ser.context().reserve(n)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    _, wire_bytes = Ser.encoded_size(gs, recs, n, offs, list_base=lbase)
    wire = torch.empty(wire_bytes + 16, dtype=torch.uint8, device=dev)
    cap = Ser.arena_bytes(gs, wire_bytes)
    arena = torch.empty(cap + 16, dtype=torch.uint8, device=dev)
    back = torch.empty(n * S, dtype=torch.uint8, device=dev)

    def best(fn):
        t = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1))
        return min(t[1:])

    enc_ms = best(lambda: Ser.serialize(gs, recs, n, list_base=lbase, out=wire, offsets=offs,
                                        sync=False))
    dec_ms = best(lambda: Ser.deserialize(gs, wire[:wire_bytes], n, offsets=offs, records=back,
                                          arena=arena, sync=False))
    st, nd, consumed = Ser.context().wait()
    if st.code or nd != n or consumed != wire_bytes:
        raise RuntimeError("nested decode failed: %s" % (st.as_tuple(),))
    again = torch.empty_like(wire)
    w2, _ = Ser.serialize(gs, back, n, list_base=arena, out=again, offsets=None)
    if w2.numel() != wire_bytes or not torch.equal(w2, wire[:wire_bytes]):
        raise RuntimeError("nested re-encode differs")
    elem = items * IS + rows * 16 + nints * 4
    alg = wire_bytes + n * S + elem  # either direction: wire + records + element arrays
    gib = wire_bytes / 2**30
    return {"records": n, "wire_bytes": wire_bytes, "record_bytes": S,
            "item_bytes": IS, "items": items, "grid_rows": rows,
            "encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3),
            "encode_GiBps": round(gib / enc_ms * 1e3, 1),
            "decode_GiBps": round(gib / dec_ms * 1e3, 1),
            "encode_plus_decode_GiBps": round(2 * gib / (enc_ms + dec_ms) * 1e3, 1),
            "roofline": {"bound": "hbm", "algorithmic_bytes_per_call": alg,
                         "decode_traffic": pmc_traffic("tgpu_jit_ndecode", n, 4, True)[0],
                         "encode_traffic": pmc_traffic("tgpu_jit_nsize+tgpu_jit_nwrite", n, 4,
                                                       True)[0],
                         "decode_achieved_GBps": round(alg / dec_ms / 1e6, 1),
                         "decode_frac": round(alg / dec_ms / 1e6 / HBM_PEAK_GBS, 4),
                         "encode_achieved_GBps": round(alg / enc_ms / 1e6, 1),
                         "encode_frac": round(alg / enc_ms / 1e6 / HBM_PEAK_GBS, 4),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s"},
            "kernels": "decode: tgpu_jit_ndecode (the nested program, one loop per "
                       "container level) + the general decoder for records it leaves; "
                       "encode: tgpu_jit_nsize -> scan_tiles_* -> tgpu_jit_nwrite (the "
                       "nested program's size and write passes)"}


def irregular(wl, dev, reps=3):
    """Config 2 streams the fixed-layout kernels cannot take whole (the
    reference reads them like any other stream): (i) the first record's
    fields 1 and 2 swapped, (ii) every record carrying an extra unknown i32
    field (a newer writer's schema; 96 bytes per record). Blocking decodes
    (tgpu_decode_batch: plan kernel, then the parallel index + decode of the
    tail) and stream-ordered ones (no host status: the strided tail decode,
    then the finish kernel), timed with HIP events around the call, each
    checked against the records; reported beside the indexed program decode
    of the canonical stream (offsets given) and the plan decode."""
    import torch

    n, L = wl.n, wl.L
    canon = wl.wire[: n * L]
    offs = torch.arange(n + 1, dtype=torch.int64, device=dev) * L
    first = canon.clone()
    first[0:11], first[11:22] = canon[11:22].clone(), canon[0:11].clone()
    ex = torch.empty((n, 96), dtype=torch.uint8, device=dev)
    c2 = canon.view(n, L)
    ex[:, :88] = c2[:, :88]
    ex[:, 88] = 8
    ex[:, 89] = 0
    ex[:, 90] = 20
    ex[:, 91:95] = c2[:, 3:7]
    ex[:, 95] = 0
    every = ex.view(-1)
    res = {"records": n}

    def timed(name, wire, offsets=None, sync=True):
        print("irregular %s: start" % name, file=sys.stderr, flush=True)
        best = None
        for _ in range(reps + 1):
            wl.back.zero_()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            if sync:
                _, _, consumed = wl.S.deserialize(wl.gs, wire, n, offsets=offsets, records=wl.back)
            else:  # stream-ordered: no host status inside the call
                wl.S.deserialize(wl.gs, wire, n, offsets=offsets, records=wl.back, sync=False)
            e1.record()
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            ms = e0.elapsed_time(e1)
            if not sync:
                st, _, consumed = wl.S.context().wait()
                if st.code:
                    raise RuntimeError("irregular decode %s: %s" % (name, st.as_tuple()))
            if consumed != wire.numel() or not torch.equal(wl.back, wl.recs):
                raise RuntimeError("irregular decode %s differs" % name)
            if best is None or ms < best[0]:
                best = (ms, wall * 1e3)
        res[name] = {"ms": round(best[0], 3), "wall_ms": round(best[1], 3),
                     "wire_GiBps": round(wire.numel() / best[0] * 1e3 / 2**30, 1)}
        print("irregular %s: %s" % (name, res[name]), file=sys.stderr, flush=True)

    timed("plan_decode_canonical", canon)
    timed("indexed_program_decode_canonical", canon, offs)
    timed("first_record_reordered", first)
    timed("every_record_extra_field", every)
    timed("async_plan_decode_canonical", canon, sync=False)
    timed("async_first_record_reordered", first, sync=False)
    timed("async_every_record_extra_field", every, sync=False)
    base = res["indexed_program_decode_canonical"]["ms"]
    for k in ("first_record_reordered", "every_record_extra_field",
              "async_first_record_reordered", "async_every_record_extra_field"):
        res[k]["x_indexed_program_decode"] = round(res[k]["ms"] / base, 2)
    del first, ex, every, offs
    return res


def config1(n=1000, seconds=3.0):
    """BASELINE config 1 ("thrift/perf"): Binary round trip of 1k flat
    {8 x i64} records on the CPU — the shape of the reference's protocol
    microbenchmarks (ThriftProtocolBenchmarks.cpp:167-219: serialize and
    deserialize of one struct, ns/op) with the oracle's codegen-equivalent
    T::write / T::readNoXfer on one core, values of config 2's generator.
    The same 1k batch also goes through the C-ABI on the GPU (plumbing: a
    1k-record call is launch-latency bound), checked byte for byte."""
    import numpy as np

    from oracle import oracle

    L = oracle.lib()
    recs = np.zeros(n * 72, np.uint8)
    L.oracle_gen_flat8(SEED, 0, n, recs.ctypes.data)
    wire = np.zeros(n * 89, np.uint8)
    back = np.zeros(n * 72, np.uint8)
    t_enc, reps_e = _timed(lambda: L.oracle_flat8_binary_encode(recs.ctypes.data, n,
                                                                wire.ctypes.data, 1), seconds)
    t_dec, reps_d = _timed(lambda: L.oracle_flat8_binary_decode(wire.ctypes.data, n,
                                                                back.ctypes.data, 1), seconds)
    assert np.array_equal(back, recs)
    line = {"metric": "CPU Binary round trip, 1k flat {8 x i64} records (config 1)",
            "value": round((t_enc + t_dec) / n * 1e9, 2), "unit": "ns/record",
            "higher_is_better": False, "dtype": "u8", "data": "synthetic (config 2 generator)",
            "config": {"workload": "config 1: thrift/perf-style CPU round trip, 1000 x flat8",
                       "records": n, "wire_bytes_per_record": 89},
            "encode_ns_per_record": round(t_enc / n * 1e9, 2),
            "decode_ns_per_record": round(t_dec / n * 1e9, 2),
            "cores": 1, "kind": "port", "reps": reps_e + reps_d}
    try:
        import torch

        if torch.cuda.is_available():
            from fbthrift_amd.schema import Schema
            from fbthrift_amd.serializer import BinarySerializer as BS, GpuSchema
            import datagen

            dev = torch.device("cuda", 0)
            gs = GpuSchema(Schema.from_table(datagen.SCHEMAS["flat8"]))
            r = torch.from_numpy(recs).to(dev)

            def gpu_round_trip():
                w, _ = BS.serialize(gs, r, n, offsets=None)
                out, _, _ = BS.deserialize(gs, w, n)
                return w, out

            w, out = gpu_round_trip()
            assert np.array_equal(w.cpu().numpy(), wire) and np.array_equal(out.cpu().numpy(), recs)
            t_gpu, reps_g = _timed(gpu_round_trip, 1.0)
            line["gpu_plumbing"] = {"us_per_round_trip_call": round(t_gpu * 1e6, 2),
                                    "ns_per_record": round(t_gpu / n * 1e9, 2),
                                    "how": "tgpu_encode_batch + tgpu_decode_batch, blocking, "
                                           "device-resident 1k batch", "reps": reps_g}
    except Exception as e:  # a CPU-only host: the CPU line stands alone
        line["gpu_plumbing"] = {"skipped": str(e)[:200]}
    return line


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


def pmc_summary(config, nested=False, root=None):
    """The committed rocprofv3 PMC summary for this tree's kernels:
    profiles/r<NN>/pmc/pmc_c<config>.json (pmc_nested.json for the nested
    leg), newest round first, written by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes (gfx950 FETCH x2 correction calibrated on a
    1 GiB copy). Only a summary stamped with the current kernel-source hash
    (tools/srchash.py) counts: counters of other kernels are refused.
    Returns (summary or None, note)."""
    import glob

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from srchash import source_hash

    root = root or ROOT
    want = source_hash(root)
    name = "pmc_nested.json" if nested else "pmc_c%d.json" % config
    stale = []
    for path in sorted(glob.glob(os.path.join(root, "profiles", "r[0-9]*", "pmc", name)),
                       reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        rel = os.path.relpath(path, root)
        if d.get("source_hash") == want:
            return d, rel
        stale.append("%s (sources %s)" % (rel, d.get("source_hash")))
    return None, ("no PMC summary of kernel sources %s; stale: %s"
                  % (want, ", ".join(stale) or "none"))


def pmc_traffic(kernel, n, config=2, nested=False, root=None):
    """HBM bytes per launch of `kernel` (the kernels of one call joined by
    '+': their sum) from pmc_summary(), scaled to this launch's record count;
    (None, why) when no summary of the current kernels has it."""
    d, note = pmc_summary(config, nested, root)
    if d is None:
        return None, note
    try:
        return int(sum(d[k]["hbm_bytes_per_record"] for k in kernel.split("+")) * n), note
    except KeyError as e:
        return None, "%s: no counters for %s" % (note, e)


def transcode(wl, dev, reps=5):
    """Device-resident Binary <-> Compact transcoding of the workload's whole
    stream (tgpu_transcode_batch), in both forms: wire to wire without
    records in HBM (tgpu_xcode.h: size pass, scan, write pass over the source
    tile in LDS — schemas with a flat program in both protocols) and the
    composed decode into an HBM workspace + re-encode (TGPU_XCODE=0); each
    with the record index given (the workload's offsets) and without (the
    stream index first). Blocking calls (host status), best of `reps`; rate =
    input wire bytes / time. Checked: every form's bytes equal, and
    transcoding back gives the original stream. Secondary line, never
    `value`."""
    import torch

    from fbthrift_amd import serializer as S

    if isinstance(wl, FileShards):
        return {"skipped": "config 5 is config 3's stream split by bytes; see config 3"}
    src = wl.S
    to = 2 if src.protocol == 0 else 0
    dst = S.CompactSerializer if to == 2 else S.BinarySerializer
    w = wl.wire[: wl.wire_bytes]
    out = torch.empty(8 * wl.wire_bytes + 16, dtype=torch.uint8, device=dev)
    res = {"from": src.protocol, "to": to}
    ref = None
    # (config 2's fixed-layout stream has no offsets array: record i at i * L;
    # unindexed, its transcoding stays on the plan decode + encode by design)
    wl_offs = getattr(wl, "offs", None)
    if wl_offs is None:
        wl_offs = torch.arange(wl.n + 1, dtype=torch.int64, device=dev) * (wl.wire_bytes // wl.n)
    old = os.environ.get("TGPU_XCODE")
    try:
        for form in ("fused", "composed"):
            os.environ["TGPU_XCODE"] = "1" if form == "fused" else "0"
            for ix in ("indexed", "unindexed"):
                offs = wl_offs if ix == "indexed" else None
                best = None
                for _ in range(reps + 1):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    _, _, st, done, size = src.transcode(wl.gs, w, wl.n, to, offsets=offs, out=out,
                                                         want_offsets=False)
                    el = time.perf_counter() - t0
                    if st.code or done != wl.n:
                        raise RuntimeError("transcode failed: %s" % (st.as_tuple(),))
                    best = el if best is None else min(best, el)
                got = out[:size].clone()
                if ref is None:
                    ref = got
                elif not torch.equal(ref, got):
                    raise RuntimeError("transcode forms disagree (%s %s)" % (form, ix))
                res["%s_%s_ms" % (form, ix)] = round(best * 1e3, 3)
                res["%s_%s_gibps_in" % (form, ix)] = round(wl.wire_bytes / best / 2**30, 3)
    finally:
        if old is None:
            os.environ.pop("TGPU_XCODE", None)
        else:
            os.environ["TGPU_XCODE"] = old
    size = ref.numel()
    out[:size].copy_(ref)
    back = torch.empty(wl.wire_bytes + 16, dtype=torch.uint8, device=dev)
    _, _, st, done, bsize = dst.transcode(wl.gs, out[:size], wl.n, src.protocol, out=back)
    if st.code or bsize != wl.wire_bytes or not torch.equal(back[:bsize], w):
        raise RuntimeError("transcode round trip mismatch")
    res["out_bytes"] = size
    res["how"] = ("blocking calls (host status), best of %d; fused = wire to wire, no records "
                  "in HBM; composed = decode + encode (TGPU_XCODE=0); indexed = the workload's "
                  "offsets given, unindexed = the stream index first" % reps)
    return res


def skim(wl, dev, reps=10):
    """Schemaless skim (tgpu_skim_batch) of the workload's encoded stream with
    its record index: per record, one 16-byte entry per top-level field —
    and, for a schema with a struct-valued field (config 4), the nested skim
    (tgpu_skim_batch_ex, one level: the struct's fields too). Algorithmic
    bytes = wire + index (8 B/record) read + entries (16 B/field) + counts
    (4 B/record) written. HIP events on the launch stream. Checked against
    the oracle on a sample of records. Secondary line, never `value`."""
    import numpy as np
    import torch

    from fbthrift_amd import serializer as S
    from oracle import oracle

    if isinstance(wl, FileShards):
        return {"skipped": "config 5 is config 3's stream split by bytes; see config 3"}
    wl.encode()
    torch.cuda.synchronize()
    if hasattr(wl, "offs"):
        offs = wl.offs
    else:
        offs = torch.arange(wl.n + 1, dtype=torch.int64, device=dev) * wl.L
    w = wl.wire[: wl.wire_bytes]
    structs = wl.gs.schema.structs

    def run(nest):
        nf = len(structs[0].fields) + (sum(len(st.fields) for st in structs[1:]) if nest else 0)
        fields, counts, done, st = wl.S.skim(w, offs, wl.n, max_fields=nf, nest=nest)
        assert st.code == 0 and done == wl.n
        times = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            wl.S.skim(w, offs, wl.n, max_fields=nf, check=False, fields=fields, counts=counts,
                      nest=nest)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / 1e3)
        # oracle check on sampled records (rebased slices)
        rng = np.random.default_rng(7)
        oc = offs.cpu().numpy().astype(np.uint64)
        cnt = counts.cpu().numpy()
        fv = fields[: nf * wl.n * 16].view(nf, wl.n, 16)
        for i in rng.integers(0, wl.n, 64):
            a, b = int(oc[i]), int(oc[i + 1])
            raw = w[a:b].cpu().numpy()
            ost, ofl, ocnt, _ = oracle.skim(wl.S.protocol, raw, np.array([0, b - a], np.uint64),
                                            1, nf, nest=nest)
            g = S.skim_records(fv[:, i].contiguous().view(-1), 1, nf)
            k = int(ocnt[0])
            assert ost.code == 0 and cnt[i] == k
            for key in ("id", "flags", "length"):
                assert np.array_equal(g[0, :k][key], ofl[0, :k][key])
            assert np.array_equal(g[0, :k]["offset"] - a, ofl[0, :k]["offset"])
        t = float(np.median(times))
        alg = wl.wire_bytes + 8 * (wl.n + 1) + int(cnt.astype(np.int64).sum()) * 16 + 4 * wl.n
        return {"kernel": "skim_kernel", "nest": nest, "records": wl.n,
                "fields_per_record": round(float(cnt.mean()), 3), "ms": round(t * 1e3, 4),
                "gibps_wire": round(wl.wire_bytes / t / 2**30, 2),
                "achieved_GBps": round(alg / t / 1e9, 1),
                "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "algorithmic_bytes": alg,
                "timing": "HIP events around the call, median of %d" % reps,
                "check": "64 sampled records vs the oracle"}

    res = run(0)
    if len(structs) > 1:
        res["nested"] = run(1)
    return res


def host_batch(wl, records=1 << 22):
    """The drop-in caller's rate, never `value`:
    serializeBatch of codegen'd C++ objects (std::string / std::vector
    members) into an IOBufQueue and deserializeBatch of the IOBuf back into
    objects, through the C++ host mirror (include/thrift_gpu/
    GpuBatchSerializer.h: host materialization on up to 16 threads, the
    device pass pipelined over PCIe); beside it one core of a reader / writer
    in the generated code's shape. Configs 3 and 4 (tools/host_batch_bench,
    a child process)."""
    import json
    import subprocess

    cfg = getattr(wl, "config_id", None)
    if cfg not in (3, 4):
        return {"skipped": "configs 3 and 4 only"}
    exe = os.path.join(ROOT, "tools", "build", "host_batch_bench")
    if not os.path.exists(exe):
        raise RuntimeError("tools/build/host_batch_bench is not built (__graft_entry__.build())")
    r = subprocess.run([exe, str(cfg), str(records), "3"], capture_output=True, text=True,
                       timeout=600)
    if r.returncode:
        raise RuntimeError("host_batch_bench failed: %s" % r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def host_start(wl, dev):
    """Host-memory start/end rates (PCIe-inclusive), never
    `value`. Config 2 runs the library's host path (tgpu_encode_host /
    tgpu_decode_host: chunked, three streams overlapping H2D, kernels and D2H)
    from pinned and from pageable host buffers, and checks the round trip;
    the other configs time H2D + kernels + D2H serialized on one stream."""
    import numpy as np
    import torch

    res = {}
    if isinstance(wl, Flat8):
        n = wl.n
        h_recs = torch.empty(n * 72, dtype=torch.uint8, pin_memory=True)
        h_recs.copy_(wl.recs)
        h_wire = torch.empty(n * 89, dtype=torch.uint8, pin_memory=True)
        h_back = torch.empty(n * 72, dtype=torch.uint8, pin_memory=True)
        torch.cuda.synchronize()
        for kind in ("pinned", "pageable"):
            if kind == "pageable":
                h_recs = h_recs.numpy().copy()
                h_wire = np.empty(n * 89, np.uint8)
                h_back = np.empty(n * 72, np.uint8)
            for name in ("encode", "decode"):
                best = None
                for _ in range(3):
                    t0 = time.perf_counter()
                    if name == "encode":
                        _, st, size = wl.S.serialize_host(wl.gs, h_recs, n, h_wire)
                    else:
                        _, st, nd, size = wl.S.deserialize_host(wl.gs, h_wire, n, h_back)
                    el = time.perf_counter() - t0
                    if st.code or size != n * 89:
                        raise RuntimeError("host %s failed: %s" % (name, st.as_tuple()))
                    best = el if best is None else min(best, el)
                res["%s_%s_gibps" % (name, kind)] = round(n * 89 / best / 2**30, 3)
            back = torch.from_numpy(np.asarray(h_back)) if kind == "pageable" else h_back
            if not torch.equal(back.to(dev), wl.recs):
                raise RuntimeError("host round trip mismatch (%s)" % kind)
        res["how"] = "tgpu_encode_host / tgpu_decode_host, 4Mi-record chunks, 3 streams"
        return res
    h_wire = torch.empty(wl.wire.numel(), dtype=torch.uint8, pin_memory=True)
    h_recs = torch.empty(wl.recs.numel(), dtype=torch.uint8, pin_memory=True)
    h_back = torch.empty(wl.back.numel(), dtype=torch.uint8, pin_memory=True)
    h_wire.copy_(wl.wire)
    h_recs.copy_(wl.recs)
    torch.cuda.synchronize()
    if not wl.gs.has_lists and not isinstance(wl, FileShards):
        # tgpu_decode_host: unindexed host stream -> host records (one
        # resident pass: copy in, fused index + decode, copy out)
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            _, st, nd, cons = wl.S.deserialize_host(wl.gs, h_wire, wl.n, h_back)
            el = time.perf_counter() - t0
            if st.code or cons != wl.wire_bytes:
                raise RuntimeError("host decode failed: %s" % (st.as_tuple(),))
            best = el if best is None else min(best, el)
        res["decode_host_api_gibps"] = round(wl.wire_bytes / best / 2**30, 3)
    for name, fn in (("decode", lambda: (wl.wire.copy_(h_wire, non_blocking=True), wl.decode(),
                                        h_back.copy_(wl.back, non_blocking=True))),
                     ("encode", lambda: (wl.recs.copy_(h_recs, non_blocking=True), wl.encode(),
                                        h_wire.copy_(wl.wire, non_blocking=True)))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / 3
        res[name + "_gibps"] = round(wl.wire_bytes / el / 2**30, 3)
    res["how"] = "pinned buffers, H2D + kernels + D2H serialized on one stream"
    return res


if __name__ == "__main__":
    sys.exit(main())
