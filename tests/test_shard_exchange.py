"""Shard-boundary exchange for one file split by bytes across ranks
(fbthrift_amd/shard.py): the host logic of BASELINE config 5, run over a
fake indexer with a known record layout, on the CPU with gloo (world sizes 2
and 4) and as a pure function."""
import os
import socket

import numpy as np
import pytest

from fbthrift_amd import shard


def _layout(seed, n=5000, max_len=400, giant=50_000):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, max_len, n)
    # a few records longer than a whole range
    lens[n // 3] = giant
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)


class FakeIndex:
    """Record starts known exactly; speculation can be made to lie."""

    def __init__(self, starts, lie_ranks=(), rank=0):
        self.starts = starts
        self.lie = rank in lie_ranks

    def range(self, begin, end, speculative):
        s = self.starts[:-1]
        L = int(self.starts[-1])
        inside = s[(s >= begin) & (s < end)]
        if inside.size == 0:
            return 0, shard.NONE, shard.NONE
        first = int(inside[0])
        if speculative and self.lie and inside.size > 2:
            inside = inside[1:]  # speculation picked a false (later) start
            first = int(inside[0])
        k = np.searchsorted(self.starts, first)
        stop = np.searchsorted(self.starts, end)
        n = int(stop - k)
        last = int(self.starts[stop]) if stop < len(self.starts) else L
        return n, first, last


def _truth(starts, begins, ends):
    s = starts[:-1]
    out = []
    for b, e in zip(begins, ends):
        inside = s[(s >= b) & (s < e)]
        out.append(int(inside.size))
    return out


def test_resolve_pure():
    starts = _layout(1)
    L = int(starts[-1])
    world = 8
    ranges = shard.byte_ranges(L, world)
    fi = FakeIndex(starts)
    rows = [fi.range(b, e, k > 0) for k, (b, e) in enumerate(ranges)]
    confirmed, redo = shard.resolve([r[0] for r in ranges], [r[1] for r in ranges],
                                    [r[1] for r in rows], [r[2] for r in rows])
    assert redo == []
    # a lying rank is sent back to the previous rank's last end
    liar = FakeIndex(starts, lie_ranks=(3,), rank=3)
    rows[3] = liar.range(*ranges[3], True)
    confirmed, redo = shard.resolve([r[0] for r in ranges], [r[1] for r in ranges],
                                    [r[1] for r in rows], [r[2] for r in rows])
    assert redo == [3] and confirmed[3] == rows[2][2]


def _worker(rank, world, port, seed, lie, q, giant=50_000):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        starts = _layout(seed, giant=giant)
        L = int(starts[-1])
        b, e = shard.byte_ranges(L, world)[rank]
        fi = FakeIndex(starts, lie_ranks=lie, rank=rank)

        def index_fn(begin, speculative):
            return fi.range(begin, e, speculative)

        def all_gather(vals):
            out = [None] * world
            dist.all_gather_object(out, vals)
            return out

        n, first, last, base, rounds = shard.exchange_boundaries(index_fn, rank, world, b, e,
                                                                 all_gather)
        q.put((rank, n, first, last, base, rounds))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,lie,giant", [(2, (1,), 50_000), (4, (1, 2), 50_000),
                                             (4, (), 50_000),
                                             # world 8 (north_star's node): one record
                                             # over 2+ whole ranges (ranges with no
                                             # record start), three ranks lying
                                             (8, (1, 3, 6), 600_000), (8, (), 600_000)])
def test_exchange_gloo(world, lie, giant):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 7, lie, q, giant))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    starts = _layout(7, giant=giant)
    ranges = shard.byte_ranges(int(starts[-1]), world)
    counts = _truth(starts, [r[0] for r in ranges], [r[1] for r in ranges])
    assert [r[1] for r in res] == counts
    assert [r[4] for r in res] == [sum(counts[:k]) for k in range(world)]
    assert sum(counts) == len(starts) - 1
    if lie:
        assert max(r[5] for r in res) >= 2
    if world == 8:
        # the giant record straddles two or more boundaries: its successors
        # come after one or more ranges that hold no record start
        assert counts.count(0) >= 1
        assert all(r[2] == shard.NONE for r in res if r[1] == 0)


# ---- the whole config-5 composition on CPU ranks ---------------------------
# What bench.py's FileShards runs on the GPUs, with the GPU calls replaced by
# the oracle: every rank encodes its share of a Compact file of config-3
# records (plus a few records larger than a whole range), the byte ranges are
# moved with all_to_all_single (shard.redistribute), each rank indexes its
# range speculatively with the oracle's sequential record walk and the ranks
# confirm their first record start (shard.exchange_boundaries over
# shard.tensor_gather, NONE-safe). The per-rank record sets must be exactly a
# whole-file sequential read's.
GIANT = {37: 70_000, 1200: 150_000}
OVERLAP = 1 << 18


def _mixed_record(i):
    import datagen
    from wire import C, W

    v = datagen.gen_mixed(i)
    w = W(C)
    for k in range(4):
        w.field(8, k + 1).i32(v[k])
    # giant payload bytes 0x0F: a candidate start inside it fails at once
    # (Compact ctype 15, "don't know what type")
    w.field(11, 5).string(v[4] if i not in GIANT else b"\x0f" * GIANT[i])
    return w.field(11, 6).string(v[5]).stop().bytes()


def _share(rank, world, n):
    return range(n * rank // world, n * (rank + 1) // world)


def _composition_worker(rank, world, port, n, q):
    import hashlib

    import torch
    import torch.distributed as dist

    from oracle import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        enc = b"".join(_mixed_record(i) for i in _share(rank, world, n))
        gather = shard.tensor_gather(dist.all_gather, torch.device("cpu"), world)
        sizes = [r[0] for r in gather([len(enc)])]
        enc_ranges, off = [], 0
        for s in sizes:
            enc_ranges.append((off, off + s))
            off += s
        file_len = off
        ranges = shard.byte_ranges(file_len, world)
        lo, hi = shard.need_range(ranges, OVERLAP, file_len, rank)
        out = torch.zeros(hi - lo + 16, dtype=torch.uint8)
        local = shard.redistribute(torch.frombuffer(bytearray(enc), dtype=torch.uint8),
                                   enc_ranges, ranges, OVERLAP, file_len, rank, out,
                                   dist.all_to_all_single)
        buf = local.numpy().copy()
        b, e = ranges[rank]

        def walk(p):
            # records back to back from p while they start before e
            count = 0
            while p < e:
                length = oracle.record_length(2, buf, p - lo)
                if length <= 0:
                    return None
                p += length
                count += 1
            return count, p

        def index_fn(begin, speculative):
            cands = range(begin, e) if speculative else [begin]
            for c in cands:
                r = walk(c)
                if r is not None and r[0] > 0:
                    return r[0], c, r[1]
            return 0, shard.NONE, shard.NONE

        res = shard.exchange_boundaries(index_fn, rank, world, b, e, gather)
        q.put((rank, hashlib.sha256(buf.tobytes()).hexdigest(), (lo, hi)) + tuple(res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_file_split_composition_gloo(world):
    import hashlib

    import torch.multiprocessing as mp

    n = 2400
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_composition_worker, args=(r, world, port, n, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    recs = [_mixed_record(i) for i in range(n)]
    data = b"".join(recs)
    starts = np.concatenate([[0], np.cumsum([len(r) for r in recs])]).astype(np.int64)
    ranges = shard.byte_ranges(len(data), world)
    empty_ranges = 0
    for (rank, digest, (lo, hi), cnt, first, last, base, rounds), (b, e) in zip(res, ranges):
        assert digest == hashlib.sha256(data[lo:hi]).hexdigest()  # bytes moved right
        inside = np.nonzero((starts[:-1] >= b) & (starts[:-1] < e))[0]
        assert cnt == inside.size
        assert base == int(np.count_nonzero(starts[:-1] < b))
        if inside.size:
            assert first == starts[inside[0]] and last == starts[inside[-1] + 1]
        else:
            empty_ranges += 1
            assert first == shard.NONE
    assert sum(r[3] for r in res) == n
    if world >= 4:
        assert empty_ranges >= 1  # a range inside one giant record took the NONE path
    if world == 8:
        # the 150 000-byte record covers more than two of the 8 ranges
        assert empty_ranges >= 2
