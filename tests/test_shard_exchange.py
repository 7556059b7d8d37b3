"""Shard-boundary exchange for one file split by bytes across ranks
(fbthrift_amd/shard.py): the host logic of BASELINE config 5, run over a
fake indexer with a known record layout, on the CPU with gloo (world sizes 2
and 4) and as a pure function."""
import os
import socket

import numpy as np
import pytest

from fbthrift_amd import shard


def _layout(seed, n=5000, max_len=400):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, max_len, n)
    # a few records longer than a whole range
    lens[n // 3] = 50_000
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


def _worker(rank, world, port, seed, lie, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        starts = _layout(seed)
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


@pytest.mark.parametrize("world,lie", [(2, (1,)), (4, (1, 2)), (4, ())])
def test_exchange_gloo(world, lie):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 7, lie, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    starts = _layout(7)
    ranges = shard.byte_ranges(int(starts[-1]), world)
    counts = _truth(starts, [r[0] for r in ranges], [r[1] for r in ranges])
    assert [r[1] for r in res] == counts
    assert [r[4] for r in res] == [sum(counts[:k]) for k in range(world)]
    assert sum(counts) == len(starts) - 1
    if lie:
        assert max(r[5] for r in res) >= 2
