"""Repair counters of the parallel stream index (tgpu_index_stats): a
canonical stream — every record in the schema's canonical form, as the
reference's writer emits it — must need no repair at all, indexed from its
first byte and as speculative shards of a file split by bytes. A recurrence of
round 2's LDS-staging corruption (tiles whose speculated chains broke, hidden
by the repair passes at a cost in speed only) shows up here as a non-zero
count. The last case checks the counters do move: one record carrying an
unknown field leaves its tile partial for the general reader."""
import ctypes
import os

import numpy as np
import pytest

import datagen
from fbthrift_amd.schema import Schema

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 1 << 20


@pytest.fixture(scope="module")
def stream(gpu):
    import torch

    from fbthrift_amd.serializer import CompactSerializer, GpuSchema

    schema = Schema.from_table(datagen.SCHEMAS["mixed"])
    rs = schema.record_size
    recs = torch.empty(N * rs, dtype=torch.uint8, device=gpu)
    side = torch.empty(N * 64, dtype=torch.uint8, device=gpu)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libtgpu_datagen.so"))
    assert lib.tgpu_gen_mixed(ctypes.c_uint64(datagen.SEED), ctypes.c_uint64(0),
                              ctypes.c_uint64(N), ctypes.c_void_p(recs.data_ptr()),
                              ctypes.c_void_p(side.data_ptr()), None) == 0
    gs = GpuSchema(schema)
    wire, offs = CompactSerializer.serialize(gs, recs, N, string_base=side)
    torch.cuda.synchronize()
    return gs, recs, wire, offs


def _decode(gs, wire, begin, end, speculative):
    from fbthrift_amd.serializer import CompactSerializer as S

    recs, _, offs, n, first, last, st = S.decode_stream(gs, wire, begin=begin, end=end,
                                                        speculative=speculative,
                                                        max_records=N + 16)
    assert st.code == 0, st.as_tuple()
    return n, first, last, S.context().index_stats()


def _clean(stats):
    return {k: v for k, v in stats.items() if k != "chunks"}


def test_canonical_stream_needs_no_repair(stream, codec):
    gs, recs, wire, offs = stream
    n, first, last, stats = _decode(gs, wire, 0, wire.numel(), False)
    assert n == N and first == 0 and last == wire.numel()
    assert stats["chunks"] > 1000
    assert _clean(stats) == dict.fromkeys(_clean(stats), 0), stats


@pytest.mark.parametrize("world", [2, 3, 8])
def test_canonical_shards_need_no_repair(stream, codec, world):
    gs, recs, wire, offs = stream
    L = wire.numel()
    o = offs.cpu().numpy()
    total = 0
    for k in range(1, world):
        b, e = L * k // world, L * (k + 1) // world
        n, first, last, stats = _decode(gs, wire, b, e, True)
        i = int(np.searchsorted(o, b))
        assert first == o[i]
        total += n
        assert _clean(stats) == dict.fromkeys(_clean(stats), 0), (k, stats)
    assert total == N - int(np.searchsorted(o, L // world))


def test_counters_see_a_non_canonical_record(stream, codec):
    import torch

    gs, recs, wire, offs = stream
    o = offs.cpu().numpy()
    k = N // 2
    a, b = int(o[k]), int(o[k + 1])
    assert int(wire[b - 1]) == 0  # the record's STOP
    # an unknown i32 field 7 (delta 1: header 0x15, zigzag 1 = 0x02) before it
    w2 = torch.cat([wire[: b - 1], torch.tensor([0x15, 0x02, 0x00], dtype=torch.uint8,
                                                device=wire.device), wire[b:]])
    n, first, last, stats = _decode(gs, w2, 0, w2.numel(), False)
    assert n == N and last == w2.numel()
    assert stats["partial"] + stats["no_start"] + stats["broken"] >= 1, stats
