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


def _adversarial(gpu, monkeypatch, programless):
    import time

    import torch

    from fbthrift_amd.serializer import CompactV1Serializer as S, GpuSchema
    from oracle import oracle

    monkeypatch.setenv("TGPU_INDEX_HMASK", "0")
    if programless:
        monkeypatch.setenv("TGPU_NESTED", "0")
    n = 1 << 20
    table = [[list(r) for r in t] for t in datagen.SCHEMAS["nested"]]
    if programless:
        table[0][0][3] = 1  # field 1 optional (TGPU_OPTIONAL): no flat program
    schema = Schema.from_table(table)
    rs = schema.record_size
    recs = torch.empty(n * rs, dtype=torch.uint8, device=gpu)
    side = torch.empty(n * 64, dtype=torch.uint8, device=gpu)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libtgpu_datagen.so"))
    assert lib.tgpu_gen_nested_packed(ctypes.c_uint64(datagen.SEED), ctypes.c_uint64(0),
                                      ctypes.c_uint64(n), ctypes.c_void_p(recs.data_ptr()),
                                      ctypes.c_void_p(side.data_ptr()), None) == 0
    gs = GpuSchema(schema)
    wire, _ = S.serialize(gs, recs, n, list_base=side)
    torch.cuda.synchronize()
    w = wire.cpu().numpy().tobytes()
    ost, orec, oarena, ond, ocons = oracle.decode(schema, 0x102, w, n)
    assert ost.code == 0 and ond == n
    S.deserialize_status(gs, wire, n)  # warm-up (workspaces)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(2):
        t0 = time.perf_counter()
        grec, garena, gst, gnd, gcons = S.deserialize_status(gs, wire, n)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    assert gst.code == 0 and gnd == n and gcons == len(w), gst.as_tuple()
    assert np.array_equal(grec.cpu().numpy()[: n * rs], orec[: n * rs])
    stats = S.context().index_stats()
    print("adversarial stream (%s): %.1f ms, %s" % ("program-less" if programless else "program",
                                                    best * 1e3, stats))
    return best, stats


def test_adversarial_v1_stream_with_the_filter_off(gpu, monkeypatch):
    """Round 4's adversarial case as the verdict states it: 1 Mi records of
    the nested schema (i64, list<i32>, a struct of three doubles) in CompactV1,
    unindexed, the root first-byte filter off (TGPU_INDEX_HMASK=0). Its little-
    endian doubles sent round 4's general speculation into false chains and
    its one-lane repair over the stream (3.8 s); round 5's V1 program takes
    the stream through the program speculation of the LDS tiles: no broken
    link, the whole decode well under 100 ms; records equal the oracle's."""
    dt, stats = _adversarial(gpu, monkeypatch, False)
    assert stats["broken"] == 0 and stats["general"] == 0, stats
    assert dt < 0.100, (dt, stats)


def test_adversarial_programless_stream_repairs_in_parallel(gpu, monkeypatch):
    """The same stream with no record program at all — field 1 optional and
    nested programs off (TGPU_NESTED=0) — so the general reader speculates
    from every byte (filter off): almost every chunk opens on a false start.
    The speculation's chunks and reach follow the mean record length
    (tgpu_api.cpp launch_index), the Jacobi merge rounds repair the links in
    parallel and the verification walks only to meeting points (k_index.hip
    walk_meet): under 100 ms (round 4: 3.8 s; 5.5 s with round 5's rounds
    but 4 KiB chunks and a 256 KiB reach); records equal the oracle's."""
    dt, stats = _adversarial(gpu, monkeypatch, True)
    assert stats["broken"] > stats["chunks"] // 2, stats  # (it is adversarial)
    assert dt < 0.100, (dt, stats)
