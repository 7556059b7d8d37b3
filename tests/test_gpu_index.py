"""Stream index (tgpu_index_stream) and the unindexed decode built on it:
record boundaries of back-to-back records found in parallel must equal the
sequential reference walk (repeated deserialize<T>(Cursor&)) — the oracle's
record offsets — including speculative shards of a stream split by bytes,
records longer than an index chunk, non-canonical records and a malformed
record in the middle of a long stream."""
import numpy as np
import pytest

import datagen
import helpers
from fbthrift_amd.schema import Schema
from oracle import oracle

pytestmark = pytest.mark.gpu


def _t(a, dev):
    import torch

    a = np.frombuffer(bytes(a), np.uint8) if isinstance(a, (bytes, bytearray)) else a
    a = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    if a.size == 0:
        a = np.zeros(1, np.uint8)
    return torch.from_numpy(a.copy()).to(dev)


def _ser(protocol):
    from fbthrift_amd import serializer as S

    return {0: S.BinarySerializer, 2: S.CompactSerializer,
            0x102: S.CompactV1Serializer}[protocol]

    return BinarySerializer if protocol == 0 else CompactSerializer


def _gs(schema):
    from fbthrift_amd.serializer import GpuSchema

    return GpuSchema(schema)


def _stream(sname, proto, n, seed=0, max_len=None):
    table = datagen.SCHEMAS[sname]
    schema = Schema.from_table(table)
    if max_len is None:
        gen = {"mixed": datagen.gen_mixed, "nested": datagen.gen_nested,
               "scalars": datagen.gen_scalars, "sparse": datagen.gen_sparse}[sname]
        vals = datagen.flatten_values(table, [gen(i + seed) for i in range(n)])
        rec, sarena, larena = helpers.pack(schema, vals, n)
    else:  # mixed with long strings
        rng = np.random.default_rng(seed)
        r = np.zeros(n, dtype=schema.dtype())
        for k in range(4):
            r["f%d" % (k + 1)] = rng.integers(-2**31, 2**31 - 1, n, dtype=np.int32)
        lens = rng.integers(0, max_len + 1, (n, 2))
        sarena = rng.integers(0, 256, max(int(lens.sum()), 1), dtype=np.uint8)
        off = 0
        for i in range(n):
            for k in range(2):
                r["f%d" % (k + 5)][i]["offset"] = off
                r["f%d" % (k + 5)][i]["length"] = lens[i, k]
                off += int(lens[i, k])
        r["__isset"] = 1
        rec, larena = r.view(np.uint8), None
    st, wire, offs = oracle.encode(schema, proto, rec, n, sarena, larena)
    assert st.code == 0
    return schema, wire, offs.astype(np.uint64)


@pytest.mark.parametrize("name", helpers.case_names())
def test_index_golden(gpu, codec, name):
    c = helpers.Case(name)
    offs, n, first, last, st = _ser(c.protocol).index_stream(_gs(c.schema), _t(c.wire, gpu))
    assert st.code == 0 and n == c.n and first == 0 and last == len(c.wire)
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), c.offsets.astype(np.uint64))


@pytest.mark.parametrize("sname,proto", [("mixed", 2), ("mixed", 0), ("nested", 0),
                                         ("nested", 2), ("scalars", 2), ("sparse", 2)])
def test_index_and_unindexed_decode_large(gpu, codec, sname, proto):
    """100k-record streams: index == oracle offsets; unindexed decode ==
    oracle decode (records, consumed)."""
    n = 100_000 if sname in ("mixed", "nested") else 30_000
    schema, wire, woffs = _stream(sname, proto, n)
    gs = _gs(schema)
    w = _t(wire, gpu)
    offs, got, first, last, st = _ser(proto).index_stream(gs, w)
    assert (st.code, got, first, last) == (0, n, 0, len(wire))
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), woffs)
    rec, arena, st2, nd, cons = _ser(proto).deserialize_status(gs, w[: len(wire)], n)
    ost, orec, oarena, ond, ocons = oracle.decode(schema, proto, wire, n)
    assert st2.as_tuple() == ost.as_tuple() and st2.code == 0
    assert (nd, cons) == (ond, ocons) == (n, len(wire))
    assert np.array_equal(rec.cpu().numpy(), orec)


@pytest.mark.parametrize("proto", [2, 0])
@pytest.mark.parametrize("max_len", [30, 3000])
def test_index_speculative_shards(gpu, codec, proto, max_len):
    """The stream split into byte ranges at arbitrary positions: each range
    indexed speculatively finds the first record start at/after its begin,
    exactly the oracle's, and its last_end is the next range's first start."""
    n = 200_000 if max_len == 30 else 3000
    schema, wire, woffs = _stream("mixed", proto, n, seed=5, max_len=max_len)
    gs = _gs(schema)
    w = _t(wire, gpu)
    L = len(wire)
    cuts = [0] + sorted(np.random.default_rng(1).integers(1, L, 6).tolist()) + [L]
    prev_last = None
    for b, e in zip(cuts[:-1], cuts[1:]):
        offs, got, first, last, st = _ser(proto).index_stream(
            gs, w[:L], begin=b, end=e, speculative=b > 0)
        inside = woffs[(woffs >= b) & (woffs < e)]
        want_last = woffs[np.searchsorted(woffs, e)] if e < L else L
        if inside.size == 0:
            # no record starts in this range (a record covers it): nothing found
            assert st.code == 0 and got == 0
            continue
        assert st.code == 0, st.as_tuple()
        assert first == inside[0] and got == inside.size and last == want_last
        assert np.array_equal(offs.cpu().numpy()[:-1].astype(np.uint64), inside)
        if prev_last is not None:
            assert prev_last == first
        prev_last = last


def test_index_error_mid_stream(gpu, codec):
    """A malformed record deep in a long unindexed stream: index and decode
    both report the reference status at that record; records before it are
    decoded exactly."""
    proto = 2
    n = 50_000
    schema, wire, woffs = _stream("mixed", proto, n, seed=9)
    bad = 37_123
    w = bytearray(wire)
    w[int(woffs[bad])] = 0x1E  # field header with ctype 14: "don't know what type"
    wire = bytes(w)
    gs = _gs(schema)
    t = _t(wire, gpu)
    offs, got, first, last, st = _ser(proto).index_stream(gs, t, check=False)
    ost, orec, _, ond, ocons = oracle.decode(schema, proto, wire, n)
    assert ost.code != 0 and ost.record == bad
    assert st.as_tuple() == ost.as_tuple()
    assert got == bad and last == woffs[bad]
    rec, arena, gst, nd, cons = _ser(proto).deserialize_status(gs, t, n)
    assert gst.as_tuple() == ost.as_tuple() and (nd, cons) == (ond, ocons)
    k = bad * schema.record_size
    assert np.array_equal(rec.cpu().numpy()[:k], orec[:k])


def test_unindexed_decode_past_end(gpu):
    """Asking for more records than the stream holds: the first missing
    record underflows exactly like the reference's cursor."""
    proto = 2
    n = 5000
    schema, wire, woffs = _stream("mixed", proto, n, seed=3)
    gs = _gs(schema)
    rec, arena, gst, nd, cons = _ser(proto).deserialize_status(gs, _t(wire, gpu), n + 7)
    ost, orec, _, ond, ocons = oracle.decode(schema, proto, wire, n + 7)
    assert gst.as_tuple() == ost.as_tuple() and gst.record == n
    assert (nd, cons) == (ond, ocons)


@pytest.mark.parametrize("n", [5000, 120_000])
def test_unindexed_decode_past_end_large(gpu, codec, n):
    """Same past-the-end rule on a stream long enough for the fused index +
    decode tiles (the first missing record is handed to the general decoder)."""
    proto = 2
    schema, wire, woffs = _stream("mixed", proto, n, seed=4)
    gs = _gs(schema)
    rec, arena, gst, nd, cons = _ser(proto).deserialize_status(gs, _t(wire, gpu), n + 3)
    ost, orec, _, ond, ocons = oracle.decode(schema, proto, wire, n + 3)
    assert gst.as_tuple() == ost.as_tuple() and gst.record == n
    assert (nd, cons) == (ond, ocons)
    assert np.array_equal(rec.cpu().numpy()[: n * schema.record_size], orec[: n * schema.record_size])


@pytest.mark.parametrize("sname,proto", [("mixed", 2), ("nested", 0), ("nested", 2),
                                         ("scalars", 2), ("sparse", 2)])
def test_decode_stream_whole(gpu, codec, sname, proto):
    """tgpu_decode_stream over a whole stream: starts == oracle offsets, records
    and list arena == oracle decode."""
    n = 100_000 if sname in ("mixed", "nested") else 30_000
    schema, wire, woffs = _stream(sname, proto, n, seed=2)
    gs = _gs(schema)
    w = _t(wire, gpu)
    rec, arena, offs, got, first, last, st = _ser(proto).decode_stream(gs, w[: len(wire)],
                                                                       max_records=n)
    assert (st.code, got, first, last) == (0, n, 0, len(wire)), st.as_tuple()
    assert np.array_equal(offs.cpu().numpy()[: n + 1].astype(np.uint64), woffs)
    ost, orec, oarena, _, _ = oracle.decode(schema, proto, wire, n)
    assert np.array_equal(rec.cpu().numpy()[: n * schema.record_size], orec)
    if arena is not None:
        helpers.assert_arena_equal(schema, orec, n, wire, arena.cpu().numpy(), oarena)


@pytest.mark.parametrize("proto", [2, 0])
def test_decode_stream_speculative_shards(gpu, codec, proto):
    """Each byte range of a stream cut at arbitrary positions, decoded
    speculatively, holds exactly the oracle's records that start in it."""
    n = 200_000
    schema, wire, woffs = _stream("mixed", proto, n, seed=6, max_len=30)
    gs = _gs(schema)
    w = _t(wire, gpu)
    L = len(wire)
    ost, orec, _, _, _ = oracle.decode(schema, proto, wire, n)
    S = schema.record_size
    cuts = [0] + sorted(np.random.default_rng(3).integers(1, L, 5).tolist()) + [L]
    for b, e in zip(cuts[:-1], cuts[1:]):
        rec, arena, offs, got, first, last, st = _ser(proto).decode_stream(
            gs, w[:L], begin=b, end=e, speculative=b > 0, max_records=n)
        i0 = int(np.searchsorted(woffs, b))
        i1 = int(np.searchsorted(woffs[:n], e))
        assert st.code == 0 and got == i1 - i0, st.as_tuple()
        if got:
            assert first == woffs[i0]
            assert np.array_equal(rec.cpu().numpy()[: got * S], orec[i0 * S: i1 * S])


def test_decode_stream_error_mid_stream(gpu, codec):
    proto = 2
    n = 60_000
    schema, wire, woffs = _stream("mixed", proto, n, seed=11)
    bad = 41_000
    w = bytearray(wire)
    w[int(woffs[bad])] = 0x1E  # ctype 14: "don't know what type"
    wire = bytes(w)
    gs = _gs(schema)
    rec, arena, offs, got, first, last, st = _ser(proto).decode_stream(gs, _t(wire, gpu),
                                                                       max_records=n)
    ost, orec, _, ond, ocons = oracle.decode(schema, proto, wire, n)
    assert st.as_tuple() == ost.as_tuple() and got == bad
    k = bad * schema.record_size
    assert np.array_equal(rec.cpu().numpy()[:k], orec[:k])


@pytest.mark.parametrize("variant", ["onepass", "fused"])
@pytest.mark.parametrize("sname,proto", [("mixed", 2), ("mixed", 0), ("nested", 0)])
def test_index_variants(gpu, sname, proto, variant, monkeypatch):
    """The index forms that are off by default give the oracle's offsets and
    records, whole and as speculative byte ranges, and a malformed record the
    reference status: the single pass (TGPU_INDEX_ONEPASS=1: look-back over
    packed tile statuses, k_index.hip launch_index_onepass; a malformed record
    makes it fall back to the two-pass index) and the two-pass index whose
    emit tiles re-walk their chains and decode the records as they go
    (TGPU_INDEX_STARTS=0; by default the emit copies the speculation pass's
    stored starts and the indexed program decode follows)."""
    if variant == "onepass":
        monkeypatch.setenv("TGPU_INDEX_ONEPASS", "1")
    else:
        monkeypatch.setenv("TGPU_INDEX_STARTS", "0")
    n = 300_000 if sname == "mixed" else 100_000
    schema, wire, woffs = _stream(sname, proto, n, seed=3)
    gs = _gs(schema)
    w = _t(wire, gpu)
    offs, got, first, last, st = _ser(proto).index_stream(gs, w)
    assert (st.code, got, first, last) == (0, n, 0, len(wire))
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), woffs)
    rec, arena, st2, nd, cons = _ser(proto).deserialize_status(gs, w[: len(wire)], n)
    ost, orec, oarena, ond, ocons = oracle.decode(schema, proto, wire, n)
    assert st2.as_tuple() == ost.as_tuple() and (nd, cons) == (ond, ocons)
    assert np.array_equal(rec.cpu().numpy(), orec)
    L = len(wire)
    b, e = L // 3 + 7, 2 * L // 3 + 5
    offs, got, first, last, st = _ser(proto).index_stream(gs, w[:L], begin=b, end=e,
                                                          speculative=True)
    inside = woffs[(woffs >= b) & (woffs < e)]
    assert st.code == 0 and first == inside[0] and got == inside.size
    assert last == woffs[np.searchsorted(woffs, e)]
    bad = n // 2
    wb = bytearray(wire)
    wb[int(woffs[bad])] = 0x1E if proto == 2 else 0x7F  # an unknown field type
    wb = bytes(wb)
    rec, arena, st3, nd, cons = _ser(proto).deserialize_status(gs, _t(wb, gpu)[:L], n)
    ost, orec, _, ond, ocons = oracle.decode(schema, proto, wb, n)
    assert st3.as_tuple() == ost.as_tuple() and (nd, cons) == (ond, ocons)
    k = (ond + 1) * schema.size[0]
    assert np.array_equal(rec.cpu().numpy()[:k], orec[:k])


@pytest.fixture
def programless(monkeypatch):
    """A stream without any record program (TGPU_NESTED=0 and a schema with
    optional fields: no flat program), the root first-byte filter off, and the
    exhaustive resolution forced (TGPU_INDEX_EXHAUSTIVE=1: every chunk
    position read, the true path followed through the tables) — so the
    general speculation and its repair decide every record start."""
    monkeypatch.setenv("TGPU_NESTED", "0")
    monkeypatch.setenv("TGPU_INDEX_HMASK", "0")
    monkeypatch.setenv("TGPU_INDEX_EXHAUSTIVE", "1")


@pytest.mark.parametrize("proto", [2, 0])
def test_exhaustive_resolution_matches_oracle(gpu, programless, proto):
    n = 30_000
    schema, wire, woffs = _stream("sparse", proto, n, seed=6)
    gs = _gs(schema)
    w = _t(wire, gpu)
    offs, got, first, last, st = _ser(proto).index_stream(gs, w)
    assert (st.code, got, first, last) == (0, n, 0, len(wire)), st.as_tuple()
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), woffs)
    rec, arena, st2, nd, cons = _ser(proto).deserialize_status(gs, w[: len(wire)], n)
    ost, orec, oarena, ond, ocons = oracle.decode(schema, proto, wire, n)
    assert st2.as_tuple() == ost.as_tuple() and (nd, cons) == (ond, ocons) == (n, len(wire))
    assert np.array_equal(rec.cpu().numpy(), orec)


@pytest.mark.parametrize("extra", [0, 7])
def test_exhaustive_resolution_errors(gpu, programless, extra):
    """A malformed record deep in the stream (and records asked for past its
    end): status, records before the failure and consumed bytes as the
    oracle's sequential reader."""
    proto = 2
    n = 30_000
    schema, wire, woffs = _stream("sparse", proto, n, seed=8)
    w = bytearray(wire)
    bad = 21_017
    if not extra:
        w[int(woffs[bad])] = 0x1E  # ctype 14 header: "don't know what type"
    wire = bytes(w)
    gs = _gs(schema)
    t = _t(wire, gpu)
    rec, arena, gst, nd, cons = _ser(proto).deserialize_status(gs, t, n + extra)
    ost, orec, _, ond, ocons = oracle.decode(schema, proto, wire, n + extra)
    assert ost.code != 0
    assert gst.as_tuple() == ost.as_tuple() and (nd, cons) == (ond, ocons)
    k = ond * schema.record_size
    assert np.array_equal(rec.cpu().numpy()[:k], orec[:k])
