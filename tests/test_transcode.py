"""Binary <-> Compact <-> CompactV1 transcoding (tgpu_transcode_batch):
serialize<To>(deserialize<From>(record)) for every record, on the device —
the bulk form of thrift/lib/cpp2/transcode (README.md:1-20: schema-driven
wire-to-wire conversion).

Pinned by the reference's own vectors: the golden cases of one schema were
written by the reference's Python protocols from the same values in every
protocol, so transcoding case X_<from> must give exactly X_<to>'s bytes.
Unknown fields are dropped (the generated codec does not retain them):
UpdatedStruct bytes transcoded under OriginalStruct's schema equal
OriginalStruct written directly.
"""
import itertools

import numpy as np
import pytest

import helpers
from oracle import oracle

PROTOS = {"binary": 0, "compact": 2, "compact_v1": 0x102}


def _pairs():
    """(from case, to case) golden pairs with the same schema and values."""
    names = helpers.case_names()
    out = []
    for a, b in itertools.permutations(names, 2):
        for pa in PROTOS:
            for pb in PROTOS:
                if a.endswith("_" + pa) and b.endswith("_" + pb):
                    ba, bb = a[: -len(pa) - 1], b[: -len(pb) - 1]
                    if ba == bb and pa != pb:
                        out.append((a, b))
    return sorted(set(out))


PAIRS = _pairs()


def _oracle_transcode(schema, pf, pt, wire, n):
    st, rec, arena, nd, _ = oracle.decode(schema, pf, wire, n)
    est, out, offs = oracle.encode(schema, pt, rec, nd, np.frombuffer(bytes(wire) or b"\0", np.uint8),
                                   arena)
    return st, nd, out, offs


@pytest.mark.parametrize("src,dst", PAIRS, ids=["%s->%s" % p for p in PAIRS])
def test_oracle_transcode_equals_reference_bytes(src, dst):
    a, b = helpers.Case(src), helpers.Case(dst)
    n = min(a.n, b.n)
    wire = a.wire[: int(a.offsets[n])]
    st, nd, out, offs = _oracle_transcode(a.schema, a.protocol, b.protocol, wire, n)
    assert st.code == 0 and nd == n
    assert out == b.wire[: int(b.offsets[n])]


@pytest.mark.parametrize("proto", ["binary", "compact"])
def test_oracle_transcode_drops_unknown_fields(proto):
    upd, orig = helpers.Case("updated_" + proto), helpers.Case("original_" + proto)
    for to in ("binary", "compact"):
        st, nd, out, _ = _oracle_transcode(orig.schema, upd.protocol, PROTOS[to], upd.wire, 1)
        assert st.code == 0 and out == helpers.Case("original_" + to).wire


def _gpu_transcode(dev, schema, pf, pt, wire, n, out_cap=None, offsets=None):
    import torch

    from fbthrift_amd import serializer as S

    ser = {0: S.BinarySerializer, 2: S.CompactSerializer, 0x102: S.CompactV1Serializer}[pf]
    gs = S.GpuSchema(schema)
    w = torch.from_numpy(np.frombuffer(bytes(wire) or b"\0", np.uint8).copy()).to(dev)
    out = None if out_cap is None else torch.empty(max(out_cap, 1), dtype=torch.uint8, device=dev)
    offs_t = None
    if offsets is not None:
        offs_t = torch.from_numpy(np.asarray(offsets, np.int64).copy()).to(dev)
    out, offs, st, done, size = ser.transcode(gs, w[: len(wire)] if len(wire) else w[:0], n, pt,
                                              offsets=offs_t, out=out)
    return st, done, bytes(out[:size].cpu().numpy()), offs[: done + 1].cpu().numpy()


@pytest.fixture(params=["onepass", "twopass", "composed"])
def xmode(request, monkeypatch):
    """Every transcoder form: wire to wire without records in HBM
    (tgpu_xcode.h; schemas with a flat program in both protocols) as the
    single pass with look-back (default) and as the two tile passes
    (TGPU_XCODE_ONEPASS=0), and the composed decode + encode (TGPU_XCODE=0)."""
    monkeypatch.setenv("TGPU_XCODE", "0" if request.param == "composed" else "1")
    monkeypatch.setenv("TGPU_XCODE_ONEPASS", "1" if request.param == "onepass" else "0")
    return request.param


@pytest.mark.gpu
@pytest.mark.parametrize("src,dst", PAIRS, ids=["%s->%s" % p for p in PAIRS])
def test_gpu_transcode_golden(gpu, xmode, src, dst):
    a, b = helpers.Case(src), helpers.Case(dst)
    n = min(a.n, b.n)
    wire = a.wire[: int(a.offsets[n])]
    for offs in (None, a.offsets[: n + 1]):
        st, done, out, o = _gpu_transcode(gpu, a.schema, a.protocol, b.protocol, wire, n,
                                          offsets=offs)
        assert st.code == 0 and done == n, st.as_tuple()
        assert out == b.wire[: int(b.offsets[n])]
        assert np.array_equal(o.astype(np.uint64), b.offsets[: n + 1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["maps_compact", "unions_binary", "nested_compact_v1",
                                  "scalars_binary"])
def test_gpu_transcode_errors_match_oracle(gpu, xmode, name):
    """Damaged input: the reader's status, the records before it transcoded
    (as the oracle does it); a small output: OUTPUT_OVERFLOW at the record
    that does not fit."""
    c = helpers.Case(name)
    rng = np.random.default_rng(3)
    to = 0 if c.protocol != 0 else 2
    for trial in range(6):
        m = np.frombuffer(c.wire, np.uint8).copy()
        pos = rng.integers(0, m.size, 2)
        m[pos] = rng.integers(0, 256, 2)
        st, done, out, _ = _gpu_transcode(gpu, c.schema, c.protocol, to, m.tobytes(), c.n)
        ost, ond, oout, _ = _oracle_transcode(c.schema, c.protocol, to, m.tobytes(), c.n)
        assert st.as_tuple() == ost.as_tuple() and done == ond, trial
        assert out == oout
    full = _oracle_transcode(c.schema, c.protocol, to, c.wire, c.n)[2]
    st, done, out, _ = _gpu_transcode(gpu, c.schema, c.protocol, to, c.wire, c.n,
                                      out_cap=len(full) // 2)
    assert st.code == 21 and 0 < done < c.n
    assert out == full[: len(out)]


def _mixed_stream(n, every, proto):
    """n config-3 records (Compact / Binary, schema `mixed`) whose record i is
    written with the fields in another order when i % every == 0 (every = 0:
    none; a record
    the generated readNoXfer reads through its unexpected-field path, and the
    record program cannot take): the oracle's bytes, record by record."""
    import datagen
    from fbthrift_amd.schema import Schema

    table = datagen.SCHEMAS["mixed"]
    perm = [5, 0, 3, 1, 4, 2]  # declaration order of the reordered writer
    t2 = [[table[0][k] for k in perm]]
    recs = [datagen.gen_mixed(i) for i in range(n)]
    sa, sb = Schema.from_table(table), Schema.from_table(t2)
    ra, sta, _ = helpers.pack(sa, datagen.flatten_values(table, recs), n)
    st, wa, oa = oracle.encode(sa, proto, ra, n, sta)
    assert st.code == 0
    rb, stb, _ = helpers.pack(sb, datagen.flatten_values(t2, [[r[k] for k in perm] for r in recs]),
                              n)
    st, wb, ob = oracle.encode(sb, proto, rb, n, stb)
    assert st.code == 0
    parts, offs = [], [0]
    for i in range(n):
        w, o = (wb, ob) if every and i % every == 0 else (wa, oa)
        parts.append(w[int(o[i]):int(o[i + 1])])
        offs.append(offs[-1] + len(parts[-1]))
    return sa, b"".join(parts), np.array(offs, np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("every", [997, 0], ids=["irregular", "canonical"])
@pytest.mark.parametrize("onepass", ["1", "0"], ids=["onepass", "twopass"])
@pytest.mark.parametrize("pf,pt", [(2, 0), (0, 2)])
def test_gpu_transcode_fused_irregular_records(gpu, codec, pf, pt, onepass, every, monkeypatch):
    """100 003 records (391 tiles: the single pass's look-back runs across
    windows of 64), every 997th off the canonical field order or none: the
    fused transcoder lists those for the general reader / writer (index_stats
    'general' counts them; the single pass then opens the gate of the two
    tile passes) and its output equals the oracle's serialize<To>(
    deserialize<From>) byte for byte — indexed and unindexed, with and without
    output offsets; an output of half the size stops at the first record that
    does not fit (OUTPUT_OVERFLOW) with every record before it written."""
    import torch

    from fbthrift_amd import serializer as S

    monkeypatch.setenv("TGPU_XCODE", "1")
    monkeypatch.setenv("TGPU_XCODE_ONEPASS", onepass)
    n = 100_003
    schema, wire, offs = _mixed_stream(n, every, pf)
    st, nd, want, woffs = _oracle_transcode(schema, pf, pt, wire, n)
    assert st.code == 0 and nd == n
    ser = {0: S.BinarySerializer, 2: S.CompactSerializer}[pf]
    gs = S.GpuSchema(schema)
    w = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).to(gpu)
    o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    for given in (o, None):
        for want_offs in (True, False):
            out, go, gst, done, size = ser.transcode(gs, w, n, pt, offsets=given,
                                                     want_offsets=want_offs)
            assert gst.code == 0 and done == n, gst.as_tuple()
            assert bytes(out[:size].cpu().numpy()) == want
            if want_offs:
                assert np.array_equal(go.cpu().numpy().astype(np.uint64), np.asarray(woffs, np.uint64))
            assert ser.context().index_stats()["general"] == ((n + every - 1) // every
                                                               if every else 0)
    cap = len(want) // 2
    out = torch.empty(cap, dtype=torch.uint8, device=gpu)
    out, go, gst, done, size = ser.transcode(gs, w, n, pt, offsets=o, out=out)
    wo = np.asarray(woffs, np.uint64)
    fit = int(np.searchsorted(wo[1:], cap, side="right"))  # records whose end is <= cap
    assert gst.code == 21 and done == fit and size == int(wo[fit]), (gst.as_tuple(), done, fit)
    assert bytes(out[:size].cpu().numpy()) == want[:size]


def _small_records(n, seed=11):
    """n records of {1..5: i64} with small values: S = 48 (5 x 8 + 5 isset
    bytes, 8-aligned), about 11 Compact wire bytes per record."""
    from fbthrift_amd.schema import Schema

    schema = Schema.from_table([[[k, 10, 0, 0, -1] for k in range(1, 6)]])
    assert schema.record_size == 48
    rng = np.random.default_rng(seed)
    rec = np.zeros(n, dtype=schema.dtype())
    for f in schema.structs[0].fields:
        rec[f.name] = rng.integers(-60, 60, n)
    rec["__isset"][:] = 1
    return schema, rec.view(np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("pt", [0x102, 0])
def test_gpu_transcode_small_records_lds_sizing(gpu, xmode, pt):
    """with the record tile in LDS (the library's own
    kernels, below the schema compiler's 64 Ki-record threshold) a light
    record (S 48, ~11 Compact bytes) made the joint LDS sizing take a 4 KiB
    wire-cap floor it had not fitted, and the output tile size went negative.
    The transcoded stream must equal the composed decode + encode (the
    oracle's) byte for byte."""
    n = 50_000
    schema, rec = _small_records(n)
    st, wire, offs = oracle.encode(schema, 2, rec, n, None)
    assert st.code == 0 and len(wire) < 12 * n
    ost, ond, want, woffs = _oracle_transcode(schema, 2, pt, wire, n)
    assert ost.code == 0 and ond == n
    for given in (None, offs):
        gst, done, out, o = _gpu_transcode(gpu, schema, 2, pt, wire, n, offsets=given)
        assert gst.code == 0 and done == n, gst.as_tuple()
        assert out == want
        assert np.array_equal(o.astype(np.uint64), np.asarray(woffs, np.uint64))
