"""Schemaless skip-scan and field projection with the
existing entry points:

* record boundaries without a schema: tgpu_index_stream with an empty
  struct as the schema — every field is unknown, so each record is read by
  the reader's skip (apache::thrift::skip, Protocol.h:187-283), which is
  exactly how `while (!cursor.isAtEnd()) deserialize<T>(cursor)` would
  walk the stream for a T that declares nothing;
* projection: decoding with a schema that declares only the wanted fields
  (the rest are skipped), as a generated struct holding a subset of the
  writer's fields reads a newer writer's bytes
  (CompactProtocolTest.cpp:140-166 'parses updated via read').
"""
import numpy as np
import pytest

import corpus
import helpers
from fbthrift_amd.schema import Field, Schema, Struct
from oracle import oracle

ANY = Schema(Struct("Any", []))


def test_oracle_schemaless_walk_matches_golden_offsets():
    for name in helpers.case_names():
        c = helpers.Case(name)
        pos, offs = 0, [0]
        for _ in range(c.n):
            pos += oracle.record_length(c.protocol, c.wire, pos)
            offs.append(pos)
        assert np.array_equal(np.array(offs, np.uint64), c.offsets), name


@pytest.mark.gpu
@pytest.mark.parametrize("name", helpers.case_names())
def test_gpu_schemaless_index(gpu, name):
    import torch

    from fbthrift_amd import serializer as S

    c = helpers.Case(name)
    ser = {0: S.BinarySerializer, 2: S.CompactSerializer, 0x102: S.CompactV1Serializer}[c.protocol]
    w = torch.from_numpy(np.frombuffer(c.wire, np.uint8).copy()).to(gpu)
    offs, n, first, last, st = ser.index_stream(S.GpuSchema(ANY), w)
    assert st.code == 0 and n == c.n and last == len(c.wire)
    assert np.array_equal(offs.cpu().numpy()[: n + 1].astype(np.uint64), c.offsets)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["scalars_binary", "scalars_compact", "maps_compact",
                                  "unions_binary"])
def test_gpu_projection(gpu, name):
    """A schema with a subset of the fields reads the same values for them."""
    import torch

    from fbthrift_amd import serializer as S

    c = helpers.Case(name)
    root = c.schema.structs[0]
    keep = [0, len(root.fields) - 1]
    sub = Schema(Struct("P", [root.fields[k] for k in keep]))
    ser = {0: S.BinarySerializer, 2: S.CompactSerializer}[c.protocol]
    w = torch.from_numpy(np.frombuffer(c.wire, np.uint8).copy()).to(gpu)
    rec, arena, st, nd, cons = ser.deserialize_status(S.GpuSchema(sub), w, c.n)
    assert st.code == 0 and nd == c.n and cons == len(c.wire)
    got = helpers.unpack(sub, rec.cpu().numpy(), c.n, c.wire, arena.cpu().numpy())
    ost, orec, oarena, _, _ = oracle.decode(sub, c.protocol, c.wire, c.n)
    helpers.assert_values_equal(got, helpers.unpack(sub, orec, c.n, c.wire, oarena))
    # and they are the full record's values for those fields
    for j, k in enumerate(keep):
        for suffix in (".set", ".val", ".len", ".count"):
            if "%d%s" % (k, suffix) in c.values:
                assert np.array_equal(got["%d%s" % (j, suffix)], c.values["%d%s" % (k, suffix)])


# ---- tgpu_skim_batch: schemaless field tables ---------------------------------
# Pinned by the golden cases (wire bytes and values written by the reference
# Python protocols, tests/golden/make_golden.py): the skim of each record must
# list exactly the fields the golden values mark as set, in declaration order
# (the reference writer's order), tile the record's bytes (header, value, ...,
# STOP), and its value bytes must decode to the golden values.
_T_BOOL, _T_BYTE, _T_DOUBLE, _T_I16, _T_I32, _T_I64, _T_STRING, _T_FLOAT = 2, 3, 4, 6, 8, 10, 11, 19


def _uvarint(b, pos):
    v, s = 0, 0
    while True:
        x = b[pos]
        pos += 1
        v |= (x & 0x7F) << s
        s += 7
        if not x & 0x80:
            return v, pos


def _scalar(proto, t, raw, flags):
    """Value of a skimmed scalar from its encoded bytes (independent of the
    oracle: big-endian / zigzag varint straight from the wire specs)."""
    if t == _T_BOOL:
        return int(bool(flags & 2)) if proto != 0 else raw[0]
    if proto == 0 or t in (_T_BYTE,):
        if t == _T_BYTE:
            return int.from_bytes(raw, "big", signed=True)
        signed = t in (_T_I16, _T_I32, _T_I64)
        return int.from_bytes(raw, "big", signed=signed)
    if t == _T_DOUBLE:
        return int.from_bytes(raw, "little" if proto == 0x102 else "big")
    if t == _T_FLOAT:
        return int.from_bytes(raw, "big")
    z, end = _uvarint(raw, 0)
    assert end == len(raw)
    return (z >> 1) ^ -(z & 1)


def _check_skim_against_golden(c, fields, counts):
    root = c.schema.structs[0]
    w = c.wire
    for i in range(c.n):
        want = [k for k in range(len(root.fields)) if c.values["%d.set" % k][i]]
        assert counts[i] == len(want), (c.name, i)
        pos_end = int(c.offsets[i])
        for j, k in enumerate(want):
            f = root.fields[k]
            e = fields[i, j]
            assert e["id"] == f.id, (c.name, i, j)
            assert e["offset"] > pos_end  # a field header precedes every value
            pos_end = int(e["offset"]) + int(e["length"])
            raw = w[e["offset"]: e["offset"] + e["length"]]
            if "%d.val" % k in c.values and f.ttype != _T_STRING:
                got = _scalar(c.protocol, int(e["ttype"]), raw, int(e["flags"]))
                v = c.values["%d.val" % k][i]
                assert got == (int(v) if f.ttype != _T_BOOL else int(bool(v))), (c.name, i, k)
        assert pos_end + 1 == int(c.offsets[i + 1]), (c.name, i)  # then STOP


@pytest.mark.parametrize("name", helpers.case_names())
def test_oracle_skim_matches_golden(name):
    c = helpers.Case(name)
    st, fields, counts, done = oracle.skim(c.protocol, c.wire, c.offsets, c.n, max_fields=32)
    assert st.code == 0 and done == c.n
    _check_skim_against_golden(c, fields, counts)


def test_oracle_skim_counts_past_max_fields():
    c = helpers.Case("scalars_binary")
    st, full, counts, _ = oracle.skim(c.protocol, c.wire, c.offsets, c.n, max_fields=32)
    st2, part, counts2, _ = oracle.skim(c.protocol, c.wire, c.offsets, c.n, max_fields=3)
    assert st2.code == 0 and np.array_equal(counts, counts2) and counts.max() > 3
    assert np.array_equal(part, full[:, :3])


def test_oracle_skim_index_mismatch():
    c = helpers.Case("flat8_binary")
    offs = c.offsets.copy()
    offs[5] += 1
    st, _, _, done = oracle.skim(c.protocol, c.wire, offs, c.n)
    assert st.code == 20 and done == 4 and st.record == 4


def _skim_both(gpu, protocol, wire, offsets, n, max_fields, limits=None):
    import torch

    from fbthrift_amd import serializer as S

    ser = {0: S.BinarySerializer, 2: S.CompactSerializer, 0x102: S.CompactV1Serializer}[protocol]
    w = torch.from_numpy(np.frombuffer(bytes(wire) or b"\0", np.uint8).copy()).to(gpu)[: len(wire)]
    o = torch.from_numpy(np.asarray(offsets, np.uint64).astype(np.int64)).to(gpu)
    fields, counts, done, st = ser.skim(w, o, n, max_fields=max_fields, limits=limits, check=False)
    ost, ofields, ocounts, odone = oracle.skim(protocol, wire, offsets, n, max_fields, limits)
    assert st.as_tuple() == ost.as_tuple() and done == odone
    got = S.skim_records(fields, n, max_fields)
    cnt = counts.cpu().numpy()
    for i in range(done):  # records before the failing one are complete
        assert cnt[i] == ocounts[i]
        k = min(int(cnt[i]), max_fields)
        assert np.array_equal(got[i, :k], ofields[i, :k]), i
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("name", helpers.case_names())
@pytest.mark.parametrize("max_fields", [2, 32])
def test_gpu_skim_golden(gpu, name, max_fields):
    c = helpers.Case(name)
    st = _skim_both(gpu, c.protocol, c.wire, c.offsets, c.n, max_fields)
    assert st.code == 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in corpus.cases() if c[4] == 1], ids=lambda c: c[0])
def test_gpu_skim_corpus(gpu, case):
    """Damaged and edge-case records (the reference's own test inputs): the
    skim's status is the oracle's, record for record."""
    name, protocol, _table, wire, n, limits, _code = case
    _skim_both(gpu, protocol, wire, [0, len(wire)], 1, 8, limits)


@pytest.mark.gpu
def test_gpu_skim_empty_and_mismatch(gpu):
    c = helpers.Case("mixed_compact")
    _skim_both(gpu, c.protocol, c.wire, c.offsets[:1], 0, 4)
    offs = c.offsets.copy()
    offs[7] -= 1
    st = _skim_both(gpu, c.protocol, c.wire, offs, c.n, 4)
    assert st.code == 20 and st.record == 6


@pytest.mark.parametrize("case", [c for c in corpus.cases() if c[4] == 1], ids=lambda c: c[0])
def test_oracle_skim_status_is_schemaless_decode_status(case):
    """A skim reads what a field-less struct's readNoXfer skips, so on every
    reference test input its status equals decoding with an empty schema —
    except a Binary bool field byte >= 2: BinaryProtocolReader::skip passes
    over it (BinaryProtocol.cpp:146-149) but parseObject reads bools
    (FieldMaskUtil.h:441-450), and readBool throws INVALID_DATA
    (BinaryProtocol-inl.h:489-495)."""
    name, protocol, _table, wire, n, limits, _code = case
    st, _, _, _ = oracle.skim(protocol, wire, [0, len(wire)], 1, 8, limits)
    dst, _, _, _, _ = oracle.decode(ANY, protocol, wire, 1, offsets=np.array([0, len(wire)],
                                                                            np.uint64),
                                    limits=limits)
    if name in ("binary_bool_2", "binary_bool_66"):
        assert dst.code == 0 and (st.code, st.byte_offset) == (3, 3), name
        return
    assert st.as_tuple() == dst.as_tuple(), name


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["flat8_binary", "mixed_compact", "nested_binary",
                                  "maps_compact_v1", "unions_compact"])
def test_gpu_skim_stream(gpu, name):
    """Unindexed stream: schemaless index, then skim — the golden index and
    the oracle's entries."""
    import torch

    from fbthrift_amd import serializer as S

    c = helpers.Case(name)
    ser = {0: S.BinarySerializer, 2: S.CompactSerializer, 0x102: S.CompactV1Serializer}[c.protocol]
    w = torch.from_numpy(np.frombuffer(c.wire, np.uint8).copy()).to(gpu)
    offs, fields, counts, n = ser.skim_stream(w, max_fields=32)
    assert n == c.n
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), c.offsets)
    ost, ofields, ocounts, _ = oracle.skim(c.protocol, c.wire, c.offsets, c.n, 32)
    got = S.skim_records(fields, n, 32)
    cnt = counts.cpu().numpy()
    assert np.array_equal(cnt, ocounts)
    for i in range(n):
        assert np.array_equal(got[i, :cnt[i]], ofields[i, :cnt[i]])
