"""Unknown values nested deeper than a lane's private skip frames.

The reference skips an unknown field recursively down to
FLAGS_thrift_protocol_max_depth = 12000 (thrift/lib/cpp2/protocol/
Protocol.cpp:21-29; the depth check in BinaryProtocol.cpp:140-143 and the
generic skip of Protocol.h:187-283). The device skip keeps 16 frames per lane
and defers a deeper value to a pass whose lanes keep max_depth frames in HBM
(DESIGN.md §4.6), so the status, record and byte offset must equal the
oracle's (a recursive restatement) at every depth up to the limit and one
past it: decode (indexed and unindexed), the schemaless index and the skim.
"""
import numpy as np
import pytest

from fbthrift_amd.schema import Schema
from oracle import oracle
from wire import B, C, W

I64, BYTE, STRUCT, LIST, SET, MAP = 10, 3, 12, 15, 14, 13
SCHEMA = [[[1, I64, 0, 0, -1], [2, I64, 0, 0, -1]]]
ANY = [[]]
DEPTHS = [0, 7, 8, 9, 15, 16, 17, 33, 100, 1000, 5900]


def deep_value(w, ttype, depth):
    """A value of `ttype` holding `depth` further levels of the same kind
    (the innermost level holds one byte), so the skip reaches depth + 1."""
    if ttype == STRUCT:
        for _ in range(depth):
            w.struct_begin().field(STRUCT, 7)
        w.struct_begin().field(BYTE, 3).byte(9).struct_end()
        for _ in range(depth):
            w.struct_end()
    elif ttype in (LIST, SET):
        for _ in range(depth):
            w.list_begin(ttype, 1)
        w.list_begin(BYTE, 1).byte(9)
    else:  # map<byte, map<...>>
        for _ in range(depth):
            w.map_begin(BYTE, MAP, 1).byte(1)
        w.map_begin(BYTE, BYTE, 1).byte(1).byte(9)


def record(proto, k, depth=None, ttype=STRUCT):
    """{1: k, [99: <deep unknown value>], 2: -k}: the unknown field sits
    between two known ones, so its skip decides where field 2 is read."""
    w = W(proto).field(I64, 1).i64(k)
    if depth is not None:
        w.field(ttype, 99)
        deep_value(w, ttype, depth)
    return w.field(I64, 2).i64(-k).stop().bytes()


def stream(proto, n, deep_at, ttype=STRUCT):
    recs = [record(proto, k, deep_at.get(k), ttype) for k in range(n)]
    offs = np.cumsum([0] + [len(r) for r in recs]).astype(np.uint64)
    return b"".join(recs), offs


def limit_boundary(proto, ttype):
    """The smallest nesting the oracle rejects (DEPTH_LIMIT) for this shape:
    the skip's depth check and the struct/container height counter
    (Protocol.h:59-78, setHeight = max_depth + 1) both apply."""
    schema = Schema.from_table(SCHEMA)

    def code(d):
        return oracle.decode(schema, proto, stream(proto, 1, {0: d}, ttype)[0], 1)[0].code

    lo, hi = 0, 12001  # code(lo) == 0, code(hi) == DEPTH_LIMIT
    assert code(lo) == 0 and code(hi) == 8
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if code(mid):
            hi = mid
        else:
            lo = mid
    return hi


def _ser(proto):
    from fbthrift_amd import serializer as S

    return {B: S.BinarySerializer, C: S.CompactSerializer}[proto]


def _dev(b, gpu):
    import torch

    return torch.from_numpy(np.frombuffer(b, np.uint8).copy()).to(gpu)


# ---- oracle (CPU): the restatement's own depth semantics ---------------------
@pytest.mark.parametrize("proto", [B, C])
@pytest.mark.parametrize("ttype", [STRUCT, LIST, SET, MAP])
def test_oracle_deep_unknown_field(proto, ttype):
    schema = Schema.from_table(SCHEMA)
    for d in (33, 1000, limit_boundary(proto, ttype) - 1):
        wire, offs = stream(proto, 3, {1: d}, ttype)
        st, rec, _, nd, cons = oracle.decode(schema, proto, wire, 3)
        assert st.code == 0 and nd == 3 and cons == len(wire), (d, st.as_tuple())
        vals = rec[: 3 * schema.record_size].view(np.int64).reshape(3, -1)[:, :2]
        assert vals.tolist() == [[0, 0], [1, -1], [2, -2]]
    # a value nested past max_depth: DEPTH_LIMIT inside record 1
    assert 5900 < limit_boundary(proto, ttype) <= 12000
    wire, _ = stream(proto, 3, {1: limit_boundary(proto, ttype)}, ttype)
    st, _, _, nd, _ = oracle.decode(schema, proto, wire, 3)
    assert st.code == 8 and nd == 1 and st.record == 1


# ---- GPU parity ----------------------------------------------------------------
def _parity(gpu, proto, wire, n, offs, limits=None, indexed=False):
    schema = Schema.from_table(SCHEMA)
    from fbthrift_amd.serializer import GpuSchema

    o = _dev(offs.astype(np.int64).tobytes(), gpu).view(__import__("torch").int64)
    rec, _, st, nd, cons = _ser(proto).deserialize_status(
        GpuSchema(schema), _dev(wire, gpu), n, o if indexed else None, limits)
    ost, orec, _, ond, ocons = oracle.decode(schema, proto, wire, n,
                                             offsets=offs if indexed else None, limits=limits)
    assert st.as_tuple() == ost.as_tuple()
    assert (nd, cons) == (ond, ocons)
    k = (nd + (1 if st.code else 0)) * schema.record_size
    assert np.array_equal(rec.cpu().numpy()[:k], orec[:k])
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [B, C])
@pytest.mark.parametrize("ttype", [STRUCT, LIST, SET, MAP])
@pytest.mark.parametrize("indexed", [False, True])
def test_gpu_deep_unknown_fields(gpu, codec, proto, ttype, indexed):
    """Deep unknown fields scattered through a stream of ordinary records,
    depths around the private frame count and up to the reference limit."""
    n = 600
    b = limit_boundary(proto, ttype)
    deep_at = {5 + 50 * j: d for j, d in enumerate(DEPTHS + [b - 2, b - 1])}
    wire, offs = stream(proto, n, deep_at, ttype)
    st = _parity(gpu, proto, wire, n, offs, indexed=indexed)
    assert st.code == 0


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [B, C])
@pytest.mark.parametrize("ttype", [STRUCT, LIST, MAP])
@pytest.mark.parametrize("indexed", [False, True])
def test_gpu_deep_past_max_depth(gpu, codec, proto, ttype, indexed):
    """One level past FLAGS_thrift_protocol_max_depth: DEPTH_LIMIT at the
    reference's record and byte offset; earlier deep records still decode."""
    n = 300
    b = limit_boundary(proto, ttype)
    wire, offs = stream(proto, n, {3: 5000, 50: b - 1, 77: b, 200: 40}, ttype)
    st = _parity(gpu, proto, wire, n, offs, indexed=indexed)
    assert st.code == 8 and st.record == 77


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [B, C])
@pytest.mark.parametrize("max_depth", [20, 64])
def test_gpu_deep_custom_limit(gpu, codec, proto, max_depth):
    n = 200
    deep_at = {10: max_depth - 3, 60: max_depth - 2, 120: max_depth - 1, 150: max_depth + 5}
    wire, offs = stream(proto, n, deep_at)
    for indexed in (False, True):
        st = _parity(gpu, proto, wire, n, offs, limits=(0, 0, max_depth, 0), indexed=indexed)
        assert st.code == 8


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [B, C])
def test_gpu_deep_index_and_skim(gpu, proto):
    """The schemaless index (every field skipped) and the skim walk deep
    values exactly like the oracle's sequential skip."""
    import torch

    from fbthrift_amd import serializer as S

    n = 2000
    deep_at = {7 * j + 3: d for j, d in enumerate([17, 40, 300, 2500, 11997] * 40)}
    wire, offs = stream(proto, n, deep_at, STRUCT)
    ser = _ser(proto)
    w = _dev(wire, gpu)
    got, m, first, last, st = ser.index_stream(S.GpuSchema(Schema.from_table(ANY)), w)
    assert st.code == 0 and m == n and last == len(wire)
    assert np.array_equal(got.cpu().numpy()[: n + 1].astype(np.uint64), offs)
    # field-table skim of the same records
    ost, ofields, ocounts, odone = oracle.skim(proto, wire, offs, n, max_fields=4)
    t_offs = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    fields, counts, done, sst = ser.skim(w, t_offs, n, max_fields=4, check=False)
    assert sst.as_tuple() == ost.as_tuple() and done == odone
    assert np.array_equal(counts.cpu().numpy()[:n], ocounts)
    got_f = S.skim_records(fields, n, 4)
    assert np.array_equal(got_f, ofields)


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [B, C])
def test_gpu_deep_skim_past_limit(gpu, proto):
    import torch

    n = 100
    wire, offs = stream(proto, n, {4: 300, 50: 12000})
    ost, ofields, ocounts, odone = oracle.skim(proto, wire, offs, n, max_fields=4)
    assert ost.code == 8 and ost.record == 50
    t_offs = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    fields, counts, done, sst = _ser(proto).skim(_dev(wire, gpu), t_offs, n, max_fields=4,
                                                 check=False)
    assert sst.as_tuple() == ost.as_tuple() and done == odone
