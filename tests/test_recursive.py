"""Recursive schemas, boxed struct fields and struct / container map keys.

Reference semantics:
  * cpp.ref / @thrift.Box fields (TGPU_BOXED, TGPU_OPTIONAL_BOXED): read into a
    fresh object that the member points to once its read completed
    (module_types_custom_protocol_h/deserialize_field.whisker:21-23,49-51);
    written always (unqualified; a null pointer as an empty struct,
    serialize_field.whisker:32-50) or when set (optional).
  * struct nesting consumes no protocol height (readStructBegin does not
    descend; BinaryProtocol.h:371-372 / CompactProtocol.h:427-428 keep
    beforeSubobject empty), containers do (Protocol.h:59-78): a tree through
    list<Tree> hits DEPTH_LIMIT at max_depth, a boxed chain does not.
  * map keys of any type (TableBasedSerializerImpl.h:300-407): the pair is
    inserted once key and value are read (EncodeHelpers.h:188-205).

The golden streams (tests/golden: keyed_*, tree_*, chain_*) are written by the
reference's Python protocols and checked in test_nested_containers.py; here
the hand-derived bytes of null pointers, schema validation, and records nested
far past the device's private frames (the deep pass with HBM frames)."""
import sys

import numpy as np
import pytest

import nested_helpers as nh
from fbthrift_amd import _lib
from fbthrift_amd.schema import BOXED, OPTIONAL_BOXED, Schema, layout_compute_c
from oracle import oracle

T_I32, T_I64, T_STRING, T_STRUCT, T_LIST = 8, 10, 11, 12, 15

CHAIN = [
    [[1, T_I64, 0, 0, -1], [2, T_STRUCT, 0, OPTIONAL_BOXED, 0], [3, T_STRUCT, 0, BOXED, 1]],
    [[1, T_I32, 0, 0, -1], [2, T_STRING, 0, 1, -1]],
]
TREE = [[[1, T_I32, 0, 0, -1], [2, T_LIST, T_STRUCT, 0, 0], [3, T_STRING, 0, 0, -1]]]


class Case:
    """A NestedCase built from a table and values (the oracle writes the
    stream)."""

    def __init__(self, table, values, protocol):
        self.name, self.n, self.protocol = "local", len(values), protocol
        self.table, self.values = table, values
        self.schema = Schema.from_table(table)
        self.layout = nh.Layout(self.schema, table)
        rec, sb, lb = nh.pack(self)
        st, wire, offs = oracle.encode(self.schema, protocol, rec, self.n, sb, lb)
        assert st.code == 0, st.as_tuple()
        self.wire, self.offsets = wire, offs


def chain(n, seed=1):
    node = None
    for k in range(n + 1):
        node = [seed * 1000 + k, node, [k, ("n%d" % k).encode().hex() if k % 3 else None]]
    return node


def tree(depth):
    return [depth, [tree(depth - 1)] if depth else [], bytes([depth % 251]).hex()]


@pytest.fixture(autouse=True)
def _deep_python():
    old = sys.getrecursionlimit()
    sys.setrecursionlimit(50000)
    yield
    sys.setrecursionlimit(old)


def test_boxed_layout():
    """A boxed member is a 16-byte span (the pointer), so a struct can hold
    itself through it; tgpu_layout_compute agrees with the Python rule."""
    s = Schema.from_table(CHAIN)
    assert s.size[0] == 8 + 16 + 16 + 8  # i64, 2 spans, 3 isset bytes padded
    structs, fields = layout_compute_c(s)
    assert structs[0][2] == s.size[0]
    assert [f[0] for f in fields[:3]] == [0, 8, 24]


def test_by_value_recursion_has_no_layout():
    import ctypes

    structs = (_lib.StructDesc * 1)()
    fields = (_lib.FieldDesc * 1)()
    structs[0].num_fields = 1
    fields[0].id, fields[0].ttype, fields[0].struct_index = 1, T_STRUCT, 0
    rc = _lib.lib().tgpu_layout_compute(ctypes.addressof(structs), 1, ctypes.addressof(fields), 1)
    assert _lib.CODES[rc] == "UNSUPPORTED"
    fields[0].qualifier = BOXED  # through a pointer it has one
    rc = _lib.lib().tgpu_layout_compute(ctypes.addressof(structs), 1, ctypes.addressof(fields), 1)
    assert rc == 0 and structs[0].size == 24 and fields[0].isset_offset == 16


@pytest.mark.parametrize("protocol", [0, 2])
def test_oracle_null_pointers(protocol):
    """Node{v=5, next unset (optional box), leaf = null cpp.ref}: the null
    unqualified ref is written as an empty struct (field header + STOP); read
    back, the member points to a fresh, empty object."""
    s = Schema.from_table(CHAIN)
    rec = np.zeros(s.size[0], np.uint8)
    rec[:8] = np.frombuffer((5).to_bytes(8, "little"), np.uint8)
    rec[s.isset[(0, 0)]] = 1
    rec[s.isset[(0, 2)]] = 1  # isset of a BOXED field plays no part in the write
    st, wire, _ = oracle.encode(s, protocol, rec, 1, np.zeros(1, np.uint8), np.zeros(8, np.uint8))
    assert st.code == 0
    want = (bytes.fromhex("0a0001 0000000000000005 0c0003 00 00") if protocol == 0
            else bytes.fromhex("16 0a 2c 00 00"))  # Compact: i64 zigzag(5) = 10; delta 2
    assert wire == want
    st, out, arena, nd, _ = oracle.decode(s, protocol, wire, 1)
    assert st.code == 0 and nd == 1
    off, length = np.frombuffer(out[24:40].tobytes(), "<u8")[0], out[32]
    assert length == 1 and not arena[off:off + s.size[1]].any()
    assert out[s.isset[(0, 1)]] == 0 and out[s.isset[(0, 2)]] == 1


@pytest.mark.parametrize("protocol", [0, 2])
def test_oracle_round_trips_deep_records(protocol):
    c = Case(CHAIN, [chain(5), chain(300), chain(0)], protocol)
    st, rec, arena, nd, _ = oracle.decode(c.schema, protocol, c.wire, c.n)
    assert st.code == 0 and nh.materialize_batch(c, rec, arena) == c.values
    t = Case(TREE, [tree(3), tree(150)], protocol)
    st, rec, arena, nd, _ = oracle.decode(t.schema, protocol, t.wire, t.n)
    assert st.code == 0 and nh.materialize_batch(t, rec, arena) == t.values
    # containers count toward the height: a 150-level tree needs max_depth > 150
    st = oracle.decode(t.schema, protocol, t.wire, t.n, limits=(0, 0, 100, 0))[0]
    assert st.code == 8 and st.record == 1  # DEPTH_LIMIT


# ---- GPU ----------------------------------------------------------------------
def _gpu_schema_rc(structs, fields, types=()):
    import ctypes

    ns, nf = len(structs), len(fields)
    S = (_lib.StructDesc * ns)(*structs)
    F = (_lib.FieldDesc * max(nf, 1))(*fields)
    Tt = (_lib.TypeDesc * max(len(types), 1))(*types)
    h = ctypes.c_void_p()
    rc = _lib.lib().tgpu_schema_create_ex(ctypes.addressof(S), ns, ctypes.addressof(F), nf,
                                          ctypes.addressof(Tt), len(types), ctypes.byref(h))
    if rc == 0:
        _lib.lib().tgpu_schema_destroy(h)
    return _lib.CODES.get(rc, rc)


def _fd(id, ttype, elem=0, q=0, si=-1, val=0, member=0, isset=0, ti=0, ki=0):
    f = _lib.FieldDesc()
    f.id, f.ttype, f.elem_ttype, f.qualifier, f.struct_index = id, ttype, elem, q, si
    f.val_ttype, f.member_offset, f.isset_offset, f.type_index, f.key_index = val, member, isset, ti, ki
    return f


def _sd(first, n, size, align):
    s = _lib.StructDesc()
    s.first_field, s.num_fields, s.size, s.align = first, n, size, align
    return s


def _td(ttype, elem=0, val=0, si=-1, ti=0, ki=0):
    t = _lib.TypeDesc()
    t.ttype, t.elem_ttype, t.val_ttype, t.struct_index, t.type_index, t.key_index = (
        ttype, elem, val, si, ti, ki)
    return t


@pytest.mark.gpu
def test_gpu_schema_validation(gpu):
    # recursive through a boxed field and through a list: accepted
    assert _gpu_schema_rc([_sd(0, 2, 32, 8)],
                          [_fd(1, T_I32, member=0, isset=24),
                           _fd(2, T_STRUCT, q=OPTIONAL_BOXED, si=0, member=8, isset=25)]) == "OK"
    assert _gpu_schema_rc([_sd(0, 1, 24, 8)], [_fd(1, T_LIST, T_STRUCT, si=0, isset=16)]) == "OK"
    # a struct holding itself by value: no layout
    assert _gpu_schema_rc([_sd(0, 1, 8, 8)], [_fd(1, T_STRUCT, si=0, isset=0)]) == "UNSUPPORTED"
    # boxed on a non-struct field
    assert _gpu_schema_rc([_sd(0, 1, 24, 8)],
                          [_fd(1, T_STRING, q=BOXED, isset=16)]) == "UNSUPPORTED"
    # key_index on a list; a map's struct key without its key node
    assert _gpu_schema_rc([_sd(0, 1, 24, 8)], [_fd(1, T_LIST, T_I32, isset=16, ki=1)],
                          [_td(T_STRUCT, si=0)]) == "INVALID_ARGUMENT"
    assert _gpu_schema_rc([_sd(0, 1, 24, 8)],
                          [_fd(1, 13, T_STRUCT, val=T_I32, isset=16)]) == "INVALID_ARGUMENT"
    # a map<Self, i32> key: accepted; a cycle of type nodes alone: rejected
    assert _gpu_schema_rc([_sd(0, 1, 24, 8)], [_fd(1, 13, T_STRUCT, val=T_I32, isset=16, ki=1)],
                          [_td(T_STRUCT, si=0)]) == "OK"
    assert _gpu_schema_rc([_sd(0, 1, 24, 8)], [_fd(1, T_LIST, T_LIST, isset=16, ti=1)],
                          [_td(T_LIST, T_LIST, ti=1)]) == "INVALID_ARGUMENT"


def nh_gpu():
    import test_nested_containers as tn

    return tn


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
@pytest.mark.parametrize("indexed", [False, True])
@pytest.mark.parametrize("wide", ["1", "0"])
def test_gpu_deep_records(gpu, protocol, indexed, wide, monkeypatch):
    """Records nested far past the private frames: boxed chains (no height)
    and list trees (height), decoded and encoded by the deep passes — with
    their wide tier (kWideFrames frames a lane: chain(2000) and tree(400)
    nest past it and go on to the max_depth lanes) and without it
    (TGPU_DEEP_WIDE=0); the device matches the oracle byte for byte
    (records, arena, wire)."""
    monkeypatch.setenv("TGPU_DEEP_WIDE", wide)
    tn = nh_gpu()
    vals = [chain(i % 7) for i in range(300)] + [chain(2000), chain(40)] + \
           [chain(i % 11) for i in range(300)]
    for c in (Case(CHAIN, vals, protocol),
              Case(TREE, [tree(i % 9) for i in range(200)] + [tree(400), tree(12)], protocol)):
        offs = c.offsets if indexed else None
        st, rec, arena, nd, cons = tn._gpu_decode(c, c.wire, c.n, offs, gpu)
        assert st.code == 0 and nd == c.n and cons == len(c.wire), st.as_tuple()
        ost, orec, oarena, _, _ = oracle.decode(c.schema, protocol, c.wire, c.n, offsets=offs)
        S = c.layout.size[0]
        assert np.array_equal(rec[: c.n * S], orec[: c.n * S])
        assert np.array_equal(arena[: oarena.size], oarena)
        r, sb, lb = nh.pack(c)
        from fbthrift_amd.serializer import GpuSchema

        gs = GpuSchema(c.schema)
        Ser = tn._ser(protocol)
        out, o = Ser.serialize(gs, tn._t(r, gpu), c.n, tn._t(sb, gpu), tn._t(lb, gpu))
        assert bytes(out.cpu().numpy()) == c.wire


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_gpu_depth_limit_parity(gpu, protocol):
    """A tree deeper than max_depth: the oracle's DEPTH_LIMIT status, record
    and offset, and the same partial records before it."""
    tn = nh_gpu()
    c = Case(TREE, [tree(5), tree(30), tree(80), tree(3)], protocol)
    for lim in ((0, 0, 50, 0), (0, 0, 12000, 40), (0, 0, 20, 0)):
        st, rec, arena, nd, cons = tn._gpu_decode(c, c.wire, c.n, None, gpu, limits=lim)
        ost, orec, oarena, ond, ocons = oracle.decode(c.schema, protocol, c.wire, c.n, limits=lim)
        assert st.as_tuple() == ost.as_tuple() and (nd, cons) == (ond, ocons), lim
        S = c.layout.size[0]
        assert np.array_equal(rec[: nd * S], orec[: nd * S])
