"""Nested record programs for the shapes round 3 left on the general
reader: boxed struct fields (cpp.ref / thrift.box, unqualified and optional),
struct and container map keys, and bools inside maps (Compact writes a
container bool as a byte 1 / 2, CompactProtocol-inl.h:692-701; Binary as
0 / 1, a byte >= 2 throws). Recursive schemas (tree / chain) have no finite
straight-line program: theirs unrolls a bounded number of struct levels,
and a record nesting deeper reaches a VOP_DEFER and goes to the general
decoder (decode and index only; such programs have no writer).

Reference semantics: deserialize_field.whisker:21-23,49-51 (a boxed field's
fresh object, pointed to once read), serialize_field.whisker:44-49 (a null
unqualified boxed field is written as an empty struct),
TableBasedSerializerImpl.h:300-407 (maps with struct / container keys),
EncodeHelpers.h:188-205 (pairs inserted once read).

CPU: the programs exist (compile for gfx950); recursive schemas have
unrolled ones (none with TGPU_NESTED_UNROLL=0).
GPU: the nested program's encode gives the oracle's bytes; its decode the
oracle's records and arena, indexed and unindexed, with no record left to
the general decoder (tgpu_index_stats 'general'); the general kernels
(TGPU_NESTED=0) give the same. The golden keyed_* streams (written by the
reference's Python protocols) go through the program too."""
import numpy as np
import pytest

import nested_helpers as nh
from fbthrift_amd.schema import Schema
from fbthrift_amd.serializer import compile_check
from oracle import oracle

T_BOOL, T_I16, T_I32, T_I64 = 2, 6, 8, 10
T_STRING, T_STRUCT, T_MAP, T_SET, T_LIST = 11, 12, 13, 14, 15
BOXED, OPTIONAL_BOXED = 4, 5

# S0 {1: i64 id; 2: Point at (cpp.ref); 3: optional Point near (thrift.box);
#     4: map<bool, i32> flags; 5: map<Point, bool> seen;
#     6: map<list<i16>, bool> paths}
# S1 Point {1: i32 x; 2: optional string tag}
TABLE = [
    [[1, T_I64, 0, 0, -1], [2, T_STRUCT, 0, BOXED, 1], [3, T_STRUCT, 0, OPTIONAL_BOXED, 1],
     [4, T_MAP, T_BOOL, 0, -1, T_I32], [5, T_MAP, T_STRUCT, 0, -1, T_BOOL, None,
                                        [T_STRUCT, 0, 0, 1]],
     [6, T_MAP, T_LIST, 0, -1, T_BOOL, None, [T_LIST, T_I16, 0, -1]]],
    [[1, T_I32, 0, 0, -1], [2, T_STRING, 0, 1, -1]],
]


class Case:
    """A batch of TABLE records in nested_helpers' JSON value form."""

    def __init__(self, protocol, n, seed):
        self.table = TABLE
        self.schema = Schema.from_table(TABLE)
        self.protocol, self.n = protocol, n
        self.layout = nh.Layout(self.schema, TABLE)
        rng = np.random.default_rng(seed)

        def point():
            tag = None if rng.random() < 0.4 else bytes(rng.integers(0, 256, rng.integers(0, 9),
                                                                     dtype=np.uint8)).hex()
            return [int(rng.integers(-2**31, 2**31 - 1)), tag]

        def rec(i):
            return [int(rng.integers(-2**62, 2**62)),
                    point(),
                    None if i % 3 == 0 else point(),
                    [[int(rng.integers(0, 2)), int(rng.integers(-9, 9))]
                     for _ in range(rng.integers(0, 4))],
                    [[point(), int(rng.integers(0, 2))] for _ in range(rng.integers(0, 3))],
                    [[[int(x) for x in rng.integers(-300, 300, rng.integers(0, 4))],
                      int(rng.integers(0, 2))] for _ in range(rng.integers(0, 3))]]

        self.values = [rec(i) for i in range(n)]


@pytest.mark.parametrize("protocol", [0, 2])
def test_programs_exist(protocol, monkeypatch):
    """TABLE compiles (Binary; Compact generated only), keyed has a program,
    the recursive schemas an unrolled one (none with TGPU_NESTED_UNROLL=0)."""
    rc, log = compile_check(Schema.from_table(TABLE), protocol, arch="gfx950" if protocol == 0 else "")
    assert rc == 0, log
    for name in ("keyed", "tree", "chain"):
        rc, log = compile_check(Schema.from_table(nh.manifest()["nested_schemas"][name]), protocol,
                                arch="")
        assert rc == 0, log
    monkeypatch.setenv("TGPU_NESTED_UNROLL", "0")
    for name in ("tree", "chain"):  # recursive: none
        rc, _ = compile_check(Schema.from_table(nh.manifest()["nested_schemas"][name]), protocol,
                              arch="")
        assert rc == 22


def test_oracle_round_trip():
    c = Case(2, 300, 1)
    rec, sb, lb = nh.pack(c)
    st, wire, offs = oracle.encode(c.schema, c.protocol, rec, c.n, sb, lb)
    assert st.code == 0
    c.wire = wire
    st, orec, oarena, nd, _ = oracle.decode(c.schema, c.protocol, wire, c.n)
    assert st.code == 0 and nd == c.n
    assert nh.materialize_batch(c, orec, oarena) == c.values


def _t(a, dev):
    import torch

    return torch.from_numpy(np.array(a, copy=True)).to(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_gpu_nested_shapes(gpu, protocol, monkeypatch):
    from fbthrift_amd import serializer as SZ

    c = Case(protocol, 5000, 0x5ab + protocol)
    rec, sb, lb = nh.pack(c)
    ost, owire, ooffs = oracle.encode(c.schema, protocol, rec, c.n, sb, lb)
    assert ost.code == 0
    c.wire = owire
    Ser = {0: SZ.BinarySerializer, 2: SZ.CompactSerializer}[protocol]
    S = c.layout.size[0]
    w = np.frombuffer(owire, np.uint8)
    got = {}
    for nested in ("1", "0"):
        monkeypatch.setenv("TGPU_JIT", "1")
        monkeypatch.setenv("TGPU_NESTED", nested)
        gs = SZ.GpuSchema(c.schema)
        if nested == "1":
            assert gs.compile(protocol)
        wire, offs = Ser.serialize(gs, _t(rec, gpu), c.n, _t(sb, gpu), _t(lb, gpu))
        assert wire.cpu().numpy().tobytes() == owire
        assert np.array_equal(offs.cpu().numpy().astype(np.uint64), ooffs)
        for indexed in (True, False):
            o = offs if indexed else None
            grec, garena, st, nd, cons = Ser.deserialize_status(gs, _t(w, gpu), c.n, o)
            assert st.code == 0 and nd == c.n and cons == len(owire), st.as_tuple()
            if nested == "1" and indexed:
                # every record through the nested program
                assert Ser.context().index_stats()["general"] == 0
            dst, drec, darena, _, _ = oracle.decode(c.schema, protocol, owire, c.n,
                                                    offsets=ooffs if indexed else None)
            grec, garena = grec.cpu().numpy(), garena.cpu().numpy()
            assert np.array_equal(grec[: c.n * S], drec[: c.n * S])
            assert np.array_equal(garena[: darena.size], darena)
            got[(nested, indexed)] = grec[: c.n * S]
    assert nh.materialize_batch(c, got[("1", True)], darena) == c.values


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["keyed_binary", "keyed_compact"])
def test_gpu_golden_keyed_through_the_program(gpu, name, monkeypatch):
    """The reference's keyed streams (map<Point, string>, map<list<i32>, i64>,
    map<set<string>, Point>, list<map<Point, list<i16>>>) decode through the
    nested program: no record left to the general decoder."""
    from fbthrift_amd import serializer as SZ

    monkeypatch.setenv("TGPU_JIT", "1")
    monkeypatch.setenv("TGPU_NESTED", "1")
    c = nh.NestedCase(name)
    gs = SZ.GpuSchema(c.schema)
    assert gs.compile(c.protocol)
    Ser = {0: SZ.BinarySerializer, 2: SZ.CompactSerializer}[c.protocol]
    offs = _t(c.offsets.astype(np.int64), gpu)
    rec, arena, st, nd, cons = Ser.deserialize_status(gs, _t(np.frombuffer(c.wire, np.uint8), gpu),
                                                      c.n, offs)
    assert st.code == 0 and nd == c.n
    assert Ser.context().index_stats()["general"] == 0
    assert nh.materialize_batch(c, rec.cpu().numpy(), arena.cpu().numpy()) == c.values


def _levels(name, v):
    """Struct levels of a golden tree (Tree {v, kids, tag}) / chain (Node {v,
    next, leaf}) record."""
    if name.startswith("tree"):
        return 1 + max([_levels(name, k) for k in v[1]] or [0])
    n = 0
    while v is not None:
        n, v = n + 1, v[1]
    return n


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tree_binary", "tree_compact", "chain_binary", "chain_compact"])
@pytest.mark.parametrize("unroll", [None, 6, 12])
def test_gpu_golden_recursive_through_the_program(gpu, name, unroll, monkeypatch):
    """The recursive schemas (Tree {list<Tree> kids}, Node {optional boxed
    Node next}) through their unrolled nested programs: a record whose
    structs nest deeper than the unrolled levels reaches a VOP_DEFER and is
    the general decoder's — exactly those, no other. Default unrolling: 16
    levels (Tree, 9 ops a level) / as many as fit 255 ops (Node, 18 ops a
    level: 14). Records and arena byte-equal the oracle's; the unindexed
    stream (nested index walk) the same; the records write back to the
    golden bytes through the unrolled writer (round 5), which defers exactly
    the same records to the general writer's deep pass — the path counter
    (index_stats 'general' after the encode) counts them."""
    import torch

    from fbthrift_amd import serializer as SZ

    monkeypatch.setenv("TGPU_JIT", "1")
    monkeypatch.setenv("TGPU_NESTED", "1")
    if unroll:
        monkeypatch.setenv("TGPU_NESTED_UNROLL", str(unroll))
    else:
        monkeypatch.delenv("TGPU_NESTED_UNROLL", raising=False)
    c = nh.NestedCase(name)
    k = unroll or (16 if name.startswith("tree") else 14)
    deep = sum(_levels(name, v) > k for v in c.values)
    gs = SZ.GpuSchema(c.schema)
    assert gs.compile(c.protocol)
    Ser = {0: SZ.BinarySerializer, 2: SZ.CompactSerializer}[c.protocol]
    w = _t(np.frombuffer(c.wire, np.uint8), gpu)
    offs = _t(c.offsets.astype(np.int64), gpu)
    rec, arena, st, nd, cons = Ser.deserialize_status(gs, w, c.n, offs)
    assert st.code == 0 and nd == c.n and cons == len(c.wire), st.as_tuple()
    assert Ser.context().index_stats()["general"] == deep
    assert deep < c.n
    ost, orec, oarena, ond, _ = oracle.decode(c.schema, c.protocol, c.wire, c.n,
                                              offsets=c.offsets.astype(np.uint64))
    assert ost.code == 0 and ond == c.n
    S = c.layout.size[0]
    grec, garena = rec.cpu().numpy(), arena.cpu().numpy()
    assert np.array_equal(grec[: c.n * S], orec[: c.n * S])
    assert np.array_equal(garena[: oarena.size], oarena)
    assert nh.materialize_batch(c, grec, garena) == c.values
    urec, uarena, ust, und, ucons = Ser.deserialize_status(gs, w, c.n, None)
    assert ust.code == 0 and und == c.n and ucons == len(c.wire), ust.as_tuple()
    assert nh.materialize_batch(c, urec.cpu().numpy(), uarena.cpu().numpy()) == c.values
    wire, woffs = Ser.serialize(gs, rec, c.n, w, arena)
    torch.cuda.synchronize()
    assert wire.cpu().numpy().tobytes() == c.wire
    assert np.array_equal(woffs.cpu().numpy().astype(np.uint64), c.offsets.astype(np.uint64))
    assert Ser.context().index_stats()["general"] == deep


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_gpu_bool_byte_in_map(gpu, protocol, monkeypatch):
    """A map<bool, i32> key byte 7: Binary throws (readBool, INVALID_DATA) —
    the program leaves the record to the general reader, same status; Compact
    reads it as false (byte != 1), as the general reader does."""
    from fbthrift_amd import serializer as SZ

    c = Case(protocol, 64, 3)
    for v in c.values:
        v[3] = [[1, 5]]
    rec, sb, lb = nh.pack(c)
    st, wire, offs = oracle.encode(c.schema, protocol, rec, c.n, sb, lb)
    w = bytearray(wire)
    k = 17  # record 17's flags key byte: find it as the one byte 0x01 after the map header
    b, e = int(offs[k]), int(offs[k + 1])
    hdr = bytes([0x0d, 0x00, 0x04, 0x02, 0x08, 0, 0, 0, 1]) if protocol == 0 else None
    if protocol == 0:
        at = w.index(hdr, b, e) + len(hdr)
    else:
        at = w.index(bytes([0x01, 0x15]), b, e)  # count 1, key ctype bool / value i32
        at += 2
    assert w[at] == 1
    w[at] = 7
    results = []
    for nested in ("1", "0"):
        monkeypatch.setenv("TGPU_JIT", "1")
        monkeypatch.setenv("TGPU_NESTED", nested)
        gs = SZ.GpuSchema(c.schema)
        Ser = {0: SZ.BinarySerializer, 2: SZ.CompactSerializer}[protocol]
        grec, garena, gst, nd, cons = Ser.deserialize_status(
            gs, _t(np.frombuffer(bytes(w), np.uint8), gpu), c.n,
            _t(offs.astype(np.int64), gpu))
        results.append((gst.as_tuple(), nd, cons, grec.cpu().numpy().tobytes()))
    ost, orec, _, ond, ocons = oracle.decode(c.schema, protocol, bytes(w), c.n, offsets=offs)
    assert results[0] == results[1]
    assert results[0][0] == ost.as_tuple() and results[0][1] == ond
