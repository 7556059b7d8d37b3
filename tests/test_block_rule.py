"""The block rule (round 6): list / set element arrays of flat-list schemas
are dense per block of 64 records (thrift_gpu.h tgpu_schema_arena_scale),
the way the reference reads each list into its own std::vector
(protocol_methods.h:390-441 -> readArithmeticVector, BinaryProtocol.cpp:
49-72). The oracle restates it (thrift_oracle.cpp pack_blocks); these tests
pin the rule's properties on the oracle and hold the device to the oracle's
records byte for byte — span offsets included — on streams that mix blocks
the compiled decode tile packs itself with blocks the general decoder reads
(records off the canonical field order), in both protocols, through the
compiled and the interpreting kernels, indexed, unindexed and through the
host chunk pipeline, and on a stream that fails inside a list."""
import functools
import os
import sys

import numpy as np
import pytest

import helpers
from fbthrift_amd.schema import Schema
from oracle import oracle

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import datagen  # noqa: E402

BLOCK = 64
T_BOOL, T_I16, T_I32, T_I64, T_DOUBLE, T_LIST, T_SET, T_STRUCT = 2, 6, 8, 10, 4, 15, 14, 12
# Rec {1: list<i32> a; 2: i64 x; 3: Inner in; 4: list<double> d}
# Inner {1: set<i16> s; 2: list<bool> b}
MULTI = [[[1, T_LIST, T_I32, 0, -1], [2, T_I64, 0, 0, -1], [3, T_STRUCT, 0, 0, 1],
          [4, T_LIST, T_DOUBLE, 0, -1]],
         [[1, T_SET, T_I16, 0, -1], [2, T_LIST, T_BOOL, 0, -1]]]
SCHEMAS = {"nested": datagen.SCHEMAS["nested"], "multi": MULTI}
NP = {T_I32: np.int32, T_I64: np.int64, T_DOUBLE: np.float64, T_I16: np.int16, T_BOOL: np.uint8}


def _values(table, i, rng):
    """Record i's values: {field id: value}; lists of 0..17 elements (a few
    lanes past 64 bytes of arrays, which the decode tile leaves to the
    packing pass)."""
    def struct(si):
        out = {}
        for fid, t, e, _, sub in (f[:5] for f in table[si]):
            if t == T_STRUCT:
                out[fid] = struct(sub)
            elif t in (T_LIST, T_SET):
                n = int(rng.integers(0, 18 if i % 13 else 3))
                if e == T_BOOL:
                    v = [int(x) for x in rng.integers(0, 2, n)]
                elif e == T_DOUBLE:
                    v = [float(x) for x in rng.standard_normal(n)]
                else:
                    lim = {T_I16: 1 << 15, T_I32: 1 << 31, T_I64: 1 << 62}[e]
                    v = [int(x) for x in rng.integers(-lim, lim, n)]
                    if t == T_SET:
                        v = sorted(set(v))
                out[fid] = v
            elif t == T_DOUBLE:
                out[fid] = float(rng.standard_normal())
            else:
                out[fid] = int(rng.integers(-(1 << 62), 1 << 62))
        return out
    return struct(0)


def _pack(table, schema, vals, order):
    """Records of `schema` (its fields declared in `order` of ids) + the list
    base holding every array."""
    n = len(vals)
    rec = np.zeros(n, dtype=schema.dtype())
    base = []
    pos = [0]

    def put(arr, si, v, sub_schema_rows):
        for k, row in enumerate(sub_schema_rows):
            fid, t, e = row[0], row[1], row[2]
            name = "f%d" % fid
            x = v[fid]
            if t == T_STRUCT:
                put(arr[name], row[4], x, [r for r in table[row[4]]])
            elif t in (T_LIST, T_SET):
                a = np.asarray(x, dtype=NP[e])
                arr[name]["offset"] = pos[0] if len(a) else 0
                arr[name]["length"] = len(a)
                base.append(a.view(np.uint8))
                pos[0] += a.nbytes
            else:
                arr[name] = x
            arr["__isset"][k] = 1

    rows0 = [next(r for r in table[0] if r[0] == fid) for fid in order]
    for i in range(n):
        put(rec[i], 0, vals[i], rows0)
    lb = np.concatenate(base) if base else np.zeros(1, np.uint8)
    return rec.view(np.uint8), lb


@functools.lru_cache(maxsize=16)
def stream(name, protocol, n, every=0, seed=5):
    """n records of schema `name`; record i written with its root fields in
    another order when every and i % every == 0 (the general reader's
    record). Returns (schema, wire bytes, offsets)."""
    table = SCHEMAS[name]
    rng = np.random.default_rng(seed)
    vals = [_values(table, i, rng) for i in range(n)]
    ids = [r[0] for r in table[0]]
    schema = Schema.from_table(table)
    rec, lb = _pack(table, schema, vals, ids)
    st, wire, offs = oracle.encode(schema, protocol, rec, n, None, lb)
    assert st.code == 0
    if not every:
        return schema, wire, np.asarray(offs, np.uint64)
    perm = ids[1:] + ids[:1]
    t2 = [[next(r for r in table[0] if r[0] == fid) for fid in perm]] + table[1:]
    s2 = Schema.from_table(t2)
    rec2, lb2 = _pack(t2, s2, vals, perm)
    st, wire2, offs2 = oracle.encode(s2, protocol, rec2, n, None, lb2)
    assert st.code == 0
    parts, o = [], [0]
    for i in range(n):
        w, f = (wire2, offs2) if i % every == 0 else (wire, offs)
        parts.append(w[int(f[i]):int(f[i + 1])])
        o.append(o[-1] + len(parts[-1]))
    return schema, b"".join(parts), np.asarray(o, np.uint64)


# ---- the rule on the oracle (CPU) ---------------------------------------------
def _arrays(schema, rec, n):
    """Per record: [(span offset, bytes)] of its list / set members."""
    dt = schema.dtype()
    r = np.frombuffer(rec[: n * schema.record_size].tobytes(), dt)
    out = []
    for i in range(n):
        row = []

        def walk(x, si):
            for f in schema.structs[si].fields:
                if f.ttype == T_STRUCT:
                    walk(x[f.name], schema.struct_index(f.struct))
                elif f.ttype in (T_LIST, T_SET):
                    w = {T_I32: 4, T_I64: 8, T_DOUBLE: 8, T_I16: 2, T_BOOL: 1}[f.elem_ttype]
                    row.append((int(x[f.name]["offset"]), int(x[f.name]["length"]) * w))
        walk(r[i], 0)
        out.append(row)
    return out


@pytest.mark.parametrize("name", sorted(SCHEMAS))
@pytest.mark.parametrize("protocol", [0, 2])
@pytest.mark.parametrize("every", [0, 7])
def test_oracle_block_rule(name, protocol, every):
    """Each block's arrays: 8-byte aligned, back to back in record order
    from align8(scale x the block's first wire byte), inside the block's
    wire bytes x scale; the values are those the position rule read."""
    n = 333
    schema, wire, offs = stream(name, protocol, n, every)
    scale = oracle.arena_scale(schema, protocol)
    st, rec, arena, nd, _ = oracle.decode(schema, protocol, wire, n, offsets=offs)
    assert st.code == 0 and nd == n
    arrs = _arrays(schema, rec, n)
    for b0 in range(0, n, BLOCK):
        cur = (scale * int(offs[b0]) + 7) & ~7
        hi = scale * int(offs[min(n, b0 + BLOCK)])
        for i in range(b0, min(n, b0 + BLOCK)):
            for off, nbytes in sorted(a for a in arrs[i] if a[1]):
                cur = (cur + 7) & ~7
                assert off == cur, (i, off, cur)
                cur += nbytes
        assert cur <= hi
    # the values: writing the records back from the packed arrays gives the
    # stream (as written by the canonical writer: the reordered records come
    # back in declaration order)
    est, again, aoffs = oracle.encode(schema, protocol, rec, n, None, arena)
    assert est.code == 0
    if not every:
        assert again == wire
    else:
        canon = stream(name, protocol, n)[1]
        assert again == canon
    st2, rec2, arena2, _, _ = oracle.decode(schema, protocol, wire, n)  # unindexed: same rule
    assert np.array_equal(rec, rec2)


# ---- the device against the oracle ----------------------------------------------
def _gpu_decode(dev, schema, protocol, wire, n, offsets):
    import torch

    from fbthrift_amd import serializer as S

    ser = {0: S.BinarySerializer, 2: S.CompactSerializer}[protocol]
    gs = S.GpuSchema(schema)
    w = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).to(dev)
    o = None if offsets is None else torch.from_numpy(offsets.astype(np.int64)).to(dev)
    rec, arena, st, nd, cons = ser.deserialize_status(gs, w, n, o)
    return st, rec.cpu().numpy(), arena.cpu().numpy(), nd, cons


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCHEMAS))
@pytest.mark.parametrize("protocol", [0, 2])
@pytest.mark.parametrize("every", [0, 97])
@pytest.mark.parametrize("indexed", [True, False])
def test_gpu_block_rule_matches_oracle(gpu, codec, name, protocol, every, indexed):
    """Records (span offsets included) equal the oracle's; the arena bytes
    the spans describe too. 20 003 records (TGPU_JIT=1 compiles the schema
    whatever the batch): the compiled tile packs the canonical waves' blocks
    and the packing pass the blocks holding a reordered record (every 97th)
    or a record with more than 64 bytes of arrays; TGPU_JIT=0 leaves every
    block to the packing pass."""
    n = 20_003
    schema, wire, offs = stream(name, protocol, n, every)
    o = offs if indexed else None
    st, rec, arena, nd, cons = _gpu_decode(gpu, schema, protocol, wire, n, o)
    assert st.code == 0 and nd == n and cons == len(wire), st.as_tuple()
    ost, orec, oarena, _, _ = oracle.decode(schema, protocol, wire, n, offsets=o)
    S = schema.record_size
    assert np.array_equal(rec[: n * S], orec[: n * S])
    helpers.assert_arena_equal(schema, orec, n, wire, arena, oarena)


@pytest.mark.gpu
@pytest.mark.parametrize("every", [0, 97])
@pytest.mark.parametrize("indexed", [True, False])
def test_gpu_block_rule_record_tile(gpu, monkeypatch, every, indexed):
    """The compiled Binary tile with an LDS record tile (TGPU_DECODE_REGREC=0
    on config 4's schema, whose default keeps records in registers): every
    wave's span rewrite lands before the tile's records leave in 16-byte
    chunks that cross the waves (a missing barrier there, round 6)."""
    monkeypatch.setenv("TGPU_JIT", "1")
    monkeypatch.setenv("TGPU_DECODE_REGREC", "0")
    n = 20_003
    schema, wire, offs = stream("nested", 0, n, every)
    o = offs if indexed else None
    st, rec, arena, nd, cons = _gpu_decode(gpu, schema, 0, wire, n, o)
    assert st.code == 0 and nd == n and cons == len(wire), st.as_tuple()
    ost, orec, oarena, _, _ = oracle.decode(schema, 0, wire, n, offsets=o)
    S = schema.record_size
    assert np.array_equal(rec[: n * S], orec[: n * S])
    helpers.assert_arena_equal(schema, orec, n, wire, arena, oarena)


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_gpu_block_rule_failing_list(gpu, protocol):
    """A stream cut inside a list of record 5000: the oracle's status, the
    records before it and the failing record (its list resized, zero-filled
    past the cut) as the oracle packs them."""
    n = 9000
    schema, wire, offs = stream("nested", protocol, n)
    cut = int(offs[5000]) + 14
    st, rec, arena, nd, _ = _gpu_decode(gpu, schema, protocol, wire[:cut], n, None)
    ost, orec, oarena, ond, _ = oracle.decode(schema, protocol, wire[:cut], n)
    assert st.as_tuple() == ost.as_tuple() and nd == ond == 5000
    k = (nd + 1) * schema.record_size
    assert np.array_equal(rec[:k], orec[:k])
    helpers.assert_arena_equal(schema, orec, nd, wire[:cut], arena, oarena)


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_gpu_block_rule_host_chunks(gpu, protocol):
    """The host chunk pipeline (small pieces: many ranges) hands back whole
    blocks, so its records and arena equal the resident pass's — the
    oracle's."""
    from fbthrift_amd.serializer import GpuSchema
    from test_gpu_host import _decode_chunks

    n = 20_000
    schema, wire, offs = stream("nested", protocol, n, every=211)
    gs = GpuSchema(schema)
    S = schema.record_size
    scale = oracle.arena_scale(schema, protocol)
    rec, arena, st, nd, cons, ranges = _decode_chunks(gs, protocol, wire, n, 64 << 10, scale)
    assert st.code == 0 and nd == n and len(ranges) > 10, st.as_tuple()
    assert all(a % BLOCK == 0 for a, _ in ranges)
    ost, orec, oarena, _, _ = oracle.decode(schema, protocol, wire, n)
    assert np.array_equal(rec, orec[: n * S])
    helpers.assert_arena_equal(schema, orec, n, wire, arena, oarena)
