"""CompactV1 (TGPU_PROTOCOL_COMPACT_V1): CompactV1ProtocolReader/Writer,
thrift/lib/cpp2/protocol/CompactV1Protocol.h — the Compact protocol with
doubles written and read little-endian (CompactV1Protocol-inl.h:36-41,
73-79); every other byte is Compact's.

Golden vectors: the reference's Python TCompactProtocol at VERSION_LOW (its
V1 double order), cases *_compact_v1 in tests/golden (decode, encode and
encoded size on the GPU run through tests/test_gpu_parity.py's golden tests).
"""
import struct

import numpy as np
import pytest

import datagen
import helpers
from fbthrift_amd.schema import Schema
from oracle import oracle

V1 = 0x102


def test_v1_differs_from_compact_only_in_doubles():
    """Same values, both protocols: identical record lengths, and the bytes
    differ exactly where a double is (byte-reversed)."""
    a, b = helpers.Case("nested_compact"), helpers.Case("nested_compact_v1")
    n = b.n
    assert np.array_equal(a.offsets[:n + 1], b.offsets)
    wa, wb = a.wire[:len(b.wire)], b.wire
    diff = [i for i in range(len(wb)) if wa[i] != wb[i]]
    assert diff
    # each record's inner struct holds 3 doubles after a 1-byte header
    rec0 = wb[:int(b.offsets[1])]
    d0 = datagen.gen_nested(0)[2][0]
    assert struct.pack("<d", d0) in rec0 and struct.pack(">d", d0) in wa[:int(a.offsets[1])]


def test_v1_without_doubles_is_compact():
    a, b = helpers.Case("flat8_compact"), helpers.Case("flat8_compact_v1")
    assert a.wire[:len(b.wire)] == b.wire


def test_oracle_rejects_unknown_protocol():
    schema = Schema.from_table(datagen.SCHEMAS["flat8"])
    st, *_ = oracle.decode(schema, 3, b"\x00", 1)
    assert st.code == 23  # INVALID_ARGUMENT


@pytest.mark.gpu
def test_v1_program_selection(gpu, monkeypatch):
    """A V1 schema without doubles runs Compact's compiled program; with
    doubles its own (Compact's ops, the doubles little-endian: kFixedLE) —
    tgpu_schema_compile compiles both."""
    from fbthrift_amd.serializer import GpuSchema

    monkeypatch.setenv("TGPU_JIT", "1")  # (the compile policy, whatever the run's)

    assert GpuSchema(Schema.from_table(datagen.SCHEMAS["mixed"])).compile(V1)
    assert GpuSchema(Schema.from_table(datagen.SCHEMAS["nested"])).compile(V1)


def test_v1_program_compiles_on_cpu():
    """The CompactV1 program of a schema with doubles (flat and nested) is
    generated and compiled for gfx950 without a GPU."""
    from fbthrift_amd.serializer import compile_check

    for name in ("nested", "scalars"):
        rc, log = compile_check(Schema.from_table(datagen.SCHEMAS[name]), V1)
        assert rc == 0, log[-2000:]


@pytest.mark.gpu
def test_gpu_v1_large_nested_roundtrip(gpu):
    """A larger V1 batch with doubles (general kernels, incl. the unindexed
    stream path): GPU bytes and records equal the oracle's."""
    import torch

    from fbthrift_amd.serializer import CompactV1Serializer as S, GpuSchema

    table = datagen.SCHEMAS["nested"]
    schema = Schema.from_table(table)
    n = 40_000
    vals = datagen.flatten_values(table, [datagen.gen_nested(i) for i in range(n)])
    rec, sa, la = helpers.pack(schema, vals, n)
    ost, owire, ooffs = oracle.encode(schema, V1, rec, n, sa, la)
    assert ost.code == 0
    gs = GpuSchema(schema)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x) if x.size else np.zeros(1, np.uint8)).to(gpu)
    wire, offs = S.serialize(gs, t(rec), n, t(sa), t(la))
    assert bytes(wire.cpu().numpy()) == owire
    grec, garena, gst, gnd, gcons = S.deserialize_status(gs, t(np.frombuffer(owire, np.uint8).copy()), n)
    assert gst.code == 0 and gnd == n and gcons == len(owire)
    # no program (V1 doubles): the general speculation, its candidates and
    # every chained record filtered by the root's first header bytes, links
    # almost every chunk (it accepted false starts in 3,170 of 3,205 and the
    # one-lane repair walked the stream for 3.8 s)
    stats = S.context().index_stats()
    assert stats["broken"] * 10 < stats["chunks"], stats
    helpers.assert_values_equal(
        helpers.unpack(schema, grec.cpu().numpy(), n, owire, garena.cpu().numpy()), vals)


@pytest.mark.gpu
def test_gpu_v1_id_ordered_root_keeps_the_speculation(gpu):
    """A root written in field-id order (@SerializeInFieldIdOrder,
    t_whisker_generator.cc:232-236) while the schema declares its fields in
    another order, with a V1 double (no program: the general speculation
    filtered by the root's first header bytes). The filter takes both orders'
    first headers, so the chunks stay linked (with declaration order alone
    every true record start was rejected and the permissive fallback pass
    read the stream); records equal the oracle's."""
    import torch

    from fbthrift_amd.serializer import CompactV1Serializer as S, GpuSchema

    T_I32, T_I64, T_DOUBLE = datagen.T_I32, datagen.T_I64, datagen.T_DOUBLE
    decl = [[[2, T_DOUBLE, 0, 0, -1], [1, T_I64, 0, 0, -1], [3, T_I32, 0, 0, -1]]]
    by_id = [[[1, T_I64, 0, 0, -1], [2, T_DOUBLE, 0, 0, -1], [3, T_I32, 0, 0, -1]]]
    n = 200_000
    sb = Schema.from_table(by_id)
    vals = datagen.flatten_values(by_id, [(i * 7919 - 5, i * 0.5, (i * 31) % 1000 - 500)
                                          for i in range(n)])
    rec, sa, la = helpers.pack(sb, vals, n)
    ost, wire, _ = oracle.encode(sb, V1, rec, n, sa, la)
    assert ost.code == 0 and wire[0] == 0x16  # field 1 (i64) first
    sd = Schema.from_table(decl)
    dst, drec, _, _, _ = oracle.decode(sd, V1, wire, n)
    assert dst.code == 0
    gs = GpuSchema(sd)
    grec, _, gst, gnd, gcons = S.deserialize_status(
        gs, torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).to(gpu), n)
    assert gst.code == 0 and gnd == n and gcons == len(wire)
    assert np.array_equal(grec.cpu().numpy()[:len(drec)], drec)
    stats = S.context().index_stats()
    assert stats["broken"] * 10 < stats["chunks"], stats
