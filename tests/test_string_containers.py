"""Strings inside lists, sets and maps: each element is a tgpu_span, read
and written like a string field (readString / writeBinary, Protocol.h:
406-449, BinaryProtocol-inl.h:195-222, CompactProtocol-inl.h:742-781), in
the list arena at 4 (Binary) / 16 (Compact) arena bytes per wire byte
(tgpu_schema_arena_scale). Oracle pinned by the strcont_* golden cases from
the reference's Python protocols; the GPU must equal the oracle.
"""
import numpy as np
import pytest

import datagen
import helpers
from fbthrift_amd.schema import Schema
from oracle import oracle


@pytest.mark.gpu
def test_arena_scale(gpu):
    from fbthrift_amd import _lib
    from fbthrift_amd.serializer import GpuSchema

    L = _lib.lib()
    for name, want in (("flat8", (0, 0)), ("nested", (1, 8)), ("maps", (1, 8)),
                       ("strcont", (4, 16))):
        gs = GpuSchema(Schema.from_table(datagen.SCHEMAS[name]))
        assert (L.tgpu_schema_arena_scale(gs.handle, 0),
                L.tgpu_schema_arena_scale(gs.handle, 2)) == want, name


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [0, 2])
def test_gpu_string_containers_match_oracle(gpu, proto):
    import torch

    from fbthrift_amd.serializer import BinarySerializer, CompactSerializer, GpuSchema

    S = BinarySerializer if proto == 0 else CompactSerializer
    table = datagen.SCHEMAS["strcont"]
    schema = Schema.from_table(table)
    n = 8000
    vals = datagen.flatten_values(table, [datagen.gen_strcont(i + 500) for i in range(n)])
    rec, sa, la = helpers.pack(schema, vals, n)
    ost, owire, ooffs = oracle.encode(schema, proto, rec, n, sa, la)
    assert ost.code == 0
    gs = GpuSchema(schema)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy() if a.size
                                   else np.zeros(1, np.uint8)).to(gpu)
    wire, offs = S.serialize(gs, t(rec), n, t(sa), t(la))
    assert bytes(wire.cpu().numpy()) == owire
    sz, total = S.encoded_size(gs, t(rec), n, list_base=t(la))
    assert total == len(owire)
    base = np.frombuffer(owire, np.uint8)
    rng = np.random.default_rng(17 + proto)
    for trial in range(10):
        m = base.copy()
        if trial:
            pos = rng.integers(0, m.size, 2)
            m[pos] = rng.integers(0, 256, 2)
        grec, garena, gst, gnd, gcons = S.deserialize_status(gs, t(m), n)
        dst, drec, darena, dnd, dcons = oracle.decode(schema, proto, m, n)
        assert gst.as_tuple() == dst.as_tuple(), trial
        assert (gnd, gcons) == (dnd, dcons)
        k = dnd + (1 if dst.code else 0)
        gr = grec.cpu().numpy()
        assert np.array_equal(gr[:k * schema.record_size], drec[:k * schema.record_size])
        if dst.code == 0:
            helpers.assert_values_equal(helpers.unpack(schema, gr, n, m, garena.cpu().numpy()),
                                        vals if trial == 0 else
                                        helpers.unpack(schema, drec, n, m, darena))
