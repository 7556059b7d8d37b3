"""Maps of scalars (T_MAP, key type in elem_ttype, value type in val_ttype).

Read: protocol_methods<map>::read (thrift/lib/cpp2/protocol/detail/
protocol_methods.h:640-677) — readMapBegin, skip_n on a key/value type
mismatch of a non-empty map, canReadNElements(n, {k, v}), the pairs in wire
order (packed {key, value} in the list arena), a failing pair not inserted
(op/detail/EncodeHelpers.h:188-205). Write: writeMapBegin (BinaryProtocol-
inl.h:69-80, CompactProtocol-inl.h:182-201) then key, value per pair.

The oracle is pinned by the maps_binary / maps_compact golden cases written
by the reference's Python protocols (tests/golden/make_golden.py) and by the
hand-built cases in tests/corpus.py; the GPU must equal the oracle on random
batches, on every prefix of a batch, and on byte-flipped streams.
"""
import ctypes

import numpy as np
import pytest

import datagen
import helpers
from fbthrift_amd import _lib
from fbthrift_amd.schema import Field, Schema, Struct
from oracle import oracle

T_MAP, T_I32, T_STRING, T_LIST = 13, 8, 11, 15


@pytest.mark.gpu
def test_map_schema_validation(gpu):
    """Maps of scalar or string keys and values; anything else is UNSUPPORTED."""
    for kt, vt, ok in ((8, 10, True), (2, 3, True), (11, 8, True), (12, 8, False), (8, 15, False),
                       (8, 0, False)):
        s = Schema(Struct("S", [Field(1, T_MAP, kt, val_ttype=vt)]))
        structs, ns, fields, nf = s.descriptors()
        h = ctypes.c_void_p()
        rc = _lib.lib().tgpu_schema_create(ctypes.addressof(structs), ns,
                                          ctypes.addressof(fields), nf, ctypes.byref(h))
        if h.value:
            _lib.lib().tgpu_schema_destroy(h)
        assert (rc == 0) == ok, (kt, vt, rc)


def test_map_layout_is_a_span():
    """A map member is a 16-byte tgpu_span; tgpu_layout_compute agrees."""
    from fbthrift_amd.schema import layout_compute_c

    s = Schema.from_table(datagen.SCHEMAS["maps"])
    assert s.dtype()["f1"].itemsize == 16
    structs, fields = layout_compute_c(s)
    assert structs[0][2] == s.record_size
    assert [f[0] for f in fields[:7]] == [s.member[(0, k)] for k in range(7)]


def _golden(proto):
    return helpers.Case("maps_" + proto)


@pytest.mark.parametrize("proto", ["binary", "compact"])
def test_oracle_map_prefixes_keep_complete_pairs(proto):
    """Every prefix of a record: the decoded map holds exactly the complete
    pairs read before the failure (and the status is the reader's)."""
    c = _golden(proto)
    # a record with a big first map
    i = next(j for j in range(c.n) if len(datagen.gen_maps(j)[0]) == 130)
    rec_bytes = c.wire[int(c.offsets[i]):int(c.offsets[i + 1])]
    want = datagen.gen_maps(i)[0]
    for cut in range(4, 60):
        st, rec, arena, nd, _ = oracle.decode(c.schema, c.protocol, rec_bytes[:cut], 1)
        assert st.code != 0
        got = helpers.unpack(c.schema, rec, 1, rec_bytes[:cut], arena)
        k = int(got["0.count"][0])
        assert list(got["0.keys"]) == [a for a, _ in want[:k]]
        assert list(got["0.vals"]) == [b for _, b in want[:k]]


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [0, 2])
def test_gpu_maps_match_oracle_random(gpu, proto):
    import torch

    from fbthrift_amd.serializer import BinarySerializer, CompactSerializer, GpuSchema

    S = BinarySerializer if proto == 0 else CompactSerializer
    table = datagen.SCHEMAS["maps"]
    schema = Schema.from_table(table)
    n = 6000
    recs = [datagen.gen_maps(i + 1000) for i in range(n)]
    vals = datagen.flatten_values(table, recs)
    rec, sa, la = helpers.pack(schema, vals, n)
    ost, owire, ooffs = oracle.encode(schema, proto, rec, n, sa, la)
    assert ost.code == 0
    gs = GpuSchema(schema)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a) if a.size else np.zeros(1, np.uint8)).to(gpu)
    wire, offs = S.serialize(gs, t(rec), n, t(sa), t(la))
    assert bytes(wire.cpu().numpy()) == owire
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), ooffs)
    w = t(np.frombuffer(owire, np.uint8).copy())
    grec, garena, gst, gnd, gcons = S.deserialize_status(gs, w, n)
    assert gst.code == 0 and gnd == n
    helpers.assert_values_equal(
        helpers.unpack(schema, grec.cpu().numpy(), n, owire, garena.cpu().numpy()), vals)
    # byte flips: statuses, records and the maps read so far equal the oracle's
    rng = np.random.default_rng(11 + proto)
    base = np.frombuffer(owire, np.uint8)
    for trial in range(12):
        m = base.copy()
        pos = rng.integers(0, m.size, 3)
        m[pos] = rng.integers(0, 256, 3)
        gm = t(m)
        grec, garena, gst, gnd, gcons = S.deserialize_status(gs, gm, n)
        dst, drec, darena, dnd, dcons = oracle.decode(schema, proto, m, n)
        assert gst.as_tuple() == dst.as_tuple(), trial
        assert (gnd, gcons) == (dnd, dcons)
        k = dnd + (1 if dst.code else 0)
        gr, dr = grec.cpu().numpy(), drec
        assert np.array_equal(gr[:k * schema.record_size], dr[:k * schema.record_size])
        helpers.assert_values_equal(helpers.unpack(schema, gr, k, m, garena.cpu().numpy()),
                                    helpers.unpack(schema, dr, k, m, darena))
