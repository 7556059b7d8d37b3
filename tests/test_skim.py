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
