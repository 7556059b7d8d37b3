"""Terse fields (@thrift.TerseWrite, qualifier TGPU_TERSE): written only when
not empty — op::isEmpty, thrift/lib/cpp2/op/detail/Clear.h:98-127 (scalars
compared bitwise with the intrinsic default, so -0.0 is written; strings and
containers by length), the guard of module_types_custom_protocol.whisker:87-90
via fields.whisker:84; read like unqualified fields. The legacy Python
protocols have no terse fields, so the expected bytes are worked out by hand
from the wire rules (protocols.md:31-193) and pin the oracle; the GPU must
then equal the oracle on random terse batches."""
import struct

import numpy as np
import pytest

from fbthrift_amd.schema import Schema
from oracle import oracle

TABLE = [[[1, 8, 0, 2, -1], [2, 11, 0, 2, -1], [3, 4, 0, 2, -1], [4, 15, 8, 2, -1],
          [5, 10, 0, 0, -1]]]  # {1: terse i32, 2: terse string, 3: terse double,
                                #  4: terse list<i32>, 5: i64}


def _records(schema, rows):
    """rows: (i32, bytes, double_bits, [i32], i64) -> (records, string arena, list arena)."""
    r = np.zeros(len(rows), dtype=schema.dtype())
    sarena, larena = bytearray(), bytearray()
    for i, (a, s, dbits, lst, z) in enumerate(rows):
        r["f1"][i] = a
        r["f2"][i]["offset"], r["f2"][i]["length"] = len(sarena), len(s)
        sarena += s
        r["f3"][i] = struct.unpack("<d", struct.pack("<Q", dbits))[0]
        r["f4"][i]["offset"], r["f4"][i]["length"] = len(larena), len(lst)  # bytes, elements
        larena += b"".join(struct.pack("<i", x) for x in lst)
        r["f5"][i] = z
        r["__isset"][i] = 1
    return (r.view(np.uint8), np.frombuffer(bytes(sarena) or b"\0", np.uint8).copy(),
            np.frombuffer(bytes(larena) or b"\0\0\0\0", np.uint8).copy())


EMPTY = (0, b"", 0, [], 7)
FULL = (-1, b"ab", 0x8000000000000000, [3], 0)  # -0.0 is not empty


def test_oracle_terse_bytes():
    schema = Schema.from_table(TABLE)
    rec, sa, la = _records(schema, [EMPTY, FULL])
    st, wire, offs = oracle.encode(schema, 0, rec, 2, sa, la)
    assert st.code == 0
    want_b = (bytes.fromhex("0a0005 0000000000000007 00") +
              bytes.fromhex("080001 ffffffff 0b0002 00000002 6162 040003 8000000000000000"
                            " 0f0004 08 00000001 00000003 0a0005 0000000000000000 00"))
    assert wire == want_b
    st, wire, offs = oracle.encode(schema, 2, rec, 2, sa, la)
    # Compact: skipped fields do not move the delta base (writeFieldBegin is
    # never called for them, CompactProtocol-inl.h:133-172)
    want_c = (bytes.fromhex("56 0e 00") +
              bytes.fromhex("15 01 18 02 6162 17 8000000000000000 19 15 06 16 00 00"))
    assert wire == want_c
    # read back: the skipped fields keep their defaults and isset 0
    st, out, _, nd, _ = oracle.decode(schema, 2, wire, 2)
    r = out.view(schema.dtype())
    assert st.code == 0 and nd == 2
    assert r["f5"][0] == 7 and list(r["__isset"][0]) == [0, 0, 0, 0, 1]
    assert list(r["__isset"][1]) == [1, 1, 1, 1, 1] and r["f1"][1] == -1


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_gpu_terse_matches_oracle(gpu, protocol):
    import torch

    from fbthrift_amd.serializer import BinarySerializer, CompactSerializer, GpuSchema

    S = BinarySerializer if protocol == 0 else CompactSerializer
    schema = Schema.from_table(TABLE)
    rng = np.random.default_rng(7)
    rows = []
    for i in range(20_000):
        e = rng.integers(0, 2, 5)
        rows.append((0 if e[0] else int(rng.integers(-2**31, 2**31 - 1)),
                     b"" if e[1] else bytes(rng.integers(0, 256, int(rng.integers(1, 9)),
                                                         dtype=np.uint8)),
                     0 if e[2] else int(rng.choice([0x8000000000000000, 1, 0x3ff0000000000000])),
                     [] if e[3] else [int(x) for x in rng.integers(-9, 9, int(rng.integers(1, 5)))],
                     int(rng.integers(-2**40, 2**40))))
    rec, sa, la = _records(schema, rows)
    n = len(rows)
    ost, owire, ooffs = oracle.encode(schema, protocol, rec, n, sa, la)
    assert ost.code == 0
    gs = GpuSchema(schema)
    dev = gpu
    wire, offs = S.serialize(gs, torch.from_numpy(rec).to(dev), n, torch.from_numpy(sa).to(dev),
                             torch.from_numpy(la).to(dev))
    assert bytes(wire.cpu().numpy()) == owire
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), ooffs)
    w = torch.from_numpy(np.frombuffer(owire, np.uint8).copy()).to(dev)
    grec, garena, gst, gnd, gcons = S.deserialize_status(gs, w, n)
    dst, drec, darena, dnd, dcons = oracle.decode(schema, protocol, owire, n)
    assert gst.as_tuple() == dst.as_tuple() and (gnd, gcons) == (dnd, dcons)
    assert np.array_equal(grec.cpu().numpy(), drec)
