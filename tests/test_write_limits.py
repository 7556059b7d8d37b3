"""Writer-side size limits on the device: a string, list, set or map whose
length does not fit the wire's i32 size is rejected before a byte of it is
read (BinaryProtocol-inl.h:201-208 checkBinarySize, protocol_methods.h
checked_container_size -> TProtocolException SIZE_LIMIT), and an invalid
bool aborts (validate_bool, Protocol.h:126-163). The batch fails at the
first such record with the oracle's exact status; the records before it are
written byte-identically."""
import ctypes

import numpy as np
import pytest

from fbthrift_amd import _lib
from fbthrift_amd.schema import Schema
from oracle import oracle

I32, I64, STR, LIST, SET, MAP, BOOL = 8, 10, 11, 15, 14, 13, 2
SCHEMAS = {
    "string": [[[1, I64, 0, 0, -1], [2, STR, 0, 0, -1]]],
    "list_i32": [[[1, I64, 0, 0, -1], [2, LIST, I32, 0, -1]]],
    "set_i64": [[[1, I64, 0, 0, -1], [2, SET, I64, 0, -1]]],
    "list_str": [[[1, I64, 0, 0, -1], [2, LIST, STR, 0, -1]]],
    "map_i32_str": [[[1, I64, 0, 0, -1], [2, MAP, I32, 0, -1, STR]]],
    "bool": [[[1, I64, 0, 0, -1], [2, BOOL, 0, 0, -1]]],
}
ELEM = {"list_i32": 4, "set_i64": 8, "list_str": 16, "map_i32_str": 20}


def batch(name, n, bad, huge):
    """n records {1: i, 2: small value}; record `bad` carries length `huge`
    (or bool byte `huge`). Returns (schema, records, string base, list base)."""
    schema = Schema.from_table(SCHEMAS[name])
    structs, _, fields, _ = schema.descriptors()
    S = schema.record_size
    m1, m2, i2 = fields[0].member_offset, fields[1].member_offset, fields[1].isset_offset
    rec = np.zeros((n, S), np.uint8)
    rec[:, m1:m1 + 8] = np.arange(n, dtype=np.int64).view(np.uint8).reshape(n, 8)
    rec[:, fields[0].isset_offset] = 1
    rec[:, i2] = 1
    strings = np.frombuffer(b"abcdefgh" * 8, np.uint8).copy()
    es = ELEM.get(name, 0)
    lists = np.zeros(max(es * 2, 16), np.uint8)
    if name in ("list_str", "map_i32_str"):
        # element 0: a span of 3 string bytes (+ the key for the map)
        span = np.array([(0, 3, 0)], dtype=[("o", "<u8"), ("l", "<u4"), ("r", "<u4")])
        k = 4 if name == "map_i32_str" else 0
        lists[k:k + 16] = span.view(np.uint8)
    if name == "bool":
        rec[:, m2] = 1
        rec[bad, m2] = huge
    else:
        length = np.full(n, 3 if name == "string" else 1, np.uint32)
        length[bad] = huge
        span = np.zeros(n, dtype=[("o", "<u8"), ("l", "<u4"), ("r", "<u4")])
        span["l"] = length
        rec[:, m2:m2 + 16] = span.view(np.uint8).reshape(n, 16)
    return schema, rec.reshape(-1), strings, lists


def gpu_encode(schema, protocol, rec, n, strings, lists, dev, cap=1 << 20):
    import torch

    from fbthrift_amd.serializer import BinarySerializer, GpuSchema

    gs = GpuSchema(schema)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    r, sb, lb = t(rec), t(strings), t(lists)
    out = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    st, size = _lib.Status(), ctypes.c_uint64()
    _lib.lib().tgpu_encode_batch(BinarySerializer.context().handle, gs.handle, protocol,
                                 ctypes.c_void_p(r.data_ptr()), n, ctypes.c_void_p(sb.data_ptr()),
                                 ctypes.c_void_p(lb.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                 cap, ctypes.c_void_p(offs.data_ptr()), None, ctypes.byref(st),
                                 ctypes.byref(size))
    return st, out.cpu().numpy()[: size.value].tobytes()


def test_oracle_limits():
    for name in SCHEMAS:
        huge = 2 if name == "bool" else 1 << 31
        schema, rec, sb, lb = batch(name, 8, 5, huge)
        for proto in (0, 2):
            st, wire, _ = oracle.encode(schema, proto, rec, 8, sb, lb)
            want = (10, 3) if name == "bool" else (11, 2)
            assert (st.code, st.exc_class, st.record) == want + (5,), (name, st.as_tuple())


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCHEMAS))
@pytest.mark.parametrize("protocol", [0, 2])
@pytest.mark.parametrize("huge", [1 << 31, 0xFFFFFFFF])
def test_gpu_write_size_limit(gpu, codec, name, protocol, huge):
    n, bad = 1000, 613
    if name == "bool":
        huge = 2 if huge == 1 << 31 else 0xFF
    schema, rec, sb, lb = batch(name, n, bad, huge)
    ost, owire, _ = oracle.encode(schema, protocol, rec, n, sb, lb, cap=1 << 20)
    st, wire = gpu_encode(schema, protocol, rec, n, sb, lb, gpu)
    assert st.as_tuple() == ost.as_tuple()
    assert st.record == bad and st.code == (10 if name == "bool" else 11)
    assert wire == owire  # the records before the failing one
