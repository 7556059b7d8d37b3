"""Records carrying fields the schema does not know, appended before the
root STOP — what a writer with a newer schema produces. The reference's
generated reader leaves its fast path at the unexpected header and skips the
unknown field (deserialize_struct.whisker: unknown ids go to skip), so the
record is the canonical one and the stream position moves past the skipped
bytes. The tolerant compiled programs (tgpu_program.h skip_unknown_tail)
take plain appends of scalars and strings themselves; everything else (a schema id, a
container, over 8 fields, a bool byte above 1 — which Binary skip takes as one
byte, BinaryProtocol.cpp:140-225) goes to the general reader. Both must
give the oracle's records, status and consumption, through the indexed decode
(offsets given), the unindexed decode (stream index) and the index itself."""
import struct

import numpy as np
import pytest

import datagen
from oracle import oracle
from test_gpu_index import _gs, _ser, _stream, _t

T_BOOL, T_BYTE, T_DOUBLE, T_I16, T_I32, T_I64 = 2, 3, 4, 6, 8, 10
T_STRING, T_LIST, T_FLOAT = 11, 15, 19
CTYPE = {T_BOOL: 1, T_BYTE: 3, T_I16: 4, T_I32: 5, T_I64: 6, T_DOUBLE: 7, T_STRING: 8,
         T_LIST: 9, T_FLOAT: 13}


def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _zz(v, bits):
    return ((v << 1) ^ (v >> (bits - 1))) & ((1 << bits) - 1)


def encode_fields(proto, last_id, fields):
    """Field headers + values (Binary: BinaryProtocol-inl.h:31-140; Compact:
    CompactProtocol-inl.h:133-260, delta headers with the long form past 15)."""
    out = bytearray()
    prev = last_id
    for fid, t, v in fields:
        if proto == 0:
            out += struct.pack(">bh", t, fid)
            if t == T_BOOL or t == T_BYTE:
                out += struct.pack(">B", v & 0xFF)
            elif t == T_I16:
                out += struct.pack(">h", v)
            elif t == T_I32:
                out += struct.pack(">i", v)
            elif t == T_I64:
                out += struct.pack(">q", v)
            elif t == T_DOUBLE:
                out += struct.pack(">d", v)
            elif t == T_FLOAT:
                out += struct.pack(">f", v)
            elif t == T_STRING:
                out += struct.pack(">i", len(v)) + v
            elif t == T_LIST:  # list<i32>
                out += struct.pack(">bi", T_I32, len(v)) + b"".join(struct.pack(">i", x) for x in v)
        else:
            ct = CTYPE[t]
            if t == T_BOOL:
                ct = 1 if v else 2
            d = fid - prev
            if 0 < d <= 15:
                out.append((d << 4) | ct)
            else:
                out.append(ct)
                out += _varint(_zz(fid, 16))
            prev = fid
            if t == T_BYTE:
                out.append(v & 0xFF)
            elif t in (T_I16, T_I32):
                out += _varint(_zz(v, 32))
            elif t == T_I64:
                out += _varint(_zz(v, 64))
            elif t == T_DOUBLE:
                out += struct.pack("<d", v)
            elif t == T_FLOAT:
                out += struct.pack(">f", v)
            elif t == T_STRING:
                out += _varint(len(v)) + v
            elif t == T_LIST:
                out.append((len(v) << 4) | CTYPE[T_I32] if len(v) < 15 else 0xF0 | CTYPE[T_I32])
                if len(v) >= 15:
                    out += _varint(len(v))
                out += b"".join(_varint(_zz(x, 32)) for x in v)
    return bytes(out)


def with_tails(wire, offs, proto, last_id, tail_of):
    """Each record i gets tail_of(i) (a field list, or None) before its STOP."""
    out = bytearray()
    new_offs = [0]
    for i in range(len(offs) - 1):
        b, e = int(offs[i]), int(offs[i + 1])
        f = tail_of(i)
        if f:
            out += wire[b:e - 1] + encode_fields(proto, last_id, f) + b"\x00"
        else:
            out += wire[b:e]
        new_offs.append(len(out))
    return bytes(out), np.array(new_offs, np.uint64)


SCHEMA_IDS = {"mixed": (6, 6), "nested": (3, 3), "scalars": (15, 15)}
APPEND = [(20, T_I32, -7), (21, T_STRING, b"newer"), (60, T_I64, 1 << 40),
          (61, T_BOOL, 1), (62, T_DOUBLE, 2.5), (63, T_BYTE, 9), (64, T_I16, -300),
          (99, T_FLOAT, 1.5)]


def _tail_cases():
    return {
        # plain appends: the programs take them
        "every_record_i32": lambda i: [APPEND[0]],
        "every_record_all_types": lambda i: APPEND,
        "one_in_three_string": lambda i: [APPEND[1]] if i % 3 == 0 else None,
        # the general reader's cases
        "schema_id_again": lambda i: [(1, T_I32, 5)] if i % 5 == 0 else None,
        "container": lambda i: [(30, T_LIST, [1, 2, 3])] if i % 7 == 0 else None,
        "nine_fields": lambda i: [(40 + k, T_BYTE, k) for k in range(9)] if i % 11 == 0 else None,
        "bool_byte_2": lambda i: [(41, T_BOOL, 2)] if i == 77 else None,
    }


CASES = sorted(_tail_cases())


def _compare(sname, proto, wire, offs, n, gpu):
    schema = __import__("fbthrift_amd.schema", fromlist=["Schema"]).Schema.from_table(
        datagen.SCHEMAS[sname])
    gs = _gs(schema)
    w = _t(wire, gpu)
    S = _ser(proto)
    ost, orec, oarena, ond, ocons = oracle.decode(schema, proto, wire, n)
    # indexed: offsets given (program decode, general reader for the rest)
    import torch

    o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    rec, arena, st, nd, cons = S.deserialize_status(gs, w[: len(wire)], n, o)
    assert st.as_tuple() == ost.as_tuple()
    k = (ond + (1 if ost.code else 0)) * schema.size[0]
    assert np.array_equal(rec.cpu().numpy()[:k], orec[:k])
    # unindexed: the stream index finds the boundaries
    rec, arena, st, nd, cons = S.deserialize_status(gs, w[: len(wire)], n)
    assert st.as_tuple() == ost.as_tuple() and (nd, cons) == (ond, ocons)
    assert np.array_equal(rec.cpu().numpy()[:k], orec[:k])
    if ost.code == 0:
        offs_g, got, first, last, ist = S.index_stream(gs, w[: len(wire)])
        assert (ist.code, got, last) == (0, n, len(wire))
        assert np.array_equal(offs_g.cpu().numpy().astype(np.uint64), offs)
    return ost


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("sname,proto", [("mixed", 0), ("mixed", 2), ("nested", 0),
                                         ("nested", 2), ("scalars", 2)])
def test_oracle_reads_tails(sname, proto, case):
    """The oracle (the reference's reader restated) skips the appended fields:
    each record equals the record without them (records read one at a time,
    so string / list positions are relative to the record)."""
    n = 400
    schema, wire, offs = _stream(sname, proto, n)
    tail = _tail_cases()[case]
    w2, o2 = with_tails(wire, offs, proto, SCHEMA_IDS[sname][1], tail)
    st, rec, _, nd, cons = oracle.decode(schema, proto, w2, n)
    assert st.code == 0 and (nd, cons) == (n, len(w2))
    if case == "schema_id_again":
        return  # field 1 read twice: the second value wins (not the canonical record)
    for i in range(0, n, 37):
        a = oracle.decode(schema, proto, wire[int(offs[i]):int(offs[i + 1])], 1)
        b = oracle.decode(schema, proto, w2[int(o2[i]):int(o2[i + 1])], 1)
        assert a[0].code == b[0].code == 0
        assert np.array_equal(a[1], b[1])


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("sname,proto", [("mixed", 0), ("mixed", 2), ("nested", 0),
                                         ("nested", 2), ("scalars", 2)])
@pytest.mark.parametrize("tails", ["strict", "tolerant"])
def test_gpu_tails_match_oracle(gpu, codec, sname, proto, case, tails, monkeypatch):
    """strict: the default programs (the appended fields go to the general
    reader); tolerant: the programs that skip them (TGPU_PROGRAM_TAILS=1,
    what the fixed-layout path selects for a stream off its stride)."""
    if tails == "tolerant":
        monkeypatch.setenv("TGPU_PROGRAM_TAILS", "1")
    n = 20_000
    schema, wire, offs = _stream(sname, proto, n)
    w2, o2 = with_tails(wire, offs, proto, SCHEMA_IDS[sname][1], _tail_cases()[case])
    _compare(sname, proto, w2, o2, n, gpu)
