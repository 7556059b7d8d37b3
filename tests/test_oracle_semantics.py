"""The oracle against semantic pins restated from the reference's C++ tests
(VarintUtilsTest, BinaryProtocolTest, ProtocolTruncatedDataTest,
ProtocolSkipTest, ProtocolTest skip-depth, CompactProtocolTest)."""
import numpy as np
import pytest

import corpus
import helpers
import wire
from fbthrift_amd.schema import Schema
from oracle import oracle


@pytest.mark.parametrize("case", corpus.cases(), ids=lambda c: c[0])
def test_corpus_codes(case):
    name, proto, table, stream, n, limits, expected = case
    st, *_ = oracle.decode(Schema.from_table(table), proto, stream, n, limits=limits)
    if expected is not None:
        assert st.code == expected, (name, st.as_tuple())


@pytest.mark.parametrize("proto", [0, 2])
@pytest.mark.parametrize("ttype", [12, 15, 14, 13])
def test_skip_check_depth(proto, ttype):
    """ProtocolTest.cpp:275-300 with kTestingProtocolMaxDepth = 4."""
    h = 4
    ok = wire.nested(proto, h, h - 1, ttype)
    assert oracle.skip_value(proto, ok, 12, height=h) == len(ok)
    deep = wire.nested(proto, h + 1, h + 1, ttype)
    assert oracle.skip_value(proto, deep, 12, height=h) == -8  # DEPTH_LIMIT


@pytest.mark.parametrize("proto", ["compact", "binary"])
def test_parses_updated_via_read(proto):
    """CompactProtocolTest.cpp:140-166: UpdatedStruct bytes read as
    OriginalStruct equal the original values (unknown fields skipped)."""
    upd = helpers.Case("updated_" + proto)
    orig = helpers.Case("original_" + proto)
    st, rec, arena, nd, cons = oracle.decode(orig.schema, upd.protocol, upd.wire, 1)
    assert st.code == 0 and cons == len(upd.wire)
    got = helpers.unpack(orig.schema, rec, 1, upd.wire, arena)
    helpers.assert_values_equal(got, orig.values)


def test_varint_medium_slow():
    """VarintUtilsTest.cpp:213-280 (u64, kMaxVarintSize = 10)."""
    for i in range(1, 10):
        buf = bytearray(b"\x80" * 10)
        buf[i] = 1
        assert oracle.read_varint(bytes(buf), 64) == (0, 1 << (7 * i), i + 1)
        buf[i] = 0
        assert oracle.read_varint(bytes(buf), 64) == (0, 0, i + 1)  # BigZeros
    assert oracle.read_varint(b"\x80" * 10, 64)[0] == 2  # Overflow -> out_of_range
    junk = b"\x80" * 9 + b"\x7f"
    assert oracle.read_varint(junk, 64) == (0, 1 << 63, 10)  # JunkHighBits
    # 32-bit reader: 5 bytes max, high bits dropped
    assert oracle.read_varint(b"\x80\x80\x80\x80\x7f", 32) == (0, 0xF0000000, 5)
    assert oracle.read_varint(b"\x80" * 5, 32)[0] == 2
    assert oracle.read_varint(b"\x80\x80", 64)[0] == 1  # underflow


def test_write_invalid_bool_and_huge_string():
    """BinaryProtocolTest.cpp:43-92: an invalid bool aborts (we report
    INVALID_BOOL_WRITE / exc_class ABORT); strings >= 2 GiB are rejected."""
    s = Schema.from_table(corpus.BOOL_SCHEMA)
    rec = np.zeros(s.record_size, np.uint8)
    rec[0] = 0x42
    for proto in (0, 2):
        st, wire_, _ = oracle.encode(s, proto, rec, 1)
        assert (st.code, st.exc_class) == (10, 3)
    s2 = Schema.from_table([[[1, 11, 0, 0, -1]]])
    rec2 = np.zeros(s2.record_size, np.uint8)
    rec2[8:12] = np.frombuffer(np.uint32(1 << 31).tobytes(), np.uint8)
    for proto in (0, 2):
        st, _, _ = oracle.encode(s2, proto, rec2, 1)
        assert (st.code, st.exc_class, st.tproto_type) == (11, 2, 3)
