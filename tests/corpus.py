"""Semantic pins restated from the reference's C++ tests, as decode cases.

Each entry: (name, protocol, schema table, stream bytes, n_records, limits,
expected code or None). `expected` comes from the cited reference test; the
oracle must produce it, and the GPU must produce the oracle's full status.
"""
import struct

from wire import B, C, W, varint, zz32, zz64

I64, I32, I16, BOOL, BYTE, STR, LIST, SET, STRUCT, MAP, DBL = 10, 8, 6, 2, 3, 11, 15, 14, 12, 13, 4

# codes (include/thrift_gpu.h)
OK, UNDERFLOW, VARINT, BOOLV, SKIPT, TRUNC, NEG, LIMIT, DEPTH, BADT = 0, 1, 2, 3, 4, 5, 6, 7, 8, 9

TRUNC_SCHEMA = [[[1, LIST, I64, 1, -1], [2, SET, I32, 1, -1], [4, STR, 0, 1, -1]]]
BOOL_SCHEMA = [[[1, BOOL, 0, 0, -1], [2, I32, 0, 0, -1]]]
FLAT = [[[k, I64, 0, 0, -1] for k in range(1, 9)]]
EMPTY = [[]]


def truncated_list(proto):
    # ProtocolTruncatedDataTest.cpp:98-108: 30 x (1 << i) as list<i64>
    w = W(proto).field(LIST, 1).list_begin(I64, 30)
    for i in range(30):
        w.i64(1 << i)
    return w.stop().bytes()


def truncated_set(proto):
    w = W(proto).field(SET, 2).list_begin(I32, 30)
    for i in range(30):
        w.i32((1 << i) - (1 << 32 if (1 << i) >= (1 << 31) else 0))
    return w.stop().bytes()


def truncated_string(proto):
    return W(proto).field(STR, 4).string(b"foobarbazstring").stop().bytes()


def cases():
    out = []
    # --- ProtocolTruncatedDataTest.cpp:28-120 (Compact list/set, both strings)
    for p, name, full, keep in [
        (C, "trunc_list", truncated_list(C), 3 + 30),
        (C, "trunc_set", truncated_set(C), 3 + 30),
        (C, "trunc_str_compact", truncated_string(C), 2 + 15),
        (B, "trunc_str_binary", truncated_string(B), 7 + 15),
    ]:
        out.append((name + "_full", p, TRUNC_SCHEMA, full, 1, None, OK))
        # trimmed to just pass the size check: std::out_of_range
        out.append((name + "_pass_check", p, TRUNC_SCHEMA, full[:keep], 1, None, UNDERFLOW))
        # one byte less: TProtocolException (throwTruncatedData)
        out.append((name + "_fail_check", p, TRUNC_SCHEMA, full[:keep - 1], 1, None, TRUNC))
    # --- BinaryProtocolTest.cpp:30-41 readBool: byte >= 2 throws INVALID_DATA
    for v, code in ((0, OK), (1, OK), (2, BOOLV), (0x42, BOOLV)):
        wb = W(B).field(BOOL, 1).byte(v).field(I32, 2).i32(5).stop().bytes()
        out.append(("binary_bool_%d" % v, B, BOOL_SCHEMA, wb, 1, None, code))
    # Compact container bools accept any byte (== 1 -> true), field bools ride
    # in the header (CompactProtocol-inl.h:692-701)
    for v in (0, 1, 2, 0x42):
        wc = W(C).field(LIST, 1).list_begin(BOOL, 2).byte(v).byte(1).stop().bytes()
        out.append(("compact_bool_list_%d" % v, C, [[[1, LIST, BOOL, 0, -1]]], wc, 1, None, OK))
    # --- VarintUtilsTest.cpp:238-280: overflow, junk high bits, big zeros
    for p_name, bits, ttype, kmax in (("i32", 32, I32, 5), ("i64", 64, I64, 10)):
        sch = [[[1, ttype, 0, 0, -1]]]
        hdr = bytes([0x10 | (5 if bits == 32 else 6)])
        out.append(("varint_overflow_" + p_name, C, sch, hdr + b"\x80" * kmax + b"\x00", 1, None,
                    VARINT))
        out.append(("varint_junk_" + p_name, C, sch, hdr + b"\x80" * (kmax - 1) + b"\x7f\x00", 1,
                    None, OK))
        for i in range(1, kmax):
            z = b"\x80" * i + b"\x00"
            out.append(("varint_bigzero_%s_%d" % (p_name, i), C, sch, hdr + z + b"\x00", 1, None,
                        OK))
        out.append(("varint_cut_" + p_name, C, sch, hdr + b"\x80\x80", 1, None, UNDERFLOW))
    # --- sizes: negative / limits (BinaryProtocol-inl.h:535-551,
    # CompactProtocol-inl.h:615-640,742-749)
    sstr = [[[1, STR, 0, 0, -1]]]
    out.append(("binary_neg_string", B, sstr, b"\x0b\x00\x01\xff\xff\xff\xff\x00", 1, None, NEG))
    out.append(("compact_neg_string", C, sstr, b"\x18" + varint(0x80000000) + b"\x00", 1, None, NEG))
    out.append(("binary_string_limit", B, sstr, W(B).field(STR, 1).string(b"abcdef").stop().bytes(),
                1, (4, 0, 12000, 0), LIMIT))
    out.append(("compact_string_limit", C, sstr,
                W(C).field(STR, 1).string(b"abcdef").stop().bytes(), 1, (4, 0, 12000, 0), LIMIT))
    slist = [[[1, LIST, I32, 0, -1]]]
    out.append(("binary_neg_list", B, slist, b"\x0f\x00\x01\x08\xff\xff\xff\xfe\x00", 1, None, NEG))
    out.append(("compact_neg_list", C, slist, b"\x19\xf5" + varint(0xFFFFFFFF) + b"\x00", 1, None,
                NEG))
    lst = W(C).field(LIST, 1).list_begin(I32, 5)
    for i in range(5):
        lst.i32(i)
    out.append(("compact_container_limit", C, slist, lst.stop().bytes(), 1, (0, 3, 12000, 0),
                LIMIT))
    # element-type mismatch: list skipped, left empty, no error
    # (protocol_methods.h:405-406)
    mm = W(B).field(LIST, 1).list_begin(I64, 2).i64(1).i64(2).stop().bytes()
    out.append(("binary_list_type_mismatch", B, slist, mm, 1, None, OK))
    mmc = W(C).field(LIST, 1).list_begin(STR, 2).string(b"x").string(b"yz").stop().bytes()
    out.append(("compact_list_type_mismatch", C, slist, mmc, 1, None, OK))
    # --- Compact "don't know what type" (CompactProtocol-inl.h:783-791)
    out.append(("compact_bad_type_field", C, EMPTY, b"\x1e\x00", 1, None, BADT))
    out.append(("compact_bad_list_elem", C, EMPTY, b"\x19\x1e\x00", 1, None, BADT))
    # --- ProtocolSkipTest.cpp: invalid skip types (VOID/STREAM/unknown) in
    # Binary unknown fields, valid ones skipped
    for t, code in ((1, SKIPT), (18, SKIPT), (0x55, SKIPT), (16, OK), (17, OK), (9, OK)):
        body = b"\x00\x00\x00\x02ab" if t in (16, 17) else (b"\x00" * 8 if t == 9 else b"")
        out.append(("binary_skip_type_%d" % t, B, EMPTY, bytes([t, 0, 7]) + body + b"\x00", 1,
                    None, code))
    # Binary skip of a string whose length passes the pre-length canAdvance
    # check but not the real one: out_of_range (BinaryProtocol.cpp:163-172)
    out.append(("binary_skip_string_edge", B, EMPTY, b"\x0b\x00\x07\x00\x00\x00\x05abcd", 1, None,
                UNDERFLOW))
    out.append(("binary_skip_string_neg", B, EMPTY, b"\x0b\x00\x07\xff\xff\xff\xff\x00", 1, None,
                TRUNC))
    # --- field ids: long form, negative, out of order, duplicates
    w = W(C)
    w.field(I64, 8).i64(-8).field(I64, 1).i64(1).field(I64, 100).i64(9)  # unknown 100
    w.field(I64, 1).i64(11)  # duplicate: later wins
    out.append(("compact_reorder_dup", C, FLAT, w.stop().bytes(), 1, None, OK))
    w = W(B)
    for k in (3, 1, 2):
        w.field(I64, k).i64(k * 1000)
    w.field(I32, 4).i32(7)  # type mismatch with schema (i64): skipped
    out.append(("binary_reorder_mismatch", B, FLAT, w.stop().bytes(), 1, None, OK))
    # --- truncation inside headers / values
    full = W(B).field(I64, 1).i64(5).stop().bytes()
    for cut in range(len(full)):
        out.append(("binary_cut_%d" % cut, B, FLAT, full[:cut], 1, None, UNDERFLOW))
    fullc = W(C).field(I64, 1).i64(-300).stop().bytes()
    for cut in range(len(fullc)):
        out.append(("compact_cut_%d" % cut, C, FLAT, fullc[:cut], 1, None, UNDERFLOW))
    # --- Compact STOP forms: any byte with zero low nibble ends the struct
    for b0 in (0x00, 0x10, 0xF0):
        out.append(("compact_stop_%02x" % b0, C, FLAT, bytes([b0]), 1, None, OK))
    # --- skip depth (ProtocolTest.cpp:275-300, kTestingProtocolMaxDepth = 4)
    for p in (B, C):
        for t in (STRUCT, LIST, SET, MAP):
            ok_stream = nested_record(p, 4, 3, t)
            out.append(("depth_ok_%d_%d" % (p, t), p, EMPTY, ok_stream, 1, (0, 0, 12000, 4), None))
            deep = nested_record(p, 5, 5, t)
            out.append(("depth_deep_%d_%d" % (p, t), p, EMPTY, deep, 1, (0, 0, 12000, 4), None))
    # --- multi-record streams with a failure in the middle: first failing
    # record index and consumed bytes
    good = W(B).field(I64, 1).i64(1).stop().bytes()
    bad = W(B).field(BOOL, 2).byte(9).stop().bytes()
    two = [[[1, I64, 0, 0, -1], [2, BOOL, 0, 0, -1]]]
    out.append(("binary_mid_failure", B, two, good * 5 + bad + good * 3, 9, None, BOOLV))
    goodc = W(C).field(I64, 1).i64(1).stop().bytes()
    badc = W(C).field(I64, 1).raw(b"\xff" * 10).stop().bytes()
    out.append(("compact_mid_failure", C, two, goodc * 7 + badc + goodc, 9, None, VARINT))
    out += map_cases()
    out += union_cases()
    out += string_elem_cases()
    out += required_cases()
    return out


MISSING_REQ = 13
REQ = 3


def _req_schema(enforce):
    # {1: required i64, 2: i32, 3: Inner{1: required i32, 2: i32}}
    return [{"fields": [[1, I64, 0, REQ, -1], [2, I32, 0, 0, -1], [3, STRUCT, 0, 0, 1]],
             "enforce_required": enforce},
            {"fields": [[1, I32, 0, REQ, -1], [2, I32, 0, 0, -1]], "enforce_required": enforce}]


def required_cases():
    """deserialize_struct.whisker:116-124 (deprecated_enforce_required): after
    readStructEnd, a required field this read of the struct did not see
    throws TProtocolException MISSING_REQUIRED_FIELD; without the option the
    record reads normally. A field of the wrong type is skipped, so it is not
    seen; a nested struct read twice is checked per read."""
    out = []
    for p, pn in ((B, "binary"), (C, "compact")):
        def rec(f1=True, f1_type=I64, inner=((1, 5), (2, 6)), inner2=None):
            w = W(p)
            if f1:
                w.field(f1_type, 1)
                w.i64(9) if f1_type == I64 else w.i32(9)
            w.field(I32, 2).i32(3)
            for ins in (inner, inner2):
                if ins is None:
                    continue
                w.field(STRUCT, 3).struct_begin()
                for fid, v in ins:
                    w.field(I32, fid).i32(v)
                w.struct_end()
            return w.stop().bytes()

        good = rec()
        for enforce in (True, False):
            tag = "%s_req_%s" % (pn, "enforced" if enforce else "off")
            sch = _req_schema(enforce)
            for name, stream, code in (
                    ("ok", good, OK),
                    ("missing_root", rec(f1=False), MISSING_REQ),
                    ("wrong_type", rec(f1_type=I32), MISSING_REQ),
                    ("missing_inner", rec(inner=((2, 6),)), MISSING_REQ),
                    ("inner_absent", rec(inner=None), OK),
                    ("inner_twice_second_missing", rec(inner2=((2, 7),)), MISSING_REQ),
                    ("third_record", good + good + rec(f1=False) + good, MISSING_REQ)):
                n = 4 if name == "third_record" else 1
                out.append(("%s_%s" % (tag, name), p, sch, stream, n, None,
                            code if enforce else OK))
    return out


def nested_record(proto, height, levels, ttype):
    import wire
    return wire.nested(proto, height, levels, ttype)


MAP_SCHEMA = [[[1, MAP, I32, 0, -1, I64], [2, I32, 0, 0, -1]]]
BMAP_SCHEMA = [[[1, MAP, BOOL, 0, -1, BYTE]]]


def map_cases():
    """protocol_methods<map>::read (protocol_methods.h:640-677) and
    readMapBegin (BinaryProtocol-inl.h:439-451, CompactProtocol-inl.h:615-650)."""
    out = []
    for p, pn in ((B, "binary"), (C, "compact")):
        def m(n, kt=I32, vt=I64, pairs=None):
            w = W(p).field(MAP, 1).map_begin(kt, vt, n)
            for k, v in (pairs if pairs is not None else [(j, -j) for j in range(n)]):
                (w.i32 if kt == I32 else w.i64)(k)
                (w.i64 if vt == I64 else w.i32)(v)
            return w

        full = m(5).field(I32, 2).i32(9).stop().bytes()
        out.append(("%s_map_ok" % pn, p, MAP_SCHEMA, full, 1, None, OK))
        out.append(("%s_map_empty" % pn, p, MAP_SCHEMA, m(0).field(I32, 2).i32(1).stop().bytes(),
                    1, None, OK))
        # key/value type mismatch of a non-empty map: skip_n, member left empty
        mm = m(3, I64, I32).field(I32, 2).i32(4).stop().bytes()
        out.append(("%s_map_type_mismatch" % pn, p, MAP_SCHEMA, mm, 1, None, OK))
        # cut inside a pair: the map keeps the complete pairs (EncodeHelpers.h:188-205)
        hdr = len(W(p).field(MAP, 1).map_begin(I32, I64, 5).bytes())
        for cut in range(hdr, len(full) - 4):
            code = TRUNC if cut - hdr < 10 else UNDERFLOW
            out.append(("%s_map_cut_%d" % (pn, cut), p, MAP_SCHEMA, full[:cut], 1, None, code))
        out.append(("%s_map_limit" % pn, p, MAP_SCHEMA, full, 1, (0, 4, 12000, 0), LIMIT))
        out.append(("%s_map_limit_ok" % pn, p, MAP_SCHEMA, full, 1, (0, 5, 12000, 0), OK))
        # each map counts as one level of nesting (descend in readMapBegin;
        # generated struct reads do not descend): a map of maps under an
        # unknown id, skipped with height 1
        mm2 = W(p).field(MAP, 9).map_begin(I32, MAP, 1).i32(1).map_begin(I32, I32, 1) \
            .i32(2).i32(3).field(I32, 2).i32(1).stop().bytes()
        out.append(("%s_map_height" % pn, p, MAP_SCHEMA, mm2, 1, (0, 0, 12000, 1), DEPTH))
        out.append(("%s_map_height_ok" % pn, p, MAP_SCHEMA, mm2, 1, (0, 0, 12000, 2), OK))
        # skipped (unknown id) map
        sk = W(p).field(MAP, 9).map_begin(I32, STR, 2).i32(1).string(b"ab").i32(2) \
            .string(b"").field(I32, 2).i32(3).stop().bytes()
        out.append(("%s_map_skipped" % pn, p, MAP_SCHEMA, sk, 1, None, OK))
    # negative sizes
    out.append(("binary_map_negative", B, MAP_SCHEMA,
                b"\x0d\x00\x01\x08\x0a\xff\xff\xff\xff\x00", 1, None, NEG))
    out.append(("compact_map_negative", C, MAP_SCHEMA,
                b"\x1b" + varint(0x80000000) + b"\x56\x00", 1, None, NEG))
    # canReadNElements(n, {k, v}): 2 bytes per pair must remain
    out.append(("compact_map_cant_read", C, MAP_SCHEMA, b"\x1b\x05\x56" + b"\x00" * 9, 1, None,
                TRUNC))
    out.append(("compact_map_can_read", C, MAP_SCHEMA,
                b"\x1b\x05\x56" + b"\x02\x01" * 5 + b"\x00", 1, None, OK))
    # a key/value nibble >= 14 is a bad type (getType, CompactProtocol-inl.h:783-791)
    out.append(("compact_map_bad_type", C, MAP_SCHEMA, b"\x1b\x01\x5e\x00\x00\x00", 1, None,
                BADT))
    # Compact empty map: no kv byte, whatever follows is the next field
    out.append(("compact_map_empty_no_kv", C, MAP_SCHEMA, b"\x1b\x00\x15\x04\x00", 1, None,
                OK))
    # bools in maps: Binary rejects bytes >= 2, Compact takes == 1 as true
    for v, code in ((1, OK), (2, BOOLV)):
        wb = W(B).field(MAP, 1).map_begin(BOOL, BYTE, 1).byte(v).byte(7).stop().bytes()
        out.append(("binary_map_bool_%d" % v, B, BMAP_SCHEMA, wb, 1, None, code))
    for v in (1, 2, 0x42):
        wc = W(C).field(MAP, 1).map_begin(BOOL, BYTE, 1).byte(v).byte(7).stop().bytes()
        out.append(("compact_map_bool_%d" % v, C, BMAP_SCHEMA, wc, 1, None, OK))
    return out


# {1: i32, 2: U} with union U {1: i64, 2: string, 3: Inner{1: i32}}
UNION_SCHEMA = [[[1, I32, 0, 0, -1], [2, STRUCT, 0, 0, 1]],
                {"union": True, "fields": [[1, I64, 0, 0, -1], [2, STR, 0, 0, -1],
                                           [3, STRUCT, 0, 0, 2]]},
                [[1, I32, 0, 0, -1]]]
ROOT_UNION = [{"union": True, "fields": [[1, I64, 0, 0, -1], [2, I32, 0, 0, -1]]}]
UNION_MISSING_STOP = 12


def union_cases():
    """deserialize_union.whisker:19-60: STOP first clears the union, one field
    (read, or skipped when unknown / of another type) then STOP, else
    throwUnionMissingStop (TProtocolException.cpp:23-27, INVALID_DATA)."""
    out = []
    for p, pn in ((B, "binary"), (C, "compact")):
        def rec(*union_fields, tail=True):
            w = W(p).field(I32, 1).i32(7).field(STRUCT, 2).struct_begin()
            for f in union_fields:
                f(w)
            w.struct_end()
            if tail:
                w.field(I32, 1).i32(8)
            return w.stop().bytes()

        i64 = lambda w: w.field(I64, 1).i64(-5)
        s = lambda w: w.field(STR, 2).string(b"abc")
        inner = lambda w: w.field(STRUCT, 3).struct_begin().field(I32, 1).i32(4).struct_end()
        unk = lambda w: w.field(I32, 9).i32(1)
        wrong = lambda w: w.field(I32, 2).i32(3)  # member 2 is a string
        for name, fields, code in (("one", (i64,), OK), ("string", (s,), OK),
                                   ("struct", (inner,), OK), ("empty", (), OK),
                                   ("two", (i64, s), UNION_MISSING_STOP),
                                   ("unknown", (unk,), OK),
                                   ("unknown_then_field", (unk, i64), UNION_MISSING_STOP),
                                   ("type_mismatch", (wrong,), OK),
                                   ("mismatch_then_field", (wrong, s), UNION_MISSING_STOP)):
            out.append(("%s_union_%s" % (pn, name), p, UNION_SCHEMA, rec(*fields), 1, None, code))
        # the union field twice: the second read replaces (emplace) or clears (STOP)
        twice = W(p).field(STRUCT, 2).struct_begin()
        i64(twice)
        twice.struct_end().field(STRUCT, 2).struct_begin()
        s(twice)
        out.append(("%s_union_twice" % pn, p, UNION_SCHEMA, twice.struct_end().stop().bytes(), 1,
                    None, OK))
        cleared = W(p).field(STRUCT, 2).struct_begin()
        s(cleared)
        cleared.struct_end().field(STRUCT, 2).struct_begin().struct_end()
        out.append(("%s_union_cleared" % pn, p, UNION_SCHEMA, cleared.stop().bytes(), 1, None, OK))
        # a root union, back to back
        r1 = W(p).field(I32, 2).i32(-9).stop().bytes()
        r2 = W(p).stop().bytes()
        r3 = W(p).field(I64, 1).i64(1).field(I32, 2).i32(2).stop().bytes()
        out.append(("%s_root_union" % pn, p, ROOT_UNION, r1 + r2 + r1, 3, None, OK))
        out.append(("%s_root_union_two" % pn, p, ROOT_UNION, r1 + r3, 2, None, UNION_MISSING_STOP))
    # thrift/test/tablebased/SerializerTest.cpp:399-418 DuplicateUnionData, the
    # reference's one checked-in wire vector: TestStructWithUnion
    # {1: TestUnion union_field} with TestUnion {1: string string_field,
    # 2: float float_field} (thrift_tablebased.thrift:105-112). The union field
    # twice, the second holding a float whose value is missing; sizeof(data)
    # keeps the literal's NUL, so one byte of the float is present.
    # EXPECT_THROW(..., std::out_of_range).
    dup = (b"\x0c" b"\x00\x01" b"\x0b" b"\x00\x01" b"\x00\x00\x00\x00" b"\x00"
           b"\x0c" b"\x00\x01" b"\x13" b"\x00\x02" b"\x00")
    out.append(("binary_duplicate_union_data", B, DUP_UNION_SCHEMA, dup, 1, None, UNDERFLOW))
    return out


FLOAT = 19
DUP_UNION_SCHEMA = [[[1, STRUCT, 0, 0, 1]],
                    {"union": True, "fields": [[1, STR, 0, 0, -1], [2, FLOAT, 0, 0, -1]]}]


LSTR = [[[1, LIST, STR, 0, -1], [2, MAP, STR, 0, -1, I32], [3, I32, 0, 0, -1]]]


def string_elem_cases():
    """Strings inside containers: each element read as a string field is
    (readString: size checks, canAdvance -> TRUNCATED), the container's
    canReadNElements counts one byte per element (two per pair)."""
    out = []
    for p, pn in ((B, "binary"), (C, "compact")):
        ok = W(p).field(LIST, 1).list_begin(STR, 3).string(b"ab").string(b"").string(b"xyz") \
            .field(MAP, 2).map_begin(STR, I32, 2).string(b"k").i32(1).string(b"").i32(-2) \
            .field(I32, 3).i32(5).stop().bytes()
        out.append(("%s_strlist_ok" % pn, p, LSTR, ok, 1, None, OK))
        for cut in range(3, len(ok) - 1, 2):
            out.append(("%s_strlist_cut_%d" % (pn, cut), p, LSTR, ok[:cut], 1, None, None))
        out.append(("%s_strlist_limit" % pn, p, LSTR, ok, 1, (2, 0, 12000, 0), LIMIT))
        # a list of i32 where strings are expected: skipped, no error
        mm = W(p).field(LIST, 1).list_begin(I32, 2).i32(1).i32(2).stop().bytes()
        out.append(("%s_strlist_mismatch" % pn, p, LSTR, mm, 1, None, OK))
    neg = W(B).field(LIST, 1).list_begin(STR, 1).raw(b"\xff\xff\xff\xfe").stop().bytes()
    out.append(("binary_strlist_negative", B, LSTR, neg, 1, None, NEG))
    return out
