"""Deterministic record generators and schemas shared by the golden-vector
script (tests/golden/make_golden.py), the parity tests and bench.py.

Pure Python + numpy; no reference code. Spec: counter-based
splitmix64 with seed 0x1729 (thrift/lib/cpp/util/test/VarintUtilsTestUtil.h:59).
"""
import struct
import sys

import numpy as np

# TType values (thrift/lib/cpp/protocol/TType.h:31-51)
T_BOOL, T_BYTE, T_DOUBLE, T_I16, T_I32, T_I64 = 2, 3, 4, 6, 8, 10
T_STRING, T_STRUCT, T_LIST, T_SET, T_FLOAT = 11, 12, 15, 14, 19
T_MAP = 13

M64 = (1 << 64) - 1
SEED = 0x1729


def splitmix64_at(seed, index):
    """Counter-based splitmix64 (same spec as oracle_splitmix64_at)."""
    z = (seed + (index + 1) * 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def s64(u):
    return u - (1 << 64) if u >= (1 << 63) else u


def s32(u):
    u &= 0xFFFFFFFF
    return u - (1 << 32) if u >= (1 << 31) else u


def unzigzag32(z):
    return s32((z >> 1) ^ -(z & 1))


def bits_to_double(b):
    return struct.unpack("<d", struct.pack("<Q", b))[0]


def bits_to_float(b):
    return struct.unpack("<f", struct.pack("<I", b))[0]


# ----------------------------------------------------------------- schemas --
# A schema is a list of structs; struct 0 is the record. Field entries:
# [id, ttype, elem_ttype, qualifier, struct_index]
SCHEMAS = {
    "flat8": [[[k, T_I64, 0, 0, -1] for k in range(1, 9)]],
    "mixed": [[[1, T_I32, 0, 0, -1], [2, T_I32, 0, 0, -1], [3, T_I32, 0, 0, -1],
               [4, T_I32, 0, 0, -1], [5, T_STRING, 0, 0, -1],
               [6, T_STRING, 0, 0, -1]]],
    "nested": [
        [[1, T_I64, 0, 0, -1], [2, T_LIST, T_I32, 0, -1], [3, T_STRUCT, 0, 0, 1]],
        [[1, T_DOUBLE, 0, 0, -1], [2, T_DOUBLE, 0, 0, -1], [3, T_DOUBLE, 0, 0, -1]],
    ],
    "scalars": [[[1, T_BOOL, 0, 0, -1], [2, T_BYTE, 0, 0, -1], [3, T_I16, 0, 0, -1],
                 [4, T_I32, 0, 0, -1], [5, T_I64, 0, 0, -1], [6, T_DOUBLE, 0, 0, -1],
                 [7, T_FLOAT, 0, 0, -1], [8, T_STRING, 0, 0, -1], [9, T_BOOL, 0, 0, -1],
                 [10, T_LIST, T_BOOL, 0, -1], [11, T_LIST, T_I64, 0, -1],
                 [12, T_LIST, T_DOUBLE, 0, -1], [13, T_LIST, T_BYTE, 0, -1],
                 [14, T_LIST, T_I16, 0, -1], [15, T_LIST, T_FLOAT, 0, -1]]],
    # thrift/lib/cpp2/protocol/test/CompactProtocolTestStructs.thrift
    "original": [
        [[1, T_BOOL, 0, 0, -1], [3, T_BOOL, 0, 0, -1], [6, T_BYTE, 0, 0, -1],
         [8, T_I16, 0, 0, -1], [48, T_I32, 0, 0, -1], [100, T_I64, 0, 0, -1],
         [20000, T_DOUBLE, 0, 0, -1], [20030, T_STRUCT, 0, 0, 1],
         [20032, T_STRING, 0, 0, -1], [20034, T_LIST, T_I32, 0, -1]],
        [[1, T_I64, 0, 0, -1]],
    ],
    "updated": [
        [[1, T_BOOL, 0, 0, -1], [2, T_BOOL, 0, 0, -1], [3, T_BOOL, 0, 0, -1],
         [4, T_BOOL, 0, 0, -1], [5, T_BOOL, 0, 0, -1], [6, T_BYTE, 0, 0, -1],
         [7, T_I32, 0, 0, -1], [8, T_I16, 0, 0, -1], [48, T_I32, 0, 0, -1],
         [68, T_I32, 0, 0, -1], [88, T_I32, 0, 0, -1], [100, T_I64, 0, 0, -1],
         [20000, T_DOUBLE, 0, 0, -1], [20020, T_STRING, 0, 0, -1],
         [20030, T_STRUCT, 0, 0, 1], [20031, T_STRUCT, 0, 0, 1],
         [20032, T_STRING, 0, 0, -1], [20033, T_STRING, 0, 0, -1],
         [20034, T_LIST, T_I32, 0, -1], [20035, T_LIST, T_I32, 0, -1]],
        [[1, T_I64, 0, 0, -1]],
    ],
    # optional fields + ids that force Compact long-form headers (negative,
    # gaps > 15, descending declaration order).
    # maps of scalars ([id, T_MAP, key type, qualifier, -1, value type]),
    # nested in a struct field too; an optional map
    "maps": [
        [[1, T_MAP, T_I32, 0, -1, T_I64], [2, T_MAP, T_I16, 0, -1, T_DOUBLE],
         [3, T_MAP, T_BOOL, 0, -1, T_BYTE], [4, T_I32, 0, 0, -1],
         [5, T_MAP, T_I64, 1, -1, T_FLOAT], [6, T_STRUCT, 0, 0, 1],
         [7, T_MAP, T_BYTE, 0, -1, T_BOOL]],
        [[1, T_MAP, T_I32, 0, -1, T_I32], [2, T_I64, 0, 0, -1]],
    ],
    # unions (TGPU_STRUCT_UNION): one active member or none; a union member
    # that is a struct holding a map; a union of the root struct twice
    "unions": [
        [[1, T_I32, 0, 0, -1], [2, T_STRUCT, 0, 0, 1], [3, T_STRUCT, 0, 0, 1],
         [4, T_I64, 0, 0, -1]],
        {"union": True, "fields": [
            [1, T_I64, 0, 0, -1], [2, T_STRING, 0, 0, -1], [3, T_DOUBLE, 0, 0, -1],
            [4, T_STRUCT, 0, 0, 2], [5, T_LIST, T_I32, 0, -1], [6, T_BOOL, 0, 0, -1],
            [20, T_MAP, T_I16, 0, -1, T_I16]]},
        [[1, T_I32, 0, 0, -1], [2, T_MAP, T_I16, 0, -1, T_I16]],
    ],
    # strings inside containers (tgpu_span elements)
    "strcont": [
        [[1, T_LIST, T_STRING, 0, -1], [2, T_MAP, T_STRING, 0, -1, T_I64],
         [3, T_MAP, T_I32, 0, -1, T_STRING], [4, T_SET, T_STRING, 0, -1],
         [5, T_STRING, 0, 0, -1], [6, T_MAP, T_STRING, 0, -1, T_STRING],
         [7, T_LIST, T_I16, 0, -1]],
    ],
    "sparse": [[[5, T_I32, 0, 1, -1], [-3, T_I64, 0, 0, -1], [40, T_STRING, 0, 1, -1],
                [300, T_BOOL, 0, 0, -1], [20, T_DOUBLE, 0, 1, -1], [21, T_I16, 0, 0, -1]]],
}


def rows(schema, si):
    """The field rows of struct si (a union is {"union": true, "fields": rows})."""
    e = schema[si]
    return e["fields"] if isinstance(e, dict) else e


def is_union(schema, si):
    return isinstance(schema[si], dict) and bool(schema[si].get("union"))


# ------------------------------------------------------------ value models --
# A record value is a list aligned with the struct's fields; None = unset
# (only legal for optional fields). Nested struct -> list; list -> python list;
# string -> bytes.
EDGES64 = [0, -1, 1, -(1 << 63), (1 << 63) - 1]


def gen_flat8(i):
    if i % 997 < 5:
        return [EDGES64[(i % 997 + k) % 5] for k in range(8)]
    return [s64(splitmix64_at(SEED, 8 * i + k)) for k in range(8)]


def gen_mixed(i):
    vals = []
    for k in range(4):
        r = splitmix64_at(SEED, 16 * i + 2 * k)
        r2 = splitmix64_at(SEED, 16 * i + 2 * k + 1)
        b = 1 + r % 5
        lo = 0 if b == 1 else 1 << (7 * (b - 1))
        hi = min((1 << (7 * b)) - 1, 0xFFFFFFFF)
        vals.append(unzigzag32(lo + r2 % (hi - lo + 1)))
    for k in range(2):
        n = splitmix64_at(SEED, 16 * i + 8 + k) % 33
        words = [splitmix64_at(SEED ^ 0x5EED, (2 * i + k) * 4 + w) for w in range(4)]
        vals.append(bytes((words[j // 8] >> (8 * (j % 8))) & 0xFF for j in range(n)))
    return vals


def finite_bits(b):
    if (b >> 52) & 0x7FF == 0x7FF:
        b &= ~(1 << 62)
    return b


def gen_nested(i):
    n = splitmix64_at(SEED, 32 * i + 1) % 17
    lst = [s32(splitmix64_at(SEED, 32 * i + 2 + j)) for j in range(n)]
    inner = [bits_to_double(finite_bits(splitmix64_at(SEED, 32 * i + 20 + k)))
             for k in range(3)]
    return [s64(splitmix64_at(SEED, 32 * i)), lst, inner]


def interesting():
    """ValueGenerator.cpp:27-90 values, per type."""
    i8 = [0, -128, 127, 1, -1]
    i16 = [0, -32768, 32767, 1, -1]
    i32 = [0, -(1 << 31), (1 << 31) - 1, 1, -1]
    i64 = [0, -(1 << 63), (1 << 63) - 1, 1, -1]
    dmax = sys.float_info.max
    dbl = [0.0, -dmax, sys.float_info.min, dmax, float(1 << 53), -float(1 << 53),
           float((1 << 53) - 1), -float((1 << 53) - 1), 0.1,
           bits_to_double(0x0010000000000001), bits_to_double(0x7FEFFFFFFFFFFFFE),
           float("inf"), float("-inf"), 1.0, -1.0, sys.float_info.epsilon,
           -sys.float_info.epsilon, 5e-324, -5e-324, 1.9156918820264798e-56,
           3788512123356.9854, -0.0]
    fmax = bits_to_float(0x7F7FFFFF)
    flt = [0.0, -fmax, bits_to_float(0x00800000), fmax, float(1 << 24), -float(1 << 24),
           0.1, float("inf"), float("-inf"), 1.0, -1.0, bits_to_float(0x34000000),
           bits_to_float(0x00000001), -bits_to_float(0x00000001), -0.0]
    flt = [bits_to_float(struct.unpack("<I", struct.pack("<f", f))[0]) for f in flt]
    strs = [b"", b"a", b"A", b" a ", b" a", b"a ", b"Hello", b"\x72\x01\xff",
            bytes(range(256)), b"x" * 200]
    return i8, i16, i32, i64, dbl, flt, strs


def gen_scalars(i):
    i8, i16, i32, i64, dbl, flt, strs = interesting()
    r = [splitmix64_at(SEED + 7, 16 * i + k) for k in range(16)]
    nb = r[9] % 20
    return [
        bool(r[0] & 1), i8[i % len(i8)], i16[(i // 2) % len(i16)],
        i32[(i // 3) % len(i32)], i64[(i // 5) % len(i64)], dbl[i % len(dbl)],
        flt[(i // 2) % len(flt)], strs[i % len(strs)], bool((r[0] >> 1) & 1),
        [bool((r[10] >> j) & 1) for j in range(nb)],
        [s64(splitmix64_at(SEED + 9, 64 * i + j)) for j in range(r[11] % 20)],
        [dbl[(i + j) % len(dbl)] for j in range(r[12] % 18)],
        [s64(splitmix64_at(SEED + 11, 64 * i + j)) % 256 - 128 for j in range(r[13] % 40)],
        [i16[(i + j) % len(i16)] for j in range(r[14] % 16)],
        [flt[(i + j) % len(flt)] for j in range(r[15] % 16)],
    ]


def gen_sparse(i):
    r = splitmix64_at(SEED + 3, i)
    return [
        s32(splitmix64_at(SEED + 4, i)) if r & 1 else None,
        s64(splitmix64_at(SEED + 5, i)),
        bytes([65 + (i + j) % 26 for j in range(i % 20)]) if r & 2 else None,
        bool(r & 4),
        bits_to_double(finite_bits(splitmix64_at(SEED + 6, i))) if r & 8 else None,
        s32(splitmix64_at(SEED + 8, i)) % 65536 - 32768,
    ]


def gen_maps(i):
    """Pairs in wire order; keys may repeat (the wire allows it, the reader
    keeps them all in the span form); sizes cross the 1-byte varint at 127."""
    i8, i16, i32, i64, dbl, flt, strs = interesting()
    r = [splitmix64_at(SEED + 21, 16 * i + k) for k in range(16)]
    big = i % 50 == 7

    def n(k, m):
        return 130 if big and k == 0 else r[k] % m

    m1 = [(s32(splitmix64_at(SEED + 22, 256 * i + j)) % 1000 - 500,
           s64(splitmix64_at(SEED + 23, 256 * i + j))) for j in range(n(0, 20))]
    m2 = [(i16[(i + j) % len(i16)], dbl[(i + 3 * j) % len(dbl)]) for j in range(n(1, 9))]
    m3 = [(bool((r[5] >> j) & 1), i8[(i + j) % len(i8)]) for j in range(n(2, 3))]
    m5 = ([(i64[(i + j) % len(i64)], flt[(i + j) % len(flt)]) for j in range(n(3, 6))]
          if r[6] & 1 else None)
    inner = [[(s32(splitmix64_at(SEED + 24, 64 * i + j)), j - 3) for j in range(n(4, 5))],
             s64(r[7])]
    m7 = [(s64(splitmix64_at(SEED + 25, 64 * i + j)) % 256 - 128, bool(j & 1))
          for j in range(n(8, 4))]
    return [m1, m2, m3, s32(r[9]), m5, inner, m7]


def gen_unions(i):
    """Two unions per record, each with member (i + j) % 8 active (7 = empty)."""
    r = [splitmix64_at(SEED + 31, 8 * i + k) for k in range(8)]

    def union(j):
        k = (i + j) % 8
        v = [None] * 7
        if k == 0:
            v[0] = s64(r[j])
        elif k == 1:
            v[1] = bytes([97 + (i + t) % 26 for t in range(r[j] % 12)])
        elif k == 2:
            v[2] = bits_to_double(finite_bits(r[j]))
        elif k == 3:
            v[3] = [s32(r[j]), [(t - 5, t * 3) for t in range(r[j] % 4)]]
        elif k == 4:
            v[4] = [s32(splitmix64_at(SEED + 32, 16 * i + t)) for t in range(r[j] % 6)]
        elif k == 5:
            v[5] = bool(r[j] & 1)
        elif k == 6:
            v[6] = [(t, -t) for t in range(r[j] % 3)]
        return v

    return [s32(r[5]), union(0), union(3), s64(r[6])]


def gen_strcont(i):
    r = [splitmix64_at(SEED + 41, 16 * i + k) for k in range(16)]

    def word(k, j):
        x = splitmix64_at(SEED + 42, 64 * i + 8 * k + j)
        return bytes(97 + (x >> (5 * t)) % 26 for t in range(x % 9))

    big = i % 40 == 11
    return [[word(0, j) for j in range(20 if big else r[0] % 6)],
            [(word(1, j), s64(r[1 + j % 3])) for j in range(r[4] % 4)],
            [(s32(r[5]) + j, word(2, j)) for j in range(r[6] % 4)],
            [word(3, j) for j in range(r[7] % 3)],
            word(4, 0),
            [(word(5, j), word(6, j)) for j in range(r[8] % 3)],
            [j - 2 for j in range(r[9] % 5)]]


ORIGINAL = [True, False, 50, 1200, 1300, 1600, 1.0, [0], b"def", [0]]
UPDATED = [True, False, False, True, False, 50, 1100, 1200, 1300, 1400, 1500,
           1600, 1.0, b"abc", [0], [1], b"def", b"ghi", [0], [1]]




# ---------------------------------------------------------- value storage --
def flatten_values(schema, records):
    """Columnar expected values: for field path P (e.g. '0.3' or '0.3/1.2'),
    P.set (uint8), P.val (scalars), P.len/P.data (strings), P.count/P.elems
    (lists). Doubles/floats are stored as raw bits."""
    out = {}

    def put(key, v):
        out.setdefault(key, []).append(v)

    def scalar_repr(ttype, v):
        if ttype == T_DOUBLE:
            return struct.unpack("<Q", struct.pack("<d", v))[0]
        if ttype == T_FLOAT:
            return struct.unpack("<I", struct.pack("<f", v))[0]
        if ttype == T_BOOL:
            return int(bool(v))
        return v

    def column(key, t, items):
        # container elements: scalars as one column; strings as
        # <key>.len (u32 per element) + <key>.data (bytes)
        if t == T_STRING:
            out.setdefault(key + ".len", []).extend(len(e) for e in items)
            out.setdefault(key + ".data", []).extend(b for e in items for b in e)
        else:
            out.setdefault(key, []).extend(scalar_repr(t, e) for e in items)

    def walk(sidx, vals, prefix):
        for k, row in enumerate(rows(schema, sidx)):
            fid, ttype, elem, qual, sub = row[:5]
            v = vals[k] if vals is not None else None
            key = "%s%d" % (prefix, k)
            put(key + ".set", 0 if v is None else 1)
            if ttype == T_STRUCT:
                walk(sub, v, key + "/")
            elif ttype == T_STRING:
                put(key + ".len", 0 if v is None else len(v))
                out.setdefault(key + ".data", []).extend(v or b"")
            elif ttype == T_MAP:
                put(key + ".count", 0 if v is None else len(v))
                column(key + ".keys", elem, [a for a, _ in (v or [])])
                column(key + ".vals", row[5], [b for _, b in (v or [])])
            elif ttype in (T_LIST, T_SET):
                put(key + ".count", 0 if v is None else len(v))
                column(key + ".elems", elem, v or [])
            else:
                put(key + ".val", 0 if v is None else scalar_repr(ttype, v))

    for rec in records:
        walk(0, rec, "")
    arrays = {}
    dt = {T_BOOL: np.uint8, T_BYTE: np.int8, T_I16: np.int16, T_I32: np.int32,
          T_I64: np.int64, T_DOUBLE: np.uint64, T_FLOAT: np.uint32}

    def ftype(path):
        sidx, ft = 0, None
        parts = path.split("/")
        for j, part in enumerate(parts):
            f = rows(schema, sidx)[int(part)]
            ft = f
            if j < len(parts) - 1:
                sidx = f[4]
        return ft

    for key, lst in out.items():
        path, kind = key.rsplit(".", 1)
        f = ftype(path) if kind in ("elems", "keys", "vals", "val") else None
        if kind in ("set",):
            arrays[key] = np.array(lst, dtype=np.uint8)
        elif kind in ("len", "count"):
            arrays[key] = np.array(lst, dtype=np.uint32)
        elif kind == "data":
            arrays[key] = np.array(lst, dtype=np.uint8)
        elif kind in ("elems", "keys"):
            arrays[key] = np.array(lst, dtype=dt[f[2]])
        elif kind == "vals":
            arrays[key] = np.array(lst, dtype=dt[f[5]])
        else:
            arrays[key] = np.array(lst, dtype=dt[f[1]])
    return arrays
