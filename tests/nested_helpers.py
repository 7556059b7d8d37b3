"""Nested-container golden cases (tests/golden/nestgen.py, written by the
reference's Python protocols) and the device layout of their values: records
in the struct layout, containers as spans into the list arena (scalars
native, strings/containers as 16-byte spans, structs in the struct layout,
maps as packed {key, value} pairs), strings as spans into the string base
(encode) or the wire (decode)."""
import json
import os
import struct

import numpy as np

import nestgen
from fbthrift_amd.schema import Schema

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T_BOOL, T_BYTE, T_DOUBLE, T_I16, T_I32, T_I64 = 2, 3, 4, 6, 8, 10
T_STRING, T_STRUCT, T_MAP, T_SET, T_LIST, T_FLOAT = 11, 12, 13, 14, 15, 19
SCALAR = {T_BOOL: (1, "<B"), T_BYTE: (1, "<b"), T_I16: (2, "<h"), T_I32: (4, "<i"),
          T_I64: (8, "<q"), T_DOUBLE: (8, "<Q"), T_FLOAT: (4, "<I")}
PROTO = {"binary": 0, "compact": 2}


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def case_names():
    return sorted(manifest()["nested_cases"].keys())


class NestedCase:
    def __init__(self, name):
        m = manifest()
        c = m["nested_cases"][name]
        self.name, self.n = name, c["n"]
        self.protocol = PROTO[c["protocol"]]
        self.table = m["nested_schemas"][c["schema"]]
        self.schema = Schema.from_table(self.table)
        with open(os.path.join(GOLDEN, name + ".wire.bin"), "rb") as f:
            self.wire = f.read()
        self.offsets = np.load(os.path.join(GOLDEN, name + ".offsets.npy"))
        with open(os.path.join(GOLDEN, name + ".values.json")) as f:
            self.values = json.load(f)
        self.layout = Layout(self.schema, self.table)


class Layout:
    """Struct sizes / member / isset offsets by table struct index."""

    def __init__(self, schema, table):
        self.table = table
        by_name = {s.name: k for k, s in enumerate(schema.structs)}
        self.size, self.member, self.isset = {}, {}, {}
        for t in range(len(table)):
            si = by_name["S%d" % t]
            self.size[t] = schema.size[si]
            for k in range(len(schema.structs[si].fields)):
                self.member[(t, k)] = schema.member[(si, k)]
                self.isset[(t, k)] = schema.isset[(si, k)]

    def slot(self, spec):
        t = spec[0]
        if t == T_STRUCT:
            return self.size[spec[1]]
        if t in (T_STRING, T_LIST, T_SET, T_MAP):
            return 16
        return SCALAR[t][0]


def _span(buf, off):
    o, n, _ = struct.unpack_from("<QII", buf, off)
    return o, n


def materialize(lay, rec, off, wire, arena, spec=(T_STRUCT, 0)):
    """The value of type `spec` at rec[off:] as nestgen's JSON form
    (decode output: strings are views into `wire`, containers in `arena`)."""
    t = spec[0]
    if t in SCALAR:
        size, fmt = SCALAR[t]
        return struct.unpack_from(fmt, rec, off)[0]
    if t == T_STRING:
        o, n = _span(rec, off)
        return bytes(wire[o:o + n]).hex()
    if t == T_STRUCT and len(spec) > 2 and spec[2]:  # boxed: a pointer into the arena
        o, n = _span(rec, off)
        return materialize(lay, arena, o, wire, arena, (T_STRUCT, spec[1])) if n else None
    if t == T_STRUCT:
        out = []
        for k, row in enumerate(lay.table[spec[1]]):
            if not rec[off + lay.isset[(spec[1], k)]]:
                out.append(None)
                continue
            out.append(materialize(lay, rec, off + lay.member[(spec[1], k)], wire, arena,
                                   nestgen.field_spec(row)))
        return out
    o, n = _span(rec, off)
    if t == T_MAP:
        ks, vs = lay.slot(spec[1]), lay.slot(spec[2])
        return [[materialize(lay, arena, o + i * (ks + vs), wire, arena, spec[1]),
                 materialize(lay, arena, o + i * (ks + vs) + ks, wire, arena, spec[2])]
                for i in range(n)]
    es = lay.slot(spec[1])
    return [materialize(lay, arena, o + i * es, wire, arena, spec[1]) for i in range(n)]


def materialize_batch(case, rec_bytes, arena, n=None):
    n = case.n if n is None else n
    rec = bytes(rec_bytes)
    ar = bytes(arena)
    S = case.layout.size[0]
    return [materialize(case.layout, rec, i * S, case.wire, ar) for i in range(n)]


def pack(case):
    """Records + string base + list arena holding case.values (encode input)."""
    lay = case.layout
    strings, lists = bytearray(), bytearray()

    def alloc(nbytes):
        o = (len(lists) + 7) & ~7
        lists.extend(b"\0" * (o + nbytes - len(lists)))
        return o

    def put(buf, off, spec, v):
        t = spec[0]
        if t in SCALAR:
            struct.pack_into(SCALAR[t][1], buf, off, v)
        elif t == T_STRING:
            b = bytes.fromhex(v)
            struct.pack_into("<QII", buf, off, len(strings), len(b), 0)
            strings.extend(b)
        elif t == T_STRUCT and len(spec) > 2 and spec[2]:  # boxed
            o = alloc(lay.size[spec[1]])
            struct.pack_into("<QII", buf, off, o, 1, 0)
            put(lists, o, (T_STRUCT, spec[1]), v)
        elif t == T_STRUCT:
            for k, row in enumerate(lay.table[spec[1]]):
                if v[k] is None:
                    continue
                buf[off + lay.isset[(spec[1], k)]] = 1
                put(buf, off + lay.member[(spec[1], k)], nestgen.field_spec(row), v[k])
        else:
            is_map = t == T_MAP
            es = lay.slot(spec[1]) + (lay.slot(spec[2]) if is_map else 0)
            o = alloc(es * len(v))
            struct.pack_into("<QII", buf, off, o, len(v), 0)
            for i, e in enumerate(v):
                # element bytes live in `lists` itself: write through it
                if is_map:
                    put(lists, o + i * es, spec[1], e[0])
                    put(lists, o + i * es + lay.slot(spec[1]), spec[2], e[1])
                else:
                    put(lists, o + i * es, spec[1], e)

    S = lay.size[0]
    rec = bytearray(S * case.n)
    for i, v in enumerate(case.values):
        put(rec, i * S, (T_STRUCT, 0), v)
    return (np.frombuffer(bytes(rec), np.uint8).copy(),
            np.frombuffer(bytes(strings) + b"\0" * 16, np.uint8).copy(),
            np.frombuffer(bytes(lists) + b"\0" * 16, np.uint8).copy())
