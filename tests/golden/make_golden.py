#!/usr/bin/env python3
"""Generate golden wire vectors with fbthrift's own pure-Python protocols.

The reference's legacy Python library (thrift/lib/py/protocol/TBinaryProtocol.py
and TCompactProtocol.py) is imported from the read-only reference checkout via
a symlink shim and drives the writers field by field in IDL declaration order,
always writing unqualified fields — exactly what the generated T::write does
(serialize_struct.whisker:40-67). Its output is the parity anchor for the
oracle (oracle/thrift_oracle.cpp) and, through it, for the HIP kernels.

Run ONLY in the build container (the reference is absent on GPU boxes):

    python3 -B tests/golden/make_golden.py

Writes, under tests/golden/:
  manifest.json            schemas, cases, sha256 of larger streams
  <case>.wire.bin          concatenated records as written by the reference
  <case>.offsets.npy       record start offsets (n+1, uint64)
  <case>.values.npz        expected field values (inputs of the writer)

Data only: no reference source is copied. Python != C++ in a few malformed-
input behaviours; those are restated from the C++ source in
tests/test_oracle_semantics.py instead.
"""
import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_PY = "/root/reference/thrift/lib/py"
SHIM = "/tmp/fbthrift_amd_oracle_shim"

sys.dont_write_bytecode = True  # never write __pycache__ into the reference


def import_reference():
    os.makedirs(SHIM, exist_ok=True)
    link = os.path.join(SHIM, "thrift")
    if not os.path.islink(link):
        os.symlink(REF_PY, link)
    sys.path.insert(0, SHIM)
    from thrift.protocol import TBinaryProtocol, TCompactProtocol  # noqa
    from thrift.transport import TTransport  # noqa
    return TBinaryProtocol, TCompactProtocol, TTransport


TBinaryProtocol, TCompactProtocol, TTransport = import_reference()
sys.path.insert(0, HERE)

from datagen import *  # noqa: F401,F403  (schemas + generators)
import nestgen  # noqa: E402


# ----------------------------------------------------------------- writing --
def write_value(p, ttype, elem, sidx, schema, v):
    if ttype == T_BOOL:
        p.writeBool(v)
    elif ttype == T_BYTE:
        p.writeByte(v)
    elif ttype == T_I16:
        p.writeI16(v)
    elif ttype == T_I32:
        p.writeI32(v)
    elif ttype == T_I64:
        p.writeI64(v)
    elif ttype == T_DOUBLE:
        p.writeDouble(v)
    elif ttype == T_FLOAT:
        p.writeFloat(v)
    elif ttype == T_STRING:
        p.writeString(v)
    elif ttype == T_STRUCT:
        write_struct(p, schema, sidx, v)
    elif ttype == T_MAP:
        kt, vt = elem
        p.writeMapBegin(kt, vt, len(v))
        for a, b in v:
            write_value(p, kt, 0, -1, schema, a)
            write_value(p, vt, 0, -1, schema, b)
        p.writeMapEnd()
    elif ttype in (T_LIST, T_SET):
        (p.writeListBegin if ttype == T_LIST else p.writeSetBegin)(elem, len(v))
        for e in v:
            write_value(p, elem, 0, -1, schema, e)
        (p.writeListEnd if ttype == T_LIST else p.writeSetEnd)()
    else:
        raise ValueError(ttype)


def write_struct(p, schema, sidx, vals):
    p.writeStructBegin("S%d" % sidx)
    for row, v in zip(rows(schema, sidx), vals):
        fid, ttype, elem, qual, sub = row[:5]
        if v is None:
            assert qual == 1 or is_union(schema, sidx)
            continue
        p.writeFieldBegin("f", ttype, fid)
        write_value(p, ttype, (elem, row[5]) if ttype == T_MAP else elem, sub, schema, v)
        p.writeFieldEnd()
    p.writeFieldStop()
    p.writeStructEnd()


def write_spec(p, table, spec, v):
    """A value of type `spec` (tests/golden/nestgen.py) through the
    reference's protocol methods; structs field by field in declaration
    order, optional fields only when set."""
    t = spec[0]
    if t == T_STRUCT:
        p.writeStructBegin("S%d" % spec[1])
        for row, x in zip(table[spec[1]], v):
            if x is None:
                assert row[3] in (1, 5)  # optional / optional boxed
                continue
            p.writeFieldBegin("f", row[1], row[0])
            write_spec(p, table, nestgen.field_spec(row), x)
            p.writeFieldEnd()
        p.writeFieldStop()
        p.writeStructEnd()
    elif t == T_MAP:
        p.writeMapBegin(spec[1][0], spec[2][0], len(v))
        for a, b in v:
            write_spec(p, table, spec[1], a)
            write_spec(p, table, spec[2], b)
        p.writeMapEnd()
    elif t in (T_LIST, T_SET):
        (p.writeListBegin if t == T_LIST else p.writeSetBegin)(spec[1][0], len(v))
        for e in v:
            write_spec(p, table, spec[1], e)
        (p.writeListEnd if t == T_LIST else p.writeSetEnd)()
    else:
        write_value(p, t, 0, -1, table, v)


def serialize_nested(proto, table, records):
    chunks, offsets, pos = [], [0], 0
    for rec in records:
        t = TTransport.TMemoryBuffer()
        p = (TBinaryProtocol.TBinaryProtocol(t) if proto == "binary"
             else TCompactProtocol.TCompactProtocol(t))
        write_spec(p, table, (T_STRUCT, 0), rec)
        b = t.getvalue()
        chunks.append(b)
        pos += len(b)
        offsets.append(pos)
    return b"".join(chunks), np.array(offsets, dtype=np.uint64)


def serialize(proto, schema, records):
    chunks, offsets, pos = [], [0], 0
    for rec in records:
        t = TTransport.TMemoryBuffer()
        p = (TBinaryProtocol.TBinaryProtocol(t) if proto == "binary"
             else TCompactProtocol.TCompactProtocol(t))
        if proto == "compact_v1":
            # version 1 of the Compact protocol: doubles in native (LE) order
            # (TCompactProtocol.py VERSION_LOW vs VERSION_DOUBLE_BE)
            p._TCompactProtocol__version = TCompactProtocol.TCompactProtocol.VERSION_LOW
        write_struct(p, schema, 0, rec)
        b = t.getvalue()
        chunks.append(b)
        pos += len(b)
        offsets.append(pos)
    return b"".join(chunks), np.array(offsets, dtype=np.uint64)


CASES = [
    # name, schema, proto, generator, n
    ("flat8_binary", "flat8", "binary", gen_flat8, 1000),
    ("flat8_compact", "flat8", "compact", gen_flat8, 1000),
    ("mixed_compact", "mixed", "compact", gen_mixed, 1000),
    ("mixed_binary", "mixed", "binary", gen_mixed, 1000),
    ("nested_binary", "nested", "binary", gen_nested, 1000),
    ("nested_compact", "nested", "compact", gen_nested, 1000),
    ("scalars_binary", "scalars", "binary", gen_scalars, 300),
    ("scalars_compact", "scalars", "compact", gen_scalars, 300),
    ("sparse_binary", "sparse", "binary", gen_sparse, 200),
    ("sparse_compact", "sparse", "compact", gen_sparse, 200),
    ("maps_binary", "maps", "binary", gen_maps, 300),
    ("maps_compact", "maps", "compact", gen_maps, 300),
    ("unions_binary", "unions", "binary", gen_unions, 200),
    ("unions_compact", "unions", "compact", gen_unions, 200),
    ("strcont_binary", "strcont", "binary", gen_strcont, 200),
    ("strcont_compact", "strcont", "compact", gen_strcont, 200),
    ("scalars_compact_v1", "scalars", "compact_v1", gen_scalars, 300),
    ("nested_compact_v1", "nested", "compact_v1", gen_nested, 500),
    ("maps_compact_v1", "maps", "compact_v1", gen_maps, 100),
    ("unions_compact_v1", "unions", "compact_v1", gen_unions, 100),
    ("flat8_compact_v1", "flat8", "compact_v1", gen_flat8, 300),
    ("original_compact", "original", "compact", lambda i: ORIGINAL, 1),
    ("original_binary", "original", "binary", lambda i: ORIGINAL, 1),
    ("updated_compact", "updated", "compact", lambda i: UPDATED, 1),
    ("updated_binary", "updated", "binary", lambda i: UPDATED, 1),
]

NESTED_CASES = [
    # containers of structs / of containers (tests/golden/nestgen.py)
    ("structlist_binary", "structlist", "binary", 400),
    ("structlist_compact", "structlist", "compact", 400),
    ("deepcont_binary", "deepcont", "binary", 300),
    ("deepcont_compact", "deepcont", "compact", 300),
    # struct / container map keys, recursion through a list and through
    # boxed fields (cpp.ref / thrift.box)
    ("keyed_binary", "keyed", "binary", 300),
    ("keyed_compact", "keyed", "compact", 300),
    ("tree_binary", "tree", "binary", 200),
    ("tree_compact", "tree", "compact", 200),
    ("chain_binary", "chain", "binary", 200),
    ("chain_compact", "chain", "compact", 200),
]

DIGESTS = [
    # name, schema, proto, generator, n: sha256 of the whole stream
    ("flat8_binary_50k", "flat8", "binary", gen_flat8, 50000),
    ("mixed_compact_50k", "mixed", "compact", gen_mixed, 50000),
    ("nested_binary_20k", "nested", "binary", gen_nested, 20000),
]


def varint_vectors():
    """VarintUtilsTest.cpp:34-115: every bit position for 16/32/64-bit values,
    encoded by the reference Python writer (zigzag'd and raw)."""
    rows = []
    for bits in (16, 32, 64):
        for pos in range(bits):
            for v in ((1 << pos), (1 << pos) - 1, (1 << (pos + 1)) - 1):
                v &= (1 << bits) - 1
                t = TTransport.TMemoryBuffer()
                p = TCompactProtocol.TCompactProtocol(t)
                p._TCompactProtocol__writeVarint(v)
                rows.append([bits, v, t.getvalue().hex()])
    return rows


def main():
    manifest = {"generator": "tests/golden/make_golden.py",
                "reference": "thrift/lib/py/protocol (fbthrift, pure Python)",
                "seed": SEED, "schemas": SCHEMAS, "cases": {}, "digests": {}}
    for name, sch, proto, gen, n in CASES:
        schema = SCHEMAS[sch]
        recs = [gen(i) for i in range(n)]
        wire, offs = serialize(proto, schema, recs)
        with open(os.path.join(HERE, name + ".wire.bin"), "wb") as f:
            f.write(wire)
        np.save(os.path.join(HERE, name + ".offsets.npy"), offs)
        np.savez(os.path.join(HERE, name + ".values.npz"), **flatten_values(schema, recs))
        manifest["cases"][name] = {"schema": sch, "protocol": proto, "n": n,
                                   "bytes": len(wire),
                                   "sha256": hashlib.sha256(wire).hexdigest()}
        print(name, n, len(wire))
    manifest["nested_schemas"] = nestgen.NESTED_SCHEMAS
    manifest["nested_cases"] = {}
    for name, sch, proto, n in NESTED_CASES:
        table = nestgen.NESTED_SCHEMAS[sch]
        recs = [nestgen.NESTED_GENERATORS[sch](i) for i in range(n)]
        wire, offs = serialize_nested(proto, table, recs)
        with open(os.path.join(HERE, name + ".wire.bin"), "wb") as f:
            f.write(wire)
        np.save(os.path.join(HERE, name + ".offsets.npy"), offs)
        with open(os.path.join(HERE, name + ".values.json"), "w") as f:
            json.dump([nestgen.to_json((T_STRUCT, 0), r, table) for r in recs], f)
        manifest["nested_cases"][name] = {"schema": sch, "protocol": proto, "n": n,
                                          "bytes": len(wire),
                                          "sha256": hashlib.sha256(wire).hexdigest()}
        print(name, n, len(wire))
    for name, sch, proto, gen, n in DIGESTS:
        schema = SCHEMAS[sch]
        wire, offs = serialize(proto, schema, [gen(i) for i in range(n)])
        manifest["digests"][name] = {"schema": sch, "protocol": proto, "n": n,
                                     "bytes": len(wire),
                                     "sha256": hashlib.sha256(wire).hexdigest(),
                                     "offsets_sha256": hashlib.sha256(offs.tobytes()).hexdigest()}
        print(name, n, len(wire))
    manifest["varints"] = varint_vectors()
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
