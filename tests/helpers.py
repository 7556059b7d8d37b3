"""Test helpers: golden-case loading and packing columnar values into the
record layout (and back)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, GOLDEN)

from fbthrift_amd.schema import SCALAR, Schema  # noqa: E402
from fbthrift_amd._lib import T_LIST, T_MAP, T_SET, T_STRING, T_STRUCT  # noqa: E402

PROTO = {"binary": 0, "compact": 2, "compact_v1": 0x102}
ELEM_NP = {2: np.uint8, 3: np.int8, 6: np.int16, 8: np.int32, 10: np.int64, 4: np.uint64,
           19: np.uint32}


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


class Case:
    def __init__(self, name):
        m = manifest()
        c = m["cases"][name]
        self.name = name
        self.protocol = PROTO[c["protocol"]]
        self.n = c["n"]
        self.table = m["schemas"][c["schema"]]
        self.schema = Schema.from_table(self.table)
        with open(os.path.join(GOLDEN, name + ".wire.bin"), "rb") as f:
            self.wire = f.read()
        self.offsets = np.load(os.path.join(GOLDEN, name + ".offsets.npy"))
        z = np.load(os.path.join(GOLDEN, name + ".values.npz"))
        self.values = {k: z[k] for k in z.files}


def case_names():
    return sorted(manifest()["cases"].keys())


def _paths(schema, si=0, prefix=()):
    for k, f in enumerate(schema.structs[si].fields):
        p = prefix + (k,)
        yield p, f
        if f.ttype == T_STRUCT:
            yield from _paths(schema, schema.struct_index(f.struct), p)


def _key(path):
    return "/".join(str(k) for k in path)


def _view(rec, schema, path):
    """(array holding the field, field, struct index, k) for a field path."""
    si, arr = 0, rec
    for j, k in enumerate(path):
        f = schema.structs[si].fields[k]
        if j == len(path) - 1:
            return arr, f, si, k
        arr = arr[f.name]
        si = schema.struct_index(f.struct)


SPAN_NP = np.dtype([("offset", "<u8"), ("length", "<u4"), ("reserved", "<u4")])


def _esize(t):
    return 16 if t == T_STRING else SCALAR[t]


def pack(schema, values, n):
    """Columnar values -> (records u8 array, string arena, list arena)."""
    rec = np.zeros(n, dtype=schema.dtype())
    sarena, larena = [], []
    pos = {"s": 0, "l": 0}

    def strings(lens, data):
        """Spans of consecutive strings appended to the string arena."""
        lens = np.asarray(lens, dtype=np.uint64)
        starts = pos["s"] + np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        sarena.append(np.asarray(data, dtype=np.uint8))
        pos["s"] += int(lens.sum())
        return np.where(lens > 0, starts, 0), lens

    def column(key, t, total):
        """(total, element size) bytes of one element column."""
        if t == T_STRING:
            off, lens = strings(values[key + ".len"], values[key + ".data"])
            sp = np.zeros(total, SPAN_NP)
            sp["offset"], sp["length"] = off, lens
            return sp.view(np.uint8).reshape(total, 16)
        return np.ascontiguousarray(values[key]).view(np.uint8).reshape(total, SCALAR[t])

    for path, f in _paths(schema):
        key = _key(path)
        arr, f, si, k = _view(rec, schema, path)
        arr["__isset"][:, k] = values[key + ".set"]
        if f.ttype in SCALAR:
            v = values[key + ".val"]
            if v.dtype in (np.uint64,):
                arr[f.name] = v.view(np.float64)
            elif v.dtype == np.uint32 and f.ttype == 19:
                arr[f.name] = v.view(np.float32)
            else:
                arr[f.name] = v
        elif f.ttype == T_STRING:
            off, lens = strings(values[key + ".len"], values[key + ".data"])
            arr[f.name]["offset"], arr[f.name]["length"] = off, lens
        elif f.ttype in (T_LIST, T_SET, T_MAP):
            cnt = values[key + ".count"].astype(np.uint64)
            tot = int(cnt.sum())
            if f.ttype == T_MAP:
                # packed {key, value} pairs (the tgpu_span map form)
                el = np.concatenate([column(key + ".keys", f.elem_ttype, tot),
                                     column(key + ".vals", f.val_ttype, tot)], axis=1)
                es = _esize(f.elem_ttype) + _esize(f.val_ttype)
            else:
                el = column(key + ".elems", f.elem_ttype, tot)
                es = _esize(f.elem_ttype)
            starts = pos["l"] + es * np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint64)
            arr[f.name]["offset"] = np.where(cnt > 0, starts, 0)
            arr[f.name]["length"] = cnt
            larena.append(el.reshape(-1))
            pos["l"] += tot * es
    s = np.concatenate(sarena) if sarena else np.zeros(0, np.uint8)
    l = np.concatenate(larena) if larena else np.zeros(0, np.uint8)
    return rec.view(np.uint8).reshape(-1), s, l


def unpack(schema, rec_bytes, n, wire, arena):
    """Record bytes (+ the stream for string views and the list arena) ->
    columnar values in the golden format."""
    rec = np.frombuffer(np.ascontiguousarray(rec_bytes)[: n * schema.record_size].tobytes(),
                        dtype=schema.dtype())
    w = np.frombuffer(bytes(wire), dtype=np.uint8)
    ar = np.ascontiguousarray(arena).view(np.uint8).reshape(-1)
    out = {}

    def strings(key, offs, lens):
        out[key + ".len"] = np.asarray(lens, dtype=np.uint32)
        parts = [w[o:o + l] for o, l in zip(np.asarray(offs).tolist(), np.asarray(lens).tolist())]
        out[key + ".data"] = np.concatenate(parts) if parts else np.zeros(0, np.uint8)

    def column(key, t, b):
        """b: (total, element size) bytes of one element column."""
        if t == T_STRING:
            sp = np.ascontiguousarray(b).reshape(-1).view(SPAN_NP)
            strings(key, sp["offset"], sp["length"])
        else:
            out[key] = np.ascontiguousarray(b).reshape(-1).view(ELEM_NP[t])

    for path, f in _paths(schema):
        key = _key(path)
        arr, f, si, k = _view(rec, schema, path)
        out[key + ".set"] = arr["__isset"][:, k].copy()
        if f.ttype in SCALAR:
            v = arr[f.name]
            if v.dtype == np.float64:
                v = v.view(np.uint64)
            elif v.dtype == np.float32:
                v = v.view(np.uint32)
            out[key + ".val"] = v.copy()
        elif f.ttype == T_STRING:
            sp = arr[f.name]
            strings(key, sp["offset"], sp["length"])
        elif f.ttype in (T_LIST, T_SET, T_MAP):
            sp = arr[f.name]
            ks = _esize(f.elem_ttype)
            es = ks + (_esize(f.val_ttype) if f.ttype == T_MAP else 0)
            out[key + ".count"] = sp["length"].astype(np.uint32)
            parts = [ar[o:o + l * es] for o, l in zip(sp["offset"].tolist(), sp["length"].tolist())]
            el = (np.concatenate(parts) if parts else np.zeros(0, np.uint8)).reshape(-1, es)
            if f.ttype == T_MAP:
                column(key + ".keys", f.elem_ttype, el[:, :ks])
                column(key + ".vals", f.val_ttype, el[:, ks:])
            else:
                column(key + ".elems", f.elem_ttype, el)
    return out


def assert_values_equal(got, want):
    assert set(got) == set(want), (sorted(set(got) ^ set(want)))
    for k in sorted(want):
        g, w = np.asarray(got[k]), np.asarray(want[k])
        assert g.shape == w.shape, (k, g.shape, w.shape)
        assert np.array_equal(g.view(np.uint8) if g.dtype.kind == "f" else g,
                              w.view(np.uint8) if w.dtype.kind == "f" else w), k


def assert_arena_equal(schema, rec_bytes, n, wire, got_arena, want_arena):
    """The list arena bytes the records' spans reference are equal (bytes of
    the arena outside the spans are unspecified)."""
    assert_values_equal(unpack(schema, rec_bytes, n, wire, got_arena),
                        unpack(schema, rec_bytes, n, wire, want_arena))
