"""Nested-container schemas and deterministic records: lists/sets of structs,
containers of containers, maps with struct or container values (the
TableBased TypeInfo nesting, thrift/lib/cpp2/protocol/TableBasedForwardTypes.h:
37-93). Shared by tests/golden/make_golden.py (which writes them with the
reference's own Python protocols) and the parity tests (which decode them
back to the same nested values).

Values: a struct is a list of field values in declaration order (None: an
optional field not set); a list/set is a list; a map is a list of [key, value]
pairs in wire order; strings are bytes; doubles are Python floats built from
bit patterns. Pure Python; no reference code.
"""
from datagen import (SEED, T_BOOL, T_BYTE, T_DOUBLE, T_FLOAT, T_I16, T_I32, T_I64, T_LIST,
                     T_MAP, T_SET, T_STRING, T_STRUCT, bits_to_double, finite_bits, s32, s64,
                     splitmix64_at)

# Field rows: [id, ttype, elem_ttype, qualifier, struct_index, val_ttype, inner,
# key] where inner = [ttype, elem_ttype, val_ttype, struct_index, inner, key]
# describes container elements / map values that are themselves containers
# and key a map's struct key ([T_STRUCT, 0, 0, struct_index]) or container
# key (an inner form). Qualifier 4 / 5: a boxed (cpp.ref / thrift.box)
# struct field, unqualified / optional.
ITEM = [[1, T_I32, 0, 0, -1], [2, T_STRING, 0, 0, -1], [3, T_LIST, T_I16, 0, -1],
        [4, T_DOUBLE, 0, 1, -1]]
POINT = [[1, T_I32, 0, 0, -1], [2, T_I32, 0, 0, -1], [3, T_STRING, 0, 1, -1]]
NESTED_SCHEMAS = {
    # struct 1 = Item {1: i32, 2: string, 3: list<i16>, 4: optional double}
    "structlist": [
        [[1, T_I64, 0, 0, -1], [2, T_LIST, T_STRUCT, 0, 1], [3, T_SET, T_STRUCT, 0, 1],
         [4, T_MAP, T_I32, 0, 1, T_STRUCT], [5, T_STRING, 0, 0, -1]],
        ITEM,
    ],
    "deepcont": [
        [[1, T_LIST, T_LIST, 0, -1, 0, [T_LIST, T_I32, 0, -1]],
         [2, T_MAP, T_STRING, 0, -1, T_LIST, [T_LIST, T_STRING, 0, -1]],
         [3, T_LIST, T_MAP, 0, -1, 0, [T_MAP, T_I32, T_STRING, -1]],
         [4, T_MAP, T_I32, 0, 1, T_MAP, [T_MAP, T_I32, T_STRUCT, 1]],
         [5, T_SET, T_LIST, 0, -1, 0, [T_LIST, T_LIST, 0, -1, [T_LIST, T_I64, 0, -1]]],
         [6, T_I32, 0, 0, -1]],
        ITEM,
    ],
    # struct 1 = Point {1: i32 x, 2: i32 y, 3: optional string label}
    "keyed": [
        [[1, T_MAP, T_STRUCT, 0, -1, T_STRING, None, [T_STRUCT, 0, 0, 1]],
         [2, T_MAP, T_LIST, 0, -1, T_I64, None, [T_LIST, T_I32, 0, -1]],
         [3, T_MAP, T_SET, 0, 1, T_STRUCT, None, [T_SET, T_STRING, 0, -1]],
         [4, T_LIST, T_MAP, 0, -1, 0,
          [T_MAP, T_STRUCT, T_LIST, -1, [T_LIST, T_I16, 0, -1], [T_STRUCT, 0, 0, 1]]],
         [5, T_I32, 0, 0, -1]],
        POINT,
    ],
    # Tree {1: i32 v, 2: list<Tree> kids, 3: string tag}: recursive through a
    # list, up to 12 levels (past the device's private frames)
    "tree": [
        [[1, T_I32, 0, 0, -1], [2, T_LIST, T_STRUCT, 0, 0], [3, T_STRING, 0, 0, -1]],
    ],
    # Node {1: i64 v, 2: optional Node next (thrift.box), 3: Leaf leaf
    # (cpp.ref)}, Leaf {1: i32 a, 2: optional string b}: a linked list of
    # 0..60 boxed nodes
    "chain": [
        [[1, T_I64, 0, 0, -1], [2, T_STRUCT, 0, 5, 0], [3, T_STRUCT, 0, 4, 1]],
        [[1, T_I32, 0, 0, -1], [2, T_STRING, 0, 1, -1]],
    ],
}


class _R:
    """splitmix64 stream for record i of a case."""

    def __init__(self, i, salt):
        self.i, self.k, self.salt = i, 0, salt

    def u(self):
        self.k += 1
        return splitmix64_at(SEED ^ self.salt, self.i * 4096 + self.k)

    def below(self, n):
        return self.u() % n if n else 0


def _count(r, i):
    # mostly short, sometimes empty, sometimes past Compact's 14-element
    # short form
    c = r.below(8)
    if i % 17 == 3:
        c = 15 + r.below(6)
    if i % 13 == 5:
        c = 0
    return c


def _str(r, maxlen=12):
    n = r.below(maxlen + 1)
    return bytes(r.below(256) for _ in range(n))


def item(r, i):
    tags = [(r.u() & 0xFFFF) - 0x8000 for _ in range(_count(r, i))]
    return [s32(r.u()), _str(r), tags,
            bits_to_double(finite_bits(r.u())) if r.below(3) else None]


def gen_structlist(i):
    r = _R(i, 0x51)
    items = [item(r, i) for _ in range(_count(r, i))]
    uniq = [item(r, i) for _ in range(r.below(4))]
    by_id = [[s32(r.u()), item(r, i)] for _ in range(r.below(5))]
    return [s64(r.u()), items, uniq, by_id, _str(r, 20)]


def gen_deepcont(i):
    r = _R(i, 0xDC)
    grid = [[s32(r.u()) for _ in range(_count(r, i + 1))] for _ in range(_count(r, i))]
    index = [[_str(r, 6), [_str(r, 5) for _ in range(r.below(4))]] for _ in range(r.below(4))]
    maps = [[[s32(r.u()), _str(r, 4)] for _ in range(r.below(3))] for _ in range(r.below(4))]
    mm = [[s32(r.u()), [[s32(r.u()), item(r, i)] for _ in range(r.below(3))]]
          for _ in range(r.below(3))]
    cube = [[[s64(r.u()) for _ in range(r.below(3))] for _ in range(r.below(3))]
            for _ in range(r.below(3))]
    return [grid, index, maps, mm, cube, s32(r.u())]


def point(r):
    return [s32(r.u()) % 1000, s32(r.u()) % 1000, _str(r, 6) if r.below(2) else None]


def gen_keyed(i):
    r = _R(i, 0x4E)
    by_point = [[point(r), _str(r, 8)] for _ in range(r.below(5))]
    by_path = [[[s32(r.u()) for _ in range(r.below(4))], s64(r.u())] for _ in range(r.below(4))]
    by_tags = [[[_str(r, 4) for _ in range(r.below(3))], point(r)] for _ in range(r.below(3))]
    grids = [[[point(r), [(r.u() & 0xFFFF) - 0x8000 for _ in range(r.below(4))]]
              for _ in range(r.below(3))] for _ in range(r.below(3))]
    return [by_point, by_path, by_tags, grids, s32(r.u())]


def _tree(r, depth):
    # a spine `depth` levels deep, with a few shallow side branches
    kids = []
    if depth > 0:
        kids = [_tree(r, depth - 1)] + [_tree(r, min(1, depth - 1)) for _ in range(r.below(2))]
        if r.below(3) == 0:
            kids.reverse()
    return [s32(r.u()), kids, _str(r, 5)]


def gen_tree(i):
    r = _R(i, 0x7E)
    return _tree(r, r.below(13) if i % 5 else 12)


def gen_chain(i):
    r = _R(i, 0xC4)
    n = r.below(61) if i % 4 == 0 else r.below(10)
    node = None
    for k in range(n + 1):
        leaf = [s32(r.u()), _str(r, 6) if r.below(2) else None]
        node = [s64(r.u()), node, leaf]
    return node


NESTED_GENERATORS = {"structlist": gen_structlist, "deepcont": gen_deepcont,
                     "keyed": gen_keyed, "tree": gen_tree, "chain": gen_chain}


# ---- type specs ------------------------------------------------------------
# A spec is (ttype, sub): sub = struct index for T_STRUCT (a boxed field:
# (T_STRUCT, sub, True)); for containers (ttype, elem_spec, val_spec) with
# val_spec None for list/set and elem_spec the key's spec for a map.
def _inner_spec(inner):
    tt, et, vt, sub = inner[:4]
    nxt = inner[4] if len(inner) > 4 else None
    key = inner[5] if len(inner) > 5 else None
    return container_spec(tt, et, vt, sub, nxt, key)


def _key_spec(et, key):
    if key is None:
        return (et, None)
    if key[0] == T_STRUCT:
        return (T_STRUCT, key[3])
    return _inner_spec(key)


def _elem_spec(t, sub, inner):
    if t == T_STRUCT:
        return (T_STRUCT, sub)
    if t in (T_LIST, T_SET, T_MAP):
        return _inner_spec(inner)
    return (t, None)


def container_spec(tt, et, vt, sub, inner, key=None):
    if tt == T_MAP:
        return (tt, _key_spec(et, key), _elem_spec(vt, sub, inner))
    return (tt, _elem_spec(et, sub, inner), None)


def field_spec(row):
    fid, tt, et, q, sub = row[:5]
    if tt == T_STRUCT:
        return (T_STRUCT, sub, True) if q in (4, 5) else (T_STRUCT, sub)
    if tt in (T_LIST, T_SET, T_MAP):
        return container_spec(tt, et, row[5] if len(row) > 5 else 0, sub,
                              row[6] if len(row) > 6 else None,
                              row[7] if len(row) > 7 else None)
    return (tt, None)


# ---- JSON form of the values (golden fixtures are data) ----------------------
def to_json(spec, v, table):
    t = spec[0]
    if v is None:
        return None
    if t == T_STRING:
        return v.hex()
    if t == T_DOUBLE:
        import struct
        return struct.unpack("<Q", struct.pack("<d", v))[0]
    if t == T_STRUCT:
        rows = table[spec[1]]
        return [to_json(field_spec(row), x, table) for row, x in zip(rows, v)]
    if t == T_MAP:
        return [[to_json(spec[1], a, table), to_json(spec[2], b, table)] for a, b in v]
    if t in (T_LIST, T_SET):
        return [to_json(spec[1], e, table) for e in v]
    return int(v)
