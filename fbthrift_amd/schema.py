"""Schema descriptors: the runtime-table form of a Thrift struct.

Mirrors the reference's table-based serializer metadata (StructInfo /
FieldInfo / TypeInfo, thrift/lib/cpp2/protocol/TableBasedSerializer.h:90-118,
205-302) and the layout of codegen'd structs (members in IDL declaration
order, thrift/compiler/generate/t_whisker_generator.cc:231-236, then one isset
byte per field, thrift/lib/cpp2/detail/Isset.h:243-296). Strings and lists use
16-byte spans (tgpu_span) in the device layout.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import (T_BOOL, T_BYTE, T_DOUBLE, T_FLOAT, T_I16, T_I32, T_I64, T_LIST,
                   T_MAP, T_SET, T_STRING, T_STRUCT)

SCALAR = {T_BOOL: 1, T_BYTE: 1, T_I16: 2, T_I32: 4, T_FLOAT: 4, T_I64: 8, T_DOUBLE: 8}
NP_SCALAR = {T_BOOL: np.uint8, T_BYTE: np.int8, T_I16: np.int16, T_I32: np.int32,
             T_I64: np.int64, T_DOUBLE: np.float64, T_FLOAT: np.float32}
SPAN = np.dtype([("offset", "<u8"), ("length", "<u4"), ("reserved", "<u4")])

OPTIONAL = 1
TERSE = 2  # @thrift.TerseWrite: written only when not empty (op::isEmpty)
REQUIRED = 3  # `required`: always written; enforced on read with Struct(enforce_required)
# cpp.ref / @thrift.Box struct fields: the member is a pointer (a span into the
# list arena / list_base; length 1 = present). BOXED is always written (a
# null one as an empty struct), OPTIONAL_BOXED when its isset byte is set.
BOXED = 4
OPTIONAL_BOXED = 5


class Type:
    """A container type held by a container (a list/set element, a map value
    or a map key that is itself a list, set or map): tgpu_type_desc. `struct`
    is the struct of T_STRUCT elements / values, `inner` the Type of
    container elements / values, `key` the Type of a map's struct or
    container key (a struct key: Type(T_STRUCT, 0, struct=S))."""

    def __init__(self, ttype, elem_ttype=0, val_ttype=0, struct=None, inner=None, key=None):
        self.ttype, self.elem_ttype, self.val_ttype = int(ttype), int(elem_ttype), int(val_ttype)
        self.struct, self.inner, self.key = struct, inner, key


class Field:
    """One field. For T_STRUCT, `struct` is the nested struct; for a list/set
    of structs (elem_ttype T_STRUCT) or a map with struct values (val_ttype
    T_STRUCT), `struct` is that struct; `inner` is the Type of container
    elements / values."""

    def __init__(self, id, ttype, elem_ttype=0, optional=False, struct=None, name=None,
                 qualifier=None, val_ttype=0, inner=None, key=None):
        self.id, self.ttype, self.elem_ttype = int(id), int(ttype), int(elem_ttype)
        self.val_ttype = int(val_ttype)  # T_MAP: value type (elem_ttype = key type)
        self.qualifier = int(qualifier) if qualifier is not None else (OPTIONAL if optional else 0)
        self.optional, self.struct = self.qualifier == OPTIONAL, struct
        self.inner = inner
        self.key = key  # T_MAP with a struct / container key: its Type
        self.boxed = self.qualifier in (BOXED, OPTIONAL_BOXED)
        self.name = name or "f%d" % self.id


def element_struct(t):
    """The struct a container description (Field or Type) holds, if any."""
    v = t.val_ttype if t.ttype == T_MAP else t.elem_ttype
    return t.struct if v == T_STRUCT else None


class Struct:
    def __init__(self, name, fields, union=False, enforce_required=False):
        self.name, self.fields = name, list(fields)
        self.union = bool(union)  # TGPU_STRUCT_UNION
        # TGPU_STRUCT_ENFORCE_REQUIRED (deprecated_enforce_required codegen)
        self.enforce_required = bool(enforce_required)


class Schema:
    """A record type (struct 0) plus the structs it nests, with the layout
    computed by the same rule as tgpu_layout_compute()."""

    def __init__(self, root):
        self.root = root
        self.structs = []
        index = {}

        self.types, tindex = [], {}

        def visit_type(t):
            if id(t) in tindex:
                return
            tindex[id(t)] = len(self.types)
            self.types.append(t)
            if t.ttype == T_STRUCT:
                visit(t.struct)
            else:
                visit_container(t)

        def visit_container(t):
            es = element_struct(t)
            if es is not None:
                visit(es)
            if getattr(t, "key", None) is not None:
                visit_type(t.key)
            if t.inner is not None:
                visit_type(t.inner)

        def visit(s):
            if id(s) in index:
                return index[id(s)]
            index[id(s)] = len(self.structs)
            self.structs.append(s)
            for f in s.fields:
                if f.ttype == T_STRUCT:
                    visit(f.struct)
                elif f.ttype in (T_LIST, T_SET, T_MAP):
                    visit_container(f)
            return index[id(s)]

        visit(root)
        self._index = index
        self._tindex = tindex
        self._layout()

    # -- layout -------------------------------------------------------------
    def _layout(self):
        self.size, self.align, self.member, self.isset = {}, {}, {}, {}
        done = set()

        def lay(si):
            if si in done:
                return
            s = self.structs[si]
            off, al_max = 0, 1
            for k, f in enumerate(s.fields):
                if f.ttype in SCALAR:
                    sz = al = SCALAR[f.ttype]
                elif f.ttype in (T_STRING, T_LIST, T_SET, T_MAP) or f.boxed:
                    sz, al = 16, 8
                elif f.ttype == T_STRUCT:
                    sub = self._index[id(f.struct)]
                    lay(sub)
                    sz, al = self.size[sub], self.align[sub]
                else:
                    raise ValueError("unsupported field type %d" % f.ttype)
                off = (off + al - 1) // al * al
                self.member[(si, k)] = off
                off += sz
                al_max = max(al_max, al)
            for k in range(len(s.fields)):
                self.isset[(si, k)] = off + k
            off += len(s.fields)
            self.align[si] = al_max
            self.size[si] = (max(off, 1) + al_max - 1) // al_max * al_max
            done.add(si)

        for si in range(len(self.structs)):
            lay(si)
        self.record_size = self.size[0]

    # -- C descriptors --------------------------------------------------------
    def descriptors(self):
        structs = (_lib.StructDesc * len(self.structs))()
        nf = sum(len(s.fields) for s in self.structs)
        fields = (_lib.FieldDesc * max(nf, 1))()
        j = 0
        for si, s in enumerate(self.structs):
            structs[si].first_field = j
            structs[si].num_fields = len(s.fields)
            structs[si].size = self.size[si]
            structs[si].align = self.align[si]
            structs[si].flags = (1 if s.union else 0) | (2 if s.enforce_required else 0)
            for k, f in enumerate(s.fields):
                fd = fields[j]
                fd.id, fd.ttype, fd.elem_ttype = f.id, f.ttype, f.elem_ttype
                fd.qualifier = f.qualifier
                fd.val_ttype = f.val_ttype
                fd.member_offset = self.member[(si, k)]
                fd.isset_offset = self.isset[(si, k)]
                fd.struct_index = self._struct_ref(f)
                fd.type_index = self._type_ref(f)
                fd.key_index = self._key_ref(f)
                j += 1
        return structs, len(self.structs), fields, nf

    def _struct_ref(self, t):
        if t.ttype == T_STRUCT or element_struct(t) is not None:
            return self._index[id(t.struct)]
        return -1

    def _type_ref(self, t):
        return 1 + self._tindex[id(t.inner)] if getattr(t, "inner", None) is not None else 0

    def _key_ref(self, t):
        return 1 + self._tindex[id(t.key)] if getattr(t, "key", None) is not None else 0

    def type_descriptors(self):
        """The nested container types (tgpu_type_desc[]) for
        tgpu_schema_create_ex: (array, count)."""
        types = (_lib.TypeDesc * max(len(self.types), 1))()
        for k, t in enumerate(self.types):
            types[k].ttype, types[k].elem_ttype, types[k].val_ttype = t.ttype, t.elem_ttype, t.val_ttype
            types[k].struct_index = (self._index[id(t.struct)] if t.ttype == T_STRUCT
                                     else self._struct_ref(t))
            types[k].type_index = self._type_ref(t)
            types[k].key_index = self._key_ref(t)
        return types, len(self.types)

    @property
    def nested(self):
        """Some container holds structs or containers (as elements, values
        or keys), or a field is boxed (arena record regions)."""
        cx = (T_STRUCT, T_LIST, T_SET, T_MAP)

        def complex_(t):
            v = t.val_ttype if t.ttype == T_MAP else t.elem_ttype
            return v in cx or (t.ttype == T_MAP and t.elem_ttype in cx)
        return any((f.ttype in (T_LIST, T_SET, T_MAP) and complex_(f)) or f.boxed
                   for s in self.structs for f in s.fields)

    # -- numpy view of the record layout -------------------------------------
    def dtype(self, si=0):
        s = self.structs[si]
        names, formats, offsets = [], [], []
        for k, f in enumerate(s.fields):
            names.append(f.name)
            if f.ttype in SCALAR:
                formats.append(NP_SCALAR[f.ttype])
            elif f.ttype in (T_STRING, T_LIST, T_SET, T_MAP) or f.boxed:
                formats.append(SPAN)
            else:
                formats.append(self.dtype(self._index[id(f.struct)]))
            offsets.append(self.member[(si, k)])
        if s.fields:
            names.append("__isset")
            formats.append((np.uint8, (len(s.fields),)))
            offsets.append(self.isset[(si, 0)])
        return np.dtype({"names": names, "formats": formats, "offsets": offsets,
                         "itemsize": self.size[si]})

    def struct_index(self, s):
        return self._index[id(s)]

    @classmethod
    def from_table(cls, table):
        """Builds a Schema from the tests/golden manifest form: a list of
        structs, each a list of [id, ttype, elem_ttype, qualifier, struct_index]
        (+ val_ttype for a map, + the nested container type of the elements /
        values as [ttype, elem_ttype, val_ttype, struct_index, nested, key],
        + a map's struct / container key type in that form, a struct key as
        [T_STRUCT, 0, 0, struct_index]); a union is {"union": true,
        "fields": [...]}. struct_index names the struct of a T_STRUCT field
        or of T_STRUCT elements / values. Structs may refer to each other
        recursively (through containers or BOXED / OPTIONAL_BOXED fields)."""
        structs = [Struct("S%d" % i, [], union=isinstance(e, dict) and e.get("union"),
                          enforce_required=isinstance(e, dict) and e.get("enforce_required"))
                   for i, e in enumerate(table)]

        def typ(spec):
            if not spec:
                return None
            tt, et, vt, sub = spec[:4]
            return Type(tt, et, vt, struct=structs[sub] if sub is not None and sub >= 0 else None,
                        inner=typ(spec[4] if len(spec) > 4 else None),
                        key=typ(spec[5] if len(spec) > 5 else None))

        for si, e in enumerate(table):
            for row in (e["fields"] if isinstance(e, dict) else e):
                fid, tt, et, q, sub = row[:5]
                structs[si].fields.append(
                    Field(fid, tt, et, qualifier=q,
                          struct=structs[sub] if sub is not None and sub >= 0 else None,
                          val_ttype=row[5] if len(row) > 5 else 0,
                          inner=typ(row[6] if len(row) > 6 else None),
                          key=typ(row[7] if len(row) > 7 else None)))
        return cls(structs[0])


def layout_compute_c(schema):
    """Runs tgpu_layout_compute on the schema's descriptors (host-only) and
    returns (structs, fields) as lists of tuples for comparison."""
    structs, ns, fields, nf = schema.descriptors()
    for i in range(nf):
        fields[i].member_offset = 0
        fields[i].isset_offset = 0
    rc = _lib.lib().tgpu_layout_compute(ctypes.addressof(structs), ns, ctypes.addressof(fields), nf)
    if rc:
        raise RuntimeError("tgpu_layout_compute failed: %s" % _lib.CODES.get(rc, rc))
    return ([(s.first_field, s.num_fields, s.size, s.align) for s in structs],
            [(f.member_offset, f.isset_offset) for f in fields[:nf]])
