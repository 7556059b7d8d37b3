"""The C-ABI library loads on a GPU-less host and exports every symbol
include/thrift_gpu.h declares; host-only entry points agree with the Python
host mirror (no device calls here)."""
import ctypes
import os
import re

import pytest

import helpers
from fbthrift_amd import _lib
from fbthrift_amd.schema import Schema, layout_compute_c

HEADER = os.path.join(helpers.ROOT, "include", "thrift_gpu.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(tgpu_\w+)\(", src, re.M)))


def test_header_symbols_listed():
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    L = _lib.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    assert L.tgpu_abi_version() == 1


@pytest.mark.parametrize("name", sorted(helpers.manifest()["schemas"]))
def test_layout_compute_matches_python(name):
    schema = Schema.from_table(helpers.manifest()["schemas"][name])
    structs, fields = layout_compute_c(schema)
    st, ns, fl, nf = schema.descriptors()
    assert structs == [(s.first_field, s.num_fields, s.size, s.align) for s in st]
    assert fields == [(f.member_offset, f.isset_offset) for f in fl[:nf]]


def test_config_layouts():
    m = helpers.manifest()["schemas"]
    assert Schema.from_table(m["flat8"]).record_size == 72
    assert Schema.from_table(m["mixed"]).record_size == 56
    nested = Schema.from_table(m["nested"])
    assert nested.record_size == 64 and nested.size[1] == 32


def test_code_classification():
    L = _lib.lib()
    e, t = ctypes.c_int32(), ctypes.c_int32()
    expect = {1: (1, 0), 2: (1, 0), 3: (2, 1), 4: (2, 1), 5: (2, 1), 6: (2, 2), 7: (2, 3),
              8: (2, 8), 9: (2, 0), 10: (3, 0), 11: (2, 3), 20: (4, 0), 0: (0, 0)}
    for code, want in expect.items():
        L.tgpu_code_classify(code, ctypes.byref(e), ctypes.byref(t))
        assert (e.value, t.value) == want, code
        assert L.tgpu_code_name(code).decode() == _lib.CODES[code]
