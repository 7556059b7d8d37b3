"""The oracle (CPU restatement) against the reference's own golden vectors.

Golden wire bytes come from fbthrift's pure-Python Binary/Compact protocols
(tests/golden/make_golden.py). This pins the oracle before it is trusted as
the GPU parity checker.
"""
import hashlib

import numpy as np
import pytest

import datagen
import helpers
from oracle import oracle


@pytest.mark.parametrize("name", helpers.case_names())
def test_oracle_decodes_golden(name):
    c = helpers.Case(name)
    for offs in (None, c.offsets):
        st, rec, arena, nd, consumed = oracle.decode(c.schema, c.protocol, c.wire, c.n, offsets=offs)
        assert st.code == 0, (name, st.as_tuple())
        assert nd == c.n and consumed == len(c.wire)
        got = helpers.unpack(c.schema, rec, c.n, c.wire, arena)
        helpers.assert_values_equal(got, c.values)


@pytest.mark.parametrize("name", helpers.case_names())
def test_oracle_encodes_golden(name):
    c = helpers.Case(name)
    rec, sarena, larena = helpers.pack(c.schema, c.values, c.n)
    st, wire, offs = oracle.encode(c.schema, c.protocol, rec, c.n, sarena, larena)
    assert st.code == 0, st.as_tuple()
    assert wire == c.wire
    assert np.array_equal(offs, c.offsets)


GEN = {"flat8": datagen.gen_flat8, "mixed": datagen.gen_mixed, "nested": datagen.gen_nested}


@pytest.mark.parametrize("name", sorted(helpers.manifest()["digests"]))
def test_oracle_matches_reference_digest(name):
    d = helpers.manifest()["digests"][name]
    table = helpers.manifest()["schemas"][d["schema"]]
    schema = helpers.Schema.from_table(table)
    recs = [GEN[d["schema"]](i) for i in range(d["n"])]
    vals = datagen.flatten_values(table, recs)
    rec, sarena, larena = helpers.pack(schema, vals, d["n"])
    st, wire, offs = oracle.encode(schema, helpers.PROTO[d["protocol"]], rec, d["n"], sarena, larena)
    assert st.code == 0
    assert hashlib.sha256(wire).hexdigest() == d["sha256"]
    assert hashlib.sha256(offs.tobytes()).hexdigest() == d["offsets_sha256"]


def test_generator_matches_c_generator():
    """oracle_gen_flat8 (C, used by the bench CPU baseline) == datagen.gen_flat8."""
    n = 3000
    buf = np.zeros(n * 72, np.uint8)
    oracle.lib().oracle_gen_flat8(datagen.SEED, 0, n, buf.ctypes.data)
    vals = buf.view(np.int64).reshape(n, 9)[:, :8]
    want = np.array([datagen.gen_flat8(i) for i in range(n)], dtype=np.int64)
    assert np.array_equal(vals, want)
    assert (buf.reshape(n, 72)[:, 64:] == 1).all()


def test_varint_vectors():
    """Every bit position (VarintUtilsTest.cpp:34-115), encoded by the
    reference Python writer: oracle writes the same bytes and reads back the
    value."""
    for bits, v, hexbytes in helpers.manifest()["varints"]:
        b = bytes.fromhex(hexbytes)
        assert oracle.write_varint(v) == b
        rc, got, used = oracle.read_varint(b, bits)
        assert rc == 0 and got == v and used == len(b)


def test_codegen_equivalent_paths_match_golden():
    """The codegen-equivalent CPU paths timed as per-config baselines
    (bench.py cpu_baseline) reproduce the golden streams and records: mixed
    Compact (config 3/5: size, encode, indexed decode, sequential file read)
    and nested Binary (config 4: size, encode, decode)."""
    L = oracle.lib()
    for name, size_fn, enc, dec in (
            ("mixed_compact", L.oracle_mixed_compact_size, None, None),
            ("nested_binary", L.oracle_nested_binary_size, None, None)):
        c = helpers.Case(name)
        rec, sarena, larena = helpers.pack(c.schema, c.values, c.n)
        sizes = np.zeros(c.n, np.uint64)
        size_fn(rec.ctypes.data, c.n, sizes.ctypes.data, 4)
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        assert np.array_equal(offs, c.offsets), name
        out = np.zeros(len(c.wire), np.uint8)
        back = np.zeros(c.n * c.schema.record_size, np.uint8)
        if name == "mixed_compact":
            L.oracle_mixed_compact_encode(rec.ctypes.data, c.n, sarena.ctypes.data,
                                          out.ctypes.data, offs.ctypes.data, 4)
            assert out.tobytes() == c.wire
            w = np.frombuffer(c.wire, np.uint8)
            assert L.oracle_mixed_compact_decode(w.ctypes.data, offs.ctypes.data, c.n,
                                                 back.ctypes.data, 4) == 0
            got = np.zeros(c.n + 1, np.uint64)
            back2 = np.zeros_like(back)
            assert L.oracle_mixed_compact_read_file(w.ctypes.data, w.size, c.n, back2.ctypes.data,
                                                    got.ctypes.data) == c.n
            assert np.array_equal(got, c.offsets) and np.array_equal(back2, back)
            arena = oarena = None
        else:
            L.oracle_nested_binary_encode(rec.ctypes.data, c.n, larena.ctypes.data,
                                          out.ctypes.data, offs.ctypes.data, 4)
            assert out.tobytes() == c.wire
            w = np.frombuffer(c.wire, np.uint8)
            arena = np.zeros(len(c.wire), np.uint8)
            assert L.oracle_nested_binary_decode(w.ctypes.data, offs.ctypes.data, c.n,
                                                 back.ctypes.data, arena.ctypes.data, 4) == 0
        ost, orec, oarena, _, _ = oracle.decode(c.schema, c.protocol, c.wire, c.n,
                                                offsets=c.offsets)
        assert np.array_equal(back, orec[: back.size]), name
        if arena is not None:
            helpers.assert_arena_equal(c.schema, orec, c.n, c.wire, arena, oarena)
