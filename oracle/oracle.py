"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/build/liboracle_thrift.so.

The CPU restatement of the reference protocols (oracle/thrift_oracle.cpp).
Used only by tests/ (as the parity checker), __graft_entry__.smoke() and the
cpu_baseline leg of bench.py. Never imported by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle_thrift.so")


class Status(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("exc_class", ctypes.c_int32),
                ("tproto_type", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("record", ctypes.c_uint64), ("byte_offset", ctypes.c_uint64)]

    def as_tuple(self):
        return (self.code, self.exc_class, self.tproto_type, self.record, self.byte_offset)


class Limits(ctypes.Structure):
    _fields_ = [("string_limit", ctypes.c_int32), ("container_limit", ctypes.c_int32),
                ("max_depth", ctypes.c_int32), ("height", ctypes.c_int32)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, U32, U64, I32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.oracle_encode_batch.restype = I32
        L.oracle_encode_batch.argtypes = [P, U32, P, U32, I32, P, U64, P, P, P, U64, P,
                                          ctypes.POINTER(Status), ctypes.POINTER(U64)]
        L.oracle_decode_batch.restype = I32
        L.oracle_decode_batch.argtypes = [P, U32, P, U32, I32, P, U64, P, U64, P, P, U64,
                                          ctypes.POINTER(Limits), ctypes.POINTER(Status),
                                          ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.oracle_encode_batch_ex.restype = I32
        L.oracle_encode_batch_ex.argtypes = [P, U32, P, U32, P, U32, I32, P, U64, P, P, P, U64, P,
                                             ctypes.POINTER(Status), ctypes.POINTER(U64)]
        L.oracle_decode_batch_ex.restype = I32
        L.oracle_decode_batch_ex.argtypes = [P, U32, P, U32, P, U32, I32, P, U64, P, U64, P, P,
                                             U64, ctypes.POINTER(Limits), ctypes.POINTER(Status),
                                             ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.oracle_arena_scale.restype = U32
        L.oracle_arena_scale.argtypes = [P, U32, P, U32, P, U32, I32]
        L.oracle_record_length.restype = ctypes.c_int64
        L.oracle_record_length.argtypes = [I32, P, U64, U64, ctypes.c_int32, ctypes.c_int32]
        L.oracle_read_varint.restype = I32
        L.oracle_read_varint.argtypes = [P, U64, I32, ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.oracle_write_varint.restype = I32
        L.oracle_write_varint.argtypes = [U64, P]
        for name in ("oracle_flat8_binary_decode",):
            getattr(L, name).restype = I32
            getattr(L, name).argtypes = [P, U64, P, I32]
        L.oracle_flat8_binary_encode.restype = I32
        L.oracle_flat8_binary_encode.argtypes = [P, U64, P, I32]
        L.oracle_mixed_compact_decode.restype = I32
        L.oracle_mixed_compact_decode.argtypes = [P, P, U64, P, I32]
        L.oracle_mixed_compact_encode.restype = I32
        L.oracle_mixed_compact_encode.argtypes = [P, U64, P, P, P, I32]
        L.oracle_mixed_compact_size.restype = I32
        L.oracle_mixed_compact_size.argtypes = [P, U64, P, I32]
        L.oracle_mixed_compact_read_file.restype = U64
        L.oracle_mixed_compact_read_file.argtypes = [P, U64, U64, P, P]
        L.oracle_nested_binary_size.restype = I32
        L.oracle_nested_binary_size.argtypes = [P, U64, P, I32]
        L.oracle_nested_binary_encode.restype = I32
        L.oracle_nested_binary_encode.argtypes = [P, U64, P, P, P, I32]
        L.oracle_nested_binary_decode.restype = I32
        L.oracle_nested_binary_decode.argtypes = [P, P, U64, P, P, I32]
        L.oracle_splitmix64_at.restype = U64
        L.oracle_splitmix64_at.argtypes = [U64, U64]
        L.oracle_gen_flat8.argtypes = [U64, U64, U64, P]
        _L = L
    return _L


def _p(a):
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def _u8(b):
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(b), dtype=np.uint8)


def encode(schema, protocol, records, n, string_base=None, list_base=None, cap=None):
    """Returns (status, wire bytes, offsets[n+1])."""
    structs, ns, fields, nf = schema.descriptors()
    types, nt = schema.type_descriptors()
    rec = _u8(records)
    sb = _u8(string_base) if string_base is not None else np.zeros(1, np.uint8)
    lb = _u8(list_base) if list_base is not None else np.zeros(1, np.uint8)
    if cap is None:
        # first pass: size only
        offs = np.zeros(n + 1, np.uint64)
        st, size = Status(), ctypes.c_uint64()
        lib().oracle_encode_batch_ex(ctypes.addressof(structs), ns, ctypes.addressof(fields), nf,
                                     ctypes.addressof(types), nt, protocol, _p(rec), n, _p(sb),
                                     _p(lb), None, 0, _p(offs), ctypes.byref(st),
                                     ctypes.byref(size))
        if st.code:
            return st, b"", offs
        cap = size.value
    out = np.zeros(max(cap, 1), np.uint8)
    offs = np.zeros(n + 1, np.uint64)
    st, size = Status(), ctypes.c_uint64()
    lib().oracle_encode_batch_ex(ctypes.addressof(structs), ns, ctypes.addressof(fields), nf,
                                 ctypes.addressof(types), nt, protocol, _p(rec), n, _p(sb),
                                 _p(lb), _p(out), cap, _p(offs), ctypes.byref(st),
                                 ctypes.byref(size))
    return st, out[: size.value].tobytes(), offs


def decode(schema, protocol, wire, n, offsets=None, limits=None, arena_cap=None):
    """Returns (status, records ndarray[u8], arena ndarray[u8], n_decoded, consumed)."""
    structs, ns, fields, nf = schema.descriptors()
    types, nt = schema.type_descriptors()
    w = _u8(wire)
    rec = np.zeros(max(n * schema.record_size, 1), np.uint8)
    if arena_cap is None:
        arena_cap = w.size * arena_scale(schema, protocol)
    arena = np.zeros(max(arena_cap, 1), np.uint8)
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lim = Limits(*limits) if limits is not None else None
    st, nd, cons = Status(), ctypes.c_uint64(), ctypes.c_uint64()
    lib().oracle_decode_batch_ex(ctypes.addressof(structs), ns, ctypes.addressof(fields), nf,
                                 ctypes.addressof(types), nt,
                                 protocol, _p(w), w.size, _p(offs), n, _p(rec), _p(arena),
                              arena_cap, ctypes.byref(lim) if lim else None, ctypes.byref(st),
                              ctypes.byref(nd), ctypes.byref(cons))
    return st, rec, arena, nd.value, cons.value


def arena_scale(schema, protocol):
    """List arena bytes per input byte (tgpu_schema_arena_scale restated)."""
    structs, ns, fields, nf = schema.descriptors()
    types, nt = schema.type_descriptors()
    return lib().oracle_arena_scale(ctypes.addressof(structs), ns, ctypes.addressof(fields), nf,
                                    ctypes.addressof(types), nt, protocol)


def record_length(protocol, buf, pos=0, max_depth=12000, height=0):
    b = _u8(buf)
    return lib().oracle_record_length(protocol, _p(b), b.size, pos, max_depth, height)


def skip_value(protocol, buf, ttype, pos=0, max_depth=12000, height=0):
    b = _u8(buf)
    L = lib()
    L.oracle_skip_value.restype = ctypes.c_int64
    L.oracle_skip_value.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                    ctypes.c_uint64, ctypes.c_int, ctypes.c_int32, ctypes.c_int32]
    return L.oracle_skip_value(protocol, _p(b), b.size, pos, ttype, max_depth, height)


def read_varint(buf, bits):
    b = _u8(buf)
    v, c = ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib().oracle_read_varint(_p(b), b.size, bits, ctypes.byref(v), ctypes.byref(c))
    return rc, v.value, c.value


def write_varint(value):
    out = np.zeros(16, np.uint8)
    n = lib().oracle_write_varint(value, _p(out))
    return out[:n].tobytes()


SKIM_DTYPE = np.dtype([("id", "<i2"), ("ttype", "u1"), ("flags", "u1"), ("length", "<u4"),
                       ("offset", "<u8")])


def skim(protocol, wire, offsets, n=None, max_fields=16, limits=None, nest=0):
    """Schemaless skim (oracle_skim_batch_ex; nest = struct levels descended
    into): returns (status, fields (n, max_fields) SKIM_DTYPE records, counts
    uint32[n], n_done)."""
    w = _u8(wire)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offs.size - 1 if n is None else n
    fields = np.zeros((max(max_fields, 1), max(n, 1)), SKIM_DTYPE)  # field-major
    counts = np.zeros(max(n, 1), np.uint32)
    L = lib()
    L.oracle_skim_batch_ex.restype = ctypes.c_int
    L.oracle_skim_batch_ex.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lim = Limits(*limits) if limits is not None else None
    st, done = Status(), ctypes.c_uint64()
    L.oracle_skim_batch_ex(protocol, _p(w), w.size, _p(offs), n, fields.ctypes.data, max_fields,
                           counts.ctypes.data, nest, ctypes.byref(lim) if lim else None,
                           ctypes.byref(st), ctypes.byref(done))
    return st, fields[:max_fields, :n].T, counts[:n], done.value
