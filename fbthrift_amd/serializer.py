"""Python host mirror of fbthrift's Serializer<Reader, Writer> for whole
batches (thrift/lib/cpp2/protocol/Serializer.h:34-224), over the C-ABI.

    BinarySerializer.serialize(schema, records)   -> (wire, offsets)
    CompactSerializer.deserialize(schema, wire, n) -> (records, arena, consumed)

Device memory comes from torch (plumbing only); every byte of protocol work is
done by the gfx950 kernels in libtgpu.so. Errors are raised as the exception
the reference would throw: TProtocolException(type) or OutOfRange (the
std::out_of_range of folly cursors / invalid varints); a bool byte > 1 on write
raises AbortError where the reference calls LOG(FATAL) (Protocol.h:126-163).
"""
import ctypes

from . import _lib
from ._lib import PROTOCOL_BINARY, PROTOCOL_COMPACT, PROTOCOL_COMPACT_V1


class TProtocolException(Exception):
    """apache::thrift::protocol::TProtocolException (TProtocolException.h:41-51)."""

    UNKNOWN, INVALID_DATA, NEGATIVE_SIZE, SIZE_LIMIT = 0, 1, 2, 3
    BAD_VERSION, NOT_IMPLEMENTED, MISSING_REQUIRED_FIELD = 4, 5, 6
    CHECKSUM_MISMATCH, DEPTH_LIMIT = 7, 8

    def __init__(self, type_, message, status=None):
        super().__init__(message)
        self.type = type_
        self.status = status


class OutOfRange(IndexError):
    """std::out_of_range (folly cursor underflow, "invalid varint read")."""

    def __init__(self, message, status=None):
        super().__init__(message)
        self.status = status


class AbortError(RuntimeError):
    """Where the reference terminates the process (validate_bool)."""

    def __init__(self, message, status=None):
        super().__init__(message)
        self.status = status


class TgpuError(RuntimeError):
    def __init__(self, message, status=None):
        super().__init__(message)
        self.status = status


def raise_for_status(st):
    if st.code == 0:
        return
    name = _lib.CODES.get(st.code, str(st.code))
    msg = "%s at record %d, byte %d" % (name, st.record, st.byte_offset)
    if st.exc_class == 1:
        raise OutOfRange(msg, st)
    if st.exc_class == 2:
        raise TProtocolException(st.tproto_type, msg, st)
    if st.exc_class == 3:
        raise AbortError(msg, st)
    raise TgpuError(msg, st)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _hptr(a):
    """Address of a host buffer (numpy array or CPU tensor)."""
    return a.ctypes.data if hasattr(a, "ctypes") else a.data_ptr()


def _hlen(a):
    return a.nbytes if hasattr(a, "nbytes") else a.numel() * a.element_size()


def _stream(stream):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class GpuSchema:
    """A Schema uploaded to the current device (tgpu_schema_create)."""

    def __init__(self, schema):
        self.schema = schema
        structs, ns, fields, nf = schema.descriptors()
        types, nt = schema.type_descriptors()
        self._keep = (structs, fields, types)
        h = ctypes.c_void_p()
        rc = _lib.lib().tgpu_schema_create_ex(ctypes.addressof(structs), ns,
                                              ctypes.addressof(fields), nf,
                                              ctypes.addressof(types), nt, ctypes.byref(h))
        if rc:
            raise TgpuError("tgpu_schema_create: %s" % _lib.CODES.get(rc, rc))
        self.handle = h
        self.record_size = _lib.lib().tgpu_schema_record_size(h)
        # containers and boxed struct fields keep their contents in the arena
        self.has_lists = any(f.ttype in (_lib.T_LIST, _lib.T_SET, _lib.T_MAP) or f.boxed
                             for s in schema.structs for f in s.fields)

    def fixed_wire_size(self, protocol):
        return _lib.lib().tgpu_schema_fixed_wire_size(self.handle, protocol)

    def compile(self, protocol):
        """Compiles the schema's kernels for `protocol` now (tgpu_schema_compile);
        True when compiled kernels will be used, False when the schema has no
        canonical program or the compiler is unavailable (interpreted)."""
        return _lib.lib().tgpu_schema_compile(self.handle, protocol) == 0

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and _lib._lib is not None:
            _lib.lib().tgpu_schema_destroy(h)
            self.handle = None


def compile_check(schema, protocol, arch="gfx950"):
    """Generates and compiles `schema`'s kernels for `arch` without a GPU
    (tgpu_schema_compile_check_ex: the record program's decode / encode /
    index kernels, or a nested schema's nested decode). arch "": the program
    and kernel sources are generated only (whether the schema has a program,
    without the seconds of compiling). Returns (code, compiler log)."""
    structs, ns, fields, nf = schema.descriptors()
    types, nt = schema.type_descriptors()
    log = ctypes.create_string_buffer(1 << 16)
    rc = _lib.lib().tgpu_schema_compile_check_ex(ctypes.addressof(structs), ns,
                                                 ctypes.addressof(fields), nf,
                                                 ctypes.addressof(types), nt, protocol,
                                                 arch.encode(), log, len(log))
    return rc, log.value.decode(errors="replace")


def transcode_compile_check(schema, from_protocol, to_protocol, arch="gfx950"):
    """The wire-to-wire transcoder's kernels (source program's decode + target
    program's writer, tgpu_xcode.h) generated and compiled for `arch` without
    a GPU (tgpu_transcode_compile_check). Returns (code, compiler log)."""
    structs, ns, fields, nf = schema.descriptors()
    log = ctypes.create_string_buffer(1 << 16)
    rc = _lib.lib().tgpu_transcode_compile_check(ctypes.addressof(structs), ns,
                                                 ctypes.addressof(fields), nf, from_protocol,
                                                 to_protocol, arch.encode(), log, len(log))
    return rc, log.value.decode(errors="replace")


class Context:
    """Workspace + result slot (tgpu_context). One in-flight call at a time."""

    def __init__(self, reserve=0):
        h = ctypes.c_void_p()
        rc = _lib.lib().tgpu_context_create(ctypes.byref(h))
        if rc:
            raise TgpuError("tgpu_context_create: %s" % _lib.CODES.get(rc, rc))
        self.handle = h
        if reserve:
            self.reserve(reserve)

    def reserve(self, n):
        rc = _lib.lib().tgpu_context_reserve(self.handle, n)
        if rc:
            raise TgpuError("tgpu_context_reserve: %s" % _lib.CODES.get(rc, rc))

    def wait(self, stream=None):
        st = _lib.Status()
        n, b = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.lib().tgpu_context_wait(self.handle, _stream(stream), ctypes.byref(st),
                                     ctypes.byref(n), ctypes.byref(b))
        return st, n.value, b.value

    INDEX_STATS = ("chunks", "partial", "no_start", "broken", "repaired", "rewalked", "general")

    def index_stats(self, stream=None):
        """Repair counters of this context's last stream index
        (tgpu_index_stats): a dict over INDEX_STATS."""
        import numpy as np

        out = np.zeros(len(self.INDEX_STATS), np.uint64)
        rc = _lib.lib().tgpu_index_stats(self.handle, _stream(stream),
                                         ctypes.c_void_p(out.ctypes.data))
        if rc and rc != 23:  # (INVALID_ARGUMENT: no index yet; "general" is still filled)
            raise TgpuError("tgpu_index_stats: %d" % rc)
        return dict(zip(self.INDEX_STATS, (int(v) for v in out)))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and _lib._lib is not None:
            _lib.lib().tgpu_context_destroy(h)
            self.handle = None


class BatchSerializer:
    """Serializer<Reader, Writer> for batches of records of one schema."""

    def __init__(self, protocol):
        self.protocol = protocol
        self._ctx = None

    def context(self):
        if self._ctx is None:
            self._ctx = Context()
        return self._ctx

    # -- size -----------------------------------------------------------------
    def encoded_size(self, gschema, records, n=None, offsets=None, stream=None, list_base=None):
        import torch

        n = records.numel() // gschema.record_size if n is None else n
        if offsets is None:
            offsets = torch.empty(n + 1, dtype=torch.int64, device=records.device)
        st, total = _lib.Status(), ctypes.c_uint64()
        _lib.lib().tgpu_encoded_size(self.context().handle, gschema.handle, self.protocol,
                                     _ptr(records), n, _ptr(list_base), _ptr(offsets),
                                     _stream(stream),
                                     ctypes.byref(st), ctypes.byref(total))
        raise_for_status(st)
        return offsets, total.value

    # -- encode ---------------------------------------------------------------
    def serialize(self, gschema, records, n=None, string_base=None, list_base=None,
                  out=None, offsets=True, stream=None, sync=True):
        """Encodes n records (a uint8 device tensor in the schema layout).
        Returns (wire[:size], offsets or None) when sync, else the raw buffers."""
        import torch

        n = records.numel() // gschema.record_size if n is None else n
        dev = records.device
        off_t = None
        if offsets is True:
            off_t = torch.empty(n + 1, dtype=torch.int64, device=dev)
        elif offsets is not None and offsets is not False:
            off_t = offsets
        if out is None:
            L = gschema.fixed_wire_size(self.protocol)
            if L:
                cap = n * L
            else:
                size_offs = off_t if off_t is not None else torch.empty(
                    n + 1, dtype=torch.int64, device=dev)
                _, cap = self.encoded_size(gschema, records, n, size_offs, stream, list_base)
            out = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
        st, size = _lib.Status(), ctypes.c_uint64()
        rc = _lib.lib().tgpu_encode_batch(
            self.context().handle, gschema.handle, self.protocol, _ptr(records), n,
            _ptr(string_base), _ptr(list_base), _ptr(out), out.numel(), _ptr(off_t),
            _stream(stream), ctypes.byref(st) if sync else None,
            ctypes.byref(size) if sync else None)
        if not sync:
            if rc:
                raise TgpuError("tgpu_encode_batch: %s" % _lib.CODES.get(rc, rc))
            return out, off_t
        raise_for_status(st)
        return out[: size.value], off_t

    # -- decode ---------------------------------------------------------------
    def arena_bytes(self, gschema, in_len):
        """List arena a decode of in_len bytes needs (tgpu_schema_arena_scale)."""
        return in_len * _lib.lib().tgpu_schema_arena_scale(gschema.handle, self.protocol)

    def deserialize(self, gschema, wire, n, offsets=None, limits=None, records=None,
                    arena=None, stream=None, sync=True):
        """Decodes n records from the stream `wire` (uint8 device tensor).
        Returns (records, arena, consumed_bytes)."""
        import torch

        dev = wire.device
        if records is None:
            records = torch.empty(max(n * gschema.record_size, 1), dtype=torch.uint8, device=dev)
        cap = self.arena_bytes(gschema, wire.numel())
        if arena is None and cap:
            arena = torch.empty(cap, dtype=torch.uint8, device=dev)
        lim = None
        if limits is not None:
            lim = _lib.Limits(*limits) if not isinstance(limits, _lib.Limits) else limits
        st = _lib.Status()
        n_dec, consumed = ctypes.c_uint64(), ctypes.c_uint64()
        rc = _lib.lib().tgpu_decode_batch(
            self.context().handle, gschema.handle, self.protocol, _ptr(wire), wire.numel(),
            _ptr(offsets), n, _ptr(records), _ptr(arena), arena.numel() if arena is not None else 0,
            ctypes.byref(lim) if lim is not None else None, _stream(stream),
            ctypes.byref(st) if sync else None, ctypes.byref(n_dec) if sync else None,
            ctypes.byref(consumed) if sync else None)
        if not sync:
            if rc:
                raise TgpuError("tgpu_decode_batch: %s" % _lib.CODES.get(rc, rc))
            return records, arena, None
        raise_for_status(st)
        return records, arena, consumed.value

    def deserialize_status(self, gschema, wire, n, offsets=None, limits=None, stream=None):
        """Like deserialize but returns (records, arena, status, n_decoded,
        consumed) instead of raising — used by the parity tests."""
        import torch

        dev = wire.device
        records = torch.zeros(max(n * gschema.record_size, 1), dtype=torch.uint8, device=dev)
        cap = self.arena_bytes(gschema, wire.numel())
        arena = torch.zeros(max(cap, 1), dtype=torch.uint8, device=dev)
        lim = None
        if limits is not None:
            lim = _lib.Limits(*limits)
        st = _lib.Status()
        n_dec, consumed = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.lib().tgpu_decode_batch(
            self.context().handle, gschema.handle, self.protocol, _ptr(wire), wire.numel(),
            _ptr(offsets), n, _ptr(records), _ptr(arena), cap,
            ctypes.byref(lim) if lim is not None else None, _stream(stream), ctypes.byref(st),
            ctypes.byref(n_dec), ctypes.byref(consumed))
        return records, arena, st, n_dec.value, consumed.value

    def transcode(self, gschema, wire, n, to_protocol, offsets=None, out=None, limits=None,
                  stream=None, want_offsets=True):
        """Re-encodes n records of `wire` (this serializer's protocol) into
        `to_protocol` on the device (tgpu_transcode_batch). Returns (out,
        out_offsets, status, n_done, out_size); never raises on data errors.
        want_offsets=False: no output offsets are asked for (out_offsets is
        None)."""
        import torch

        dev = wire.device
        if out is None:
            # no wire byte grows by more than 8x in another protocol (a
            # 1-byte Compact varint list element is 8 Binary bytes)
            out = torch.empty(max(8 * wire.numel() + 16, 16), dtype=torch.uint8, device=dev)
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev) if want_offsets else None
        lim = _lib.Limits(*limits) if limits is not None else None
        st = _lib.Status()
        done, size = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.lib().tgpu_transcode_batch(
            self.context().handle, gschema.handle, self.protocol, to_protocol, _ptr(wire),
            wire.numel(), _ptr(offsets), n, _ptr(out), out.numel(), _ptr(offs),
            ctypes.byref(lim) if lim is not None else None, _stream(stream), ctypes.byref(st),
            ctypes.byref(done), ctypes.byref(size))
        return out, offs, st, done.value, size.value


    def decode_stream(self, gschema, wire, begin=0, end=None, speculative=False,
                      max_records=None, offsets=None, records=None, arena=None, limits=None,
                      stream=None):
        """Index + decode of the records beginning in [begin, end) of an
        unindexed stream (tgpu_decode_stream). Returns (records, arena,
        offsets, n, first_start, last_end, status) without raising."""
        import torch

        end = wire.numel() if end is None else end
        dev = wire.device
        if max_records is None:
            # a record can be one byte (STOP), so end - begin bounds the count;
            # sizing records for that is up to 8 x S per byte: count first
            # (an extra index pass: hot callers pass max_records, as
            # bench.py's config 5 does)
            max_records = self._count_records(gschema, wire, begin, end, speculative, limits,
                                              stream)
        if offsets is None:
            offsets = torch.empty(max_records + 1, dtype=torch.int64, device=dev)
        if records is None:
            records = torch.zeros(max(max_records * gschema.record_size, 1), dtype=torch.uint8,
                                  device=dev)
        cap = self.arena_bytes(gschema, wire.numel())
        if arena is None and cap:
            arena = torch.zeros(cap, dtype=torch.uint8, device=dev)
        lim = _lib.Limits(*limits) if limits is not None else None
        st = _lib.Status()
        n, first, last = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _lib.lib().tgpu_decode_stream(
            self.context().handle, gschema.handle, self.protocol, _ptr(wire), wire.numel(),
            begin, end, 1 if speculative else 0, _ptr(offsets), max_records, _ptr(records),
            _ptr(arena), arena.numel() if arena is not None else 0,
            ctypes.byref(lim) if lim is not None else None, _stream(stream), ctypes.byref(st),
            ctypes.byref(n), ctypes.byref(first), ctypes.byref(last))
        return records, arena, offsets, n.value, first.value, last.value, st

    # -- host memory ----------------------------------------------------------
    def deserialize_host(self, gschema, wire, n, records=None, chunk=0, limits=None):
        """Host-memory decode (tgpu_decode_host): `wire` and `records` are host
        buffers (numpy uint8 arrays or CPU tensors, pinned or pageable); the
        batch is pipelined through the GPU in chunks of `chunk` records.
        Returns (records, status, n_decoded, consumed) without raising."""
        import numpy as np

        if records is None:
            records = np.zeros(max(n * gschema.record_size, 1), np.uint8)
        lim = _lib.Limits(*limits) if limits is not None else None
        st = _lib.Status()
        n_dec, consumed = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.lib().tgpu_decode_host(
            self.context().handle, gschema.handle, self.protocol, _hptr(wire), _hlen(wire), n,
            _hptr(records), chunk, ctypes.byref(lim) if lim is not None else None,
            ctypes.byref(st), ctypes.byref(n_dec), ctypes.byref(consumed))
        return records, st, n_dec.value, consumed.value

    def deserialize_host_ex(self, gschema, wire, n, limits=None):
        """Host-memory decode of any schema (tgpu_decode_host_ex, one resident
        pass). Returns (records, arena, status, n_decoded, consumed); spans
        index `wire` (strings) and `arena` (list elements)."""
        import numpy as np

        records = np.zeros(max(n * gschema.record_size, 1), np.uint8)
        cap = self.arena_bytes(gschema, _hlen(wire))
        arena = np.zeros(max(cap, 1), np.uint8)
        lim = _lib.Limits(*limits) if limits is not None else None
        st = _lib.Status()
        n_dec, consumed = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.lib().tgpu_decode_host_ex(
            self.context().handle, gschema.handle, self.protocol, _hptr(wire), _hlen(wire), n,
            _hptr(records), _hptr(arena) if cap else None, cap,
            ctypes.byref(lim) if lim is not None else None, ctypes.byref(st),
            ctypes.byref(n_dec), ctypes.byref(consumed))
        return records, arena, st, n_dec.value, consumed.value

    def serialize_host_ex(self, gschema, records, n, strings=None, lists=None, out=None):
        """Host-memory encode of any schema (tgpu_encode_host_ex). Returns
        (out, offsets, status, size)."""
        import numpy as np

        if out is None:
            total = _hlen(records) + (_hlen(strings) if strings is not None else 0) + \
                (_hlen(lists) if lists is not None else 0)
            out = np.zeros(max(8 * total + 16, 16), np.uint8)
        offs = np.zeros(n + 1, np.uint64)
        st, size = _lib.Status(), ctypes.c_uint64()
        _lib.lib().tgpu_encode_host_ex(
            self.context().handle, gschema.handle, self.protocol, _hptr(records), n,
            _hptr(strings) if strings is not None else None,
            _hlen(strings) if strings is not None else 0,
            _hptr(lists) if lists is not None else None, _hlen(lists) if lists is not None else 0,
            _hptr(out), _hlen(out), offs.ctypes.data, ctypes.byref(st), ctypes.byref(size))
        return out, offs, st, size.value

    def serialize_host(self, gschema, records, n, out=None, chunk=0):
        """Host-memory encode (tgpu_encode_host) of n records held in host
        memory into `out` (allocated when None). Returns (out, status, size)."""
        import numpy as np

        if out is None:
            out = np.zeros(max(n * gschema.fixed_wire_size(self.protocol), 1), np.uint8)
        st, size = _lib.Status(), ctypes.c_uint64()
        _lib.lib().tgpu_encode_host(self.context().handle, gschema.handle, self.protocol,
                                    _hptr(records), n, _hptr(out), _hlen(out), chunk,
                                    ctypes.byref(st), ctypes.byref(size))
        return out, st, size.value

    # -- stream index -------------------------------------------------------
    def _count_records(self, gschema, wire, begin, end, speculative, limits, stream):
        """Records beginning in [begin, end): an index into a small buffer
        (an estimate of one record per 16 bytes) that reports the exact count
        when it overflows (TGPU_ERR_OUTPUT_OVERFLOW), so callers that did
        not give max_records allocate for the records found, not for one
        record per byte."""
        span = max(end - begin, 0)
        guess = min(span, max(1024, span // 16))
        _, n, _, _, st = self.index_stream(gschema, wire, begin, end, speculative,
                                           max_records=guess, limits=limits, stream=stream,
                                           check=False)
        return max(n, guess)

    def index_stream(self, gschema, wire, begin=0, end=None, speculative=False,
                     max_records=None, offsets=None, limits=None, stream=None, check=True):
        """Record starts of an unindexed stream (tgpu_index_stream): the records
        beginning in [begin, end) of `wire` (a uint8 device tensor; records may
        run past `end`). Returns (offsets[:n+1], n, first_start, last_end,
        status); raises on a reader error when `check`."""
        import torch

        end = wire.numel() if end is None else end
        if max_records is None:
            # sized by a first index into a guessed buffer; when the guess
            # holds every record that index is the result (no second pass)
            span = max(end - begin, 0)
            guess = min(span, max(1024, span // 16))
            r = self.index_stream(gschema, wire, begin, end, speculative, max_records=guess,
                                  limits=limits, stream=stream, check=False)
            if r[1] <= guess and r[4].code != 21:  # TGPU_ERR_OUTPUT_OVERFLOW
                if check:
                    raise_for_status(r[4])
                return r
            max_records = r[1]
            offsets = None
        if offsets is None:
            offsets = torch.empty(max_records + 1, dtype=torch.int64, device=wire.device)
        lim = None
        if limits is not None:
            lim = _lib.Limits(*limits) if not isinstance(limits, _lib.Limits) else limits
        st = _lib.Status()
        n, first, last = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _lib.lib().tgpu_index_stream(
            self.context().handle, gschema.handle, self.protocol, _ptr(wire), wire.numel(),
            begin, end, 1 if speculative else 0, _ptr(offsets), max_records,
            ctypes.byref(lim) if lim is not None else None, _stream(stream), ctypes.byref(st),
            ctypes.byref(n), ctypes.byref(first), ctypes.byref(last))
        if check:
            raise_for_status(st)
        k = min(n.value, max_records)
        return offsets[: k + 1], n.value, first.value, last.value, st


    # -- schemaless skim ----------------------------------------------------
    def skim(self, wire, offsets, n=None, max_fields=16, limits=None, stream=None, check=True,
             fields=None, counts=None, nest=0):
        """Top-level fields of records [0, n) of an indexed stream
        (tgpu_skim_batch; nest > 0: also the fields of struct-valued fields
        that many levels down, pre-order, level in flags bits 2-5 —
        tgpu_skim_batch_ex): `wire` a uint8 device tensor, `offsets` its n+1
        record starts (device int64). Returns (fields, counts, n_done,
        status): fields a uint8 device tensor of max_fields * n
        tgpu_skim_field entries, field-major (skim_records() views it as a
        numpy (n, max_fields) record array),
        counts an int32 device tensor of each record's field count. `fields`
        / `counts` may be given (preallocated, reused across calls)."""
        import torch

        if n is None:
            n = offsets.numel() - 1
        if fields is None:
            fields = torch.zeros(max(n * max_fields * 16, 16), dtype=torch.uint8,
                                 device=wire.device)
        if counts is None:
            counts = torch.zeros(max(n, 1), dtype=torch.int32, device=wire.device)
        assert fields.numel() >= n * max_fields * 16 and counts.numel() >= n
        lim = None
        if limits is not None:
            lim = _lib.Limits(*limits) if not isinstance(limits, _lib.Limits) else limits
        st, done = _lib.Status(), ctypes.c_uint64()
        _lib.lib().tgpu_skim_batch_ex(
            self.context().handle, self.protocol, _ptr(wire), wire.numel(), _ptr(offsets), n,
            _ptr(fields), max_fields, _ptr(counts), nest,
            ctypes.byref(lim) if lim is not None else None, _stream(stream), ctypes.byref(st),
            ctypes.byref(done))
        if check:
            raise_for_status(st)
        return fields, counts[:n], done.value, st

    def skim_stream(self, wire, max_fields=16, limits=None, stream=None):
        """Skim of an unindexed stream of back-to-back records (a file): the
        record index is found first without a schema (tgpu_index_stream with
        a field-less struct: every record walked by the reader's skip), then
        tgpu_skim_batch runs over it. Returns (offsets[:n+1], fields, counts,
        n); raises on the first record the reader rejects."""
        from .schema import Schema, Struct

        if getattr(self, "_any_schema", None) is None:
            self._any_schema = GpuSchema(Schema(Struct("Any", [])))
        offs, n, _, _, _ = self.index_stream(self._any_schema, wire, limits=limits, stream=stream)
        fields, counts, _, _ = self.skim(wire, offs, n, max_fields=max_fields, limits=limits,
                                         stream=stream)
        return offs, fields, counts, n


def skim_records(fields, n, max_fields):
    """Field-major tgpu_skim_field entries (uint8 tensor or array) as a numpy
    record array of shape (n, max_fields): [i, k] = field k of record i."""
    import numpy as np

    a = fields.cpu().numpy() if hasattr(fields, "cpu") else np.asarray(fields)
    a = a[: n * max_fields * 16].view(np.dtype(_lib.SKIM_FIELDS))
    return a.reshape(max_fields, n).T

BinarySerializer = BatchSerializer(PROTOCOL_BINARY)
CompactSerializer = BatchSerializer(PROTOCOL_COMPACT)
CompactV1Serializer = BatchSerializer(PROTOCOL_COMPACT_V1)
