/*
 * thrift_gpu.h — C-ABI boundary of the MI355X bulk Thrift record codec.
 *
 * This is the drop-in boundary for fbthrift's bulk serialization path: whole
 * batches of same-schema records cross it into gfx950 HIP kernels. Every entry
 * point is plain C (pointers + sizes, no C++/torch types), so it can be bound
 * from C++ (include/thrift_gpu/GpuBatchSerializer.h), ctypes, cgo or JNI.
 *
 * What each entry point replaces in the reference (fbthrift, paths relative to
 * the fbthrift source tree):
 *
 *  tgpu_schema_create
 *      the codegen'd per-type metadata that drives T::readNoXfer / T::write
 *      (thrift/compiler/generate/templates/cpp2/module_types_custom_protocol_h/
 *       deserialize_struct.whisker:19-160, serialize_struct.whisker:40-67) and
 *      its runtime-table twin StructInfo/FieldInfo/TypeInfo
 *      (thrift/lib/cpp2/protocol/TableBasedSerializer.h:90-118,205-302).
 *  tgpu_encode_batch
 *      N x Serializer<R,W>::serialize(obj, &queue) appending to one IOBufQueue
 *      (thrift/lib/cpp2/protocol/Serializer.h:136-148) i.e. N x T::write<P>.
 *  tgpu_index_stream
 *      the record boundaries that repeated deserialize<T>(Cursor&) walks over
 *      a concatenated stream (Serializer.h:97-100), found in parallel.
 *  tgpu_decode_batch
 *      N x Serializer<R,W>::deserialize<T>(Cursor&) over a concatenated record
 *      stream (Serializer.h:97-100, :192-204), i.e. N x T::readNoXfer<P>.
 *  tgpu_status
 *      the exceptions the reference throws: TProtocolException{type}
 *      (thrift/lib/cpp/protocol/TProtocolException.h:41-51) and
 *      std::out_of_range (folly cursor underflow; invalid varint,
 *      thrift/lib/cpp/util/VarintUtils.cpp:125-127). A C-ABI cannot throw, so
 *      the first failing record, its byte offset and exception class are
 *      latched (the transcode C-ABI precedent:
 *      thrift/lib/cpp2/transcode/TranscodeErrc.h:32-44).
 *  tgpu_limits
 *      gflags thrift_cpp2_protocol_reader_string_limit / _container_limit
 *      (thrift/lib/cpp2/protocol/BinaryProtocol.cpp:23-30) and
 *      thrift_protocol_max_depth (thrift/lib/cpp2/protocol/Protocol.cpp:21-24).
 *
 * Memory: every data pointer passed to encode/decode is a DEVICE pointer
 * (hipMalloc'd HBM) unless stated otherwise; `stream` is a hipStream_t passed
 * as void* (NULL = the default stream). Calls are asynchronous with respect to
 * the host unless a host `tgpu_status*` is passed, in which case the call waits
 * for the stream and fills it (the synchronous, exception-equivalent form).
 *
 * Record layout (the "codegen'd struct layout", device form): members in IDL
 * declaration order at natural alignment, then one isset byte per field
 * (thrift/lib/cpp2/detail/Isset.h:243-296), size rounded up to the alignment.
 * Device-unfriendly members use 16-byte spans instead of std::string /
 * std::vector: see tgpu_span. tgpu_layout_compute() fills offsets by that rule.
 */
#ifndef THRIFT_GPU_H_
#define THRIFT_GPU_H_

#ifndef __HIPCC_RTC__ /* runtime-compiled device code declares its own types */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define TGPU_ABI_VERSION 1

/* Protocol ids: thrift/lib/cpp/protocol/TProtocolTypes.h:24-27. */
enum tgpu_protocol {
  TGPU_PROTOCOL_BINARY = 0,
  TGPU_PROTOCOL_COMPACT = 2,
  /* CompactV1ProtocolReader/Writer (thrift/lib/cpp2/protocol/
     CompactV1Protocol.h, -inl.h:36-41,73-79): Compact with doubles written
     little-endian. It has no PROTOCOL_TYPES id; this value is the library's. */
  TGPU_PROTOCOL_COMPACT_V1 = 0x102,
};

/* Wire types: thrift/lib/cpp/protocol/TType.h:31-51 (same numeric values). */
enum tgpu_ttype {
  TGPU_T_STOP = 0,
  TGPU_T_VOID = 1,
  TGPU_T_BOOL = 2,
  TGPU_T_BYTE = 3,
  TGPU_T_DOUBLE = 4,
  TGPU_T_I16 = 6,
  TGPU_T_I32 = 8,
  TGPU_T_U64 = 9,
  TGPU_T_I64 = 10,
  TGPU_T_STRING = 11,
  TGPU_T_STRUCT = 12,
  TGPU_T_MAP = 13,
  TGPU_T_SET = 14,
  TGPU_T_LIST = 15,
  TGPU_T_UTF8 = 16,
  TGPU_T_UTF16 = 17,
  TGPU_T_STREAM = 18,
  TGPU_T_FLOAT = 19,
};

/* Field qualifiers (module_types_custom_protocol.whisker:79-94). */
enum tgpu_qualifier {
  TGPU_UNQUALIFIED = 0, /* always written, isset set on read */
  TGPU_OPTIONAL = 1,    /* written only when isset != 0 */
  /* @thrift.TerseWrite: written only when not empty (op::isEmpty,
     thrift/lib/cpp2/op/detail/Clear.h:98-127 via fields.whisker:84): a
     scalar whose bits are not all zero (-0.0 is written), a non-empty
     string/list/set; read like an unqualified field. Not for struct fields. */
  TGPU_TERSE = 2,
  /* `required`: always written; read like an unqualified field. With the
     struct flag TGPU_STRUCT_ENFORCE_REQUIRED (the generated reader built with
     the deprecated_enforce_required compiler option) a struct whose read
     did not see the field fails with TGPU_ERR_MISSING_REQUIRED_FIELD
     (deserialize_struct.whisker:116-124). Its isset byte records the read. */
  TGPU_REQUIRED = 3,
  /* A boxed struct field: cpp.ref / @cpp.Ref (std::unique_ptr<T>) or
     @thrift.Box (thrift::box<T>), the form recursive structs take
     (struct Node { 2: optional Node next (cpp.ref) }). The member is a
     tgpu_span pointing at the struct's object in the list arena (decode)
     or relative to list_base (encode): length 1 = present, 0 = null.
     Read: a fresh object is read and assigned once its read completed
     (deserialize_field.whisker:21-23,49-51: make_mutable_smart_ptr, read,
     move). Write (serialize_field.whisker:32-50): TGPU_BOXED is always
     written, a null one as an empty struct (writeStructBegin,
     writeFieldStop, writeStructEnd); TGPU_OPTIONAL_BOXED only when its
     isset byte is set (a null one then also as an empty struct). */
  TGPU_BOXED = 4,
  TGPU_OPTIONAL_BOXED = 5,
};

/*
 * One field of a struct, in IDL declaration order (= serialization order,
 * thrift/compiler/generate/t_whisker_generator.cc:231-236).
 *   ttype        T_BOOL..T_FLOAT scalar, T_STRING (binary/string), T_STRUCT,
 *                T_LIST or T_SET, T_MAP.
 *   elem_ttype   element type for T_LIST/T_SET, key type for T_MAP, else 0.
 *                A list/set element, a map key and a map value may each be
 *                a scalar, a string, a struct or itself a list/set/map.
 *   val_ttype    value type for T_MAP (any type, like a list element), else 0.
 * A string inside a container is a tgpu_span (like a string field); the
 * list arena then needs tgpu_schema_arena_scale bytes per input byte.
 *   struct_index the struct (index into the schema's struct table) of a
 *                T_STRUCT field, of a list/set's T_STRUCT elements or of a
 *                map's T_STRUCT values; else -1.
 *   type_index   1 + index into the schema's type table (tgpu_type_desc,
 *                tgpu_schema_create_ex) of the container that is this
 *                list/set's element or this map's value type; 0 otherwise.
 *   key_index    T_MAP whose key is a struct or a container: 1 + index into
 *                the type table of the key's type (a node of ttype T_STRUCT
 *                naming the struct, or the key container's node); else 0.
 * Structs may be recursive through containers (struct Tree
 * { 1: list<Tree> kids }) and through boxed fields; a struct cannot hold
 * itself by value. Records nest as deep as the data does: the device reader
 * and writer keep a few frames per lane and redo deeper records in a pass
 * whose lanes keep their frames in HBM (tgpu_limits.max_depth bounds the
 * containers, as the reference's descend/ascend does).
 * Containers hold their elements in the list arena: scalars in native
 * layout, strings and containers as tgpu_span, structs in the struct layout;
 * a map holds packed {key, value} pairs. This is the shape of the
 * reference's TypeInfo / ListFieldExt / MapFieldExt tables
 * (thrift/lib/cpp2/protocol/TableBasedForwardTypes.h:37-93), which nest the
 * same way.
 */
typedef struct tgpu_field_desc {
  int16_t id;
  uint8_t ttype;
  uint8_t elem_ttype;
  uint8_t qualifier;
  uint8_t val_ttype;
  uint16_t key_index;
  uint32_t member_offset;
  uint32_t isset_offset;
  int32_t struct_index;
  uint32_t type_index;
} tgpu_field_desc; /* 24 bytes */

/*
 * A container type nested inside a container (list<list<i32>>,
 * map<string, list<Struct>>, ...): the same description a container field
 * carries (elem_ttype / val_ttype / struct_index / type_index / key_index as
 * in tgpu_field_desc), for a list/set element, a map value or a map key.
 * A map key that is a struct is a node of ttype T_STRUCT whose struct_index
 * names the struct (referenced only through key_index).
 */
typedef struct tgpu_type_desc {
  uint8_t ttype;      /* T_LIST, T_SET or T_MAP (T_STRUCT: a struct key) */
  uint8_t elem_ttype;
  uint8_t val_ttype;
  uint8_t reserved0;
  int32_t struct_index;
  uint32_t type_index;
  uint32_t key_index;
} tgpu_type_desc; /* 16 bytes */

/* Struct flags. */
enum tgpu_struct_flags {
  /* A Thrift union (deserialize_union.whisker / serialize_union.whisker):
     each member has its own slot and isset byte; the active member is the
     one whose isset byte is set (at most one on read, the first set one is
     written). Reading a member first clears the whole union (emplace), an
     immediate STOP clears it (apache::thrift::clear), a second field is
     TGPU_ERR_UNION_MISSING_STOP. Members must be unqualified. */
  TGPU_STRUCT_UNION = 1,
  /* Readers check the struct's required fields (TGPU_REQUIRED): one not
     read by this struct's read -> TGPU_ERR_MISSING_REQUIRED_FIELD, after its
     STOP. Structs with required fields past the 64th field are rejected. */
  TGPU_STRUCT_ENFORCE_REQUIRED = 2,
};

/* A struct = a contiguous run of fields. Struct 0 is the record (root) type. */
typedef struct tgpu_struct_desc {
  uint32_t first_field;
  uint32_t num_fields;
  uint32_t size;  /* sizeof(record), multiple of align */
  uint32_t align;
  uint32_t flags; /* tgpu_struct_flags */
} tgpu_struct_desc; /* 20 bytes */

/*
 * Device form of a string/binary, list/set or map member (16 bytes, align 8).
 * Decode: a string's `offset` is relative to the decoded input stream `in`
 *         (zero-copy view, ExternalBufferSharing::SHARE_EXTERNAL_BUFFER,
 *         thrift/lib/cpp2/protocol/Protocol.h:96-99); a list's `offset` is
 *         relative to `list_arena` where its elements were written in native
 *         little-endian layout. Empty strings/lists decode to {0, 0}.
 * Encode: a string's `offset` is relative to `string_base`, a list's to
 *         `list_base`; `length` is bytes (string) or elements (list).
 * Map:    `length` = pairs, in wire order, packed {key, value} (stride key
 *         size + value size, no padding) from `offset`. Inserting the
 *         pairs in order with emplace (the first of equal keys wins) gives
 *         the reference's std::map (deserialize_known_length_map,
 *         thrift/lib/cpp2/op/detail/EncodeHelpers.h:188-205); a map whose
 *         read fails keeps the pairs read before the failure. Encode writes
 *         the pairs in the order given (sorted keys = std::map's order).
 */
typedef struct tgpu_span {
  uint64_t offset;
  uint32_t length;
  uint32_t reserved;
} tgpu_span;

/* Reader limits. 0 = unlimited for string/container (reference defaults).
 * max_depth is FLAGS_thrift_protocol_max_depth (skip recursion limit,
 * Protocol.h:202-205); height is ProtocolBase::setHeight (container/struct
 * nesting counter, Protocol.h:59-78), 0 = max_depth as in the reference. */
typedef struct tgpu_limits {
  int32_t string_limit;
  int32_t container_limit;
  int32_t max_depth; /* default 12000 */
  int32_t height;    /* default 0 (= max_depth) */
} tgpu_limits;

/* Result codes. */
enum tgpu_code {
  TGPU_OK = 0,
  /* std::out_of_range */
  TGPU_ERR_UNDERFLOW = 1,        /* cursor ran out of bytes (folly readBE) */
  TGPU_ERR_INVALID_VARINT = 2,   /* "invalid varint read" */
  /* TProtocolException */
  TGPU_ERR_BOOL_VALUE = 3,       /* INVALID_DATA: Binary bool byte >= 2 */
  TGPU_ERR_INVALID_SKIP_TYPE = 4,/* INVALID_DATA */
  TGPU_ERR_TRUNCATED = 5,        /* INVALID_DATA: throwTruncatedData */
  TGPU_ERR_NEGATIVE_SIZE = 6,    /* NEGATIVE_SIZE */
  TGPU_ERR_SIZE_LIMIT = 7,       /* SIZE_LIMIT */
  TGPU_ERR_DEPTH_LIMIT = 8,      /* DEPTH_LIMIT */
  TGPU_ERR_BAD_TYPE = 9,         /* UNKNOWN: Compact "don't know what type" */
  TGPU_ERR_UNION_MISSING_STOP = 12, /* INVALID_DATA: throwUnionMissingStop
                                       (TProtocolException.cpp:23-27) */
  TGPU_ERR_MISSING_REQUIRED_FIELD = 13, /* MISSING_REQUIRED_FIELD:
                                           throwMissingRequiredField
                                           (TProtocolException.cpp:54-58) */
  /* writer-side: the reference aborts the process (validate_bool,
     thrift/lib/cpp2/protocol/Protocol.h:126-163) or throws SIZE_LIMIT */
  TGPU_ERR_INVALID_BOOL_WRITE = 10,
  TGPU_ERR_WRITE_SIZE_LIMIT = 11,
  /* boundary / runtime errors (no reference counterpart) */
  TGPU_ERR_INDEX_MISMATCH = 20,  /* record length disagrees with offsets[] */
  TGPU_ERR_OUTPUT_OVERFLOW = 21, /* encode output / list arena too small */
  TGPU_ERR_UNSUPPORTED = 22,     /* schema feature not supported on device */
  TGPU_ERR_INVALID_ARGUMENT = 23,
  TGPU_ERR_HIP = 24,
};

enum tgpu_exc_class {
  TGPU_EXC_NONE = 0,
  TGPU_EXC_OUT_OF_RANGE = 1,  /* std::out_of_range */
  TGPU_EXC_PROTOCOL = 2,      /* apache::thrift::protocol::TProtocolException */
  TGPU_EXC_ABORT = 3,         /* reference would LOG(FATAL) */
  TGPU_EXC_RUNTIME = 4,       /* tgpu usage / HIP error */
};

typedef struct tgpu_status {
  int32_t code;         /* enum tgpu_code */
  int32_t exc_class;    /* enum tgpu_exc_class */
  int32_t tproto_type;  /* TProtocolExceptionType when exc_class == PROTOCOL */
  int32_t reserved;
  uint64_t record;      /* index of the first failing record */
  uint64_t byte_offset; /* stream offset of the read/write that failed */
} tgpu_status;

typedef struct tgpu_schema tgpu_schema;   /* opaque; lives on one device */
typedef struct tgpu_context tgpu_context; /* opaque; workspace + result slot */

/* ---- library ---------------------------------------------------------- */
int tgpu_abi_version(void);
const char* tgpu_code_name(int code);
/* Maps a code to (exc_class, tproto_type). */
void tgpu_code_classify(int code, int32_t* exc_class, int32_t* tproto_type);

/* ---- schema ----------------------------------------------------------- */
/* Fills member_offset / isset_offset of every field and size/align of every
 * struct by the declaration-order layout rule. Host-only, no device work. */
int tgpu_layout_compute(tgpu_struct_desc* structs, uint32_t n_structs,
                        tgpu_field_desc* fields, uint32_t n_fields);
/* Validates and uploads a schema to the current HIP device. */
int tgpu_schema_create(const tgpu_struct_desc* structs, uint32_t n_structs,
                       const tgpu_field_desc* fields, uint32_t n_fields,
                       tgpu_schema** out);
/* The same with a table of nested container types (types[k] is referenced
 * as type_index k + 1 by fields and by other types). */
int tgpu_schema_create_ex(const tgpu_struct_desc* structs, uint32_t n_structs,
                          const tgpu_field_desc* fields, uint32_t n_fields,
                          const tgpu_type_desc* types, uint32_t n_types, tgpu_schema** out);
void tgpu_schema_destroy(tgpu_schema* schema);
/* sizeof(record) of the root struct. */
uint32_t tgpu_schema_record_size(const tgpu_schema* schema);
/* List arena bytes a decode needs per input byte: 0 without lists/sets/
 * maps; 1 Binary / 8 Compact for scalar elements; 4 Binary / 16 Compact
 * when some container holds strings (16-byte spans). A schema with
 * containers of structs or of containers ("nested") reads each record's
 * containers into a region of its own, scale x [record start, record end)
 * of the arena, allocated in wire order (8-byte aligned); its scale bounds
 * element bytes per wire byte (e.g. sizeof(struct) for a list of structs,
 * as an element struct can be a single STOP byte on the wire).
 * Where arrays go (the records' spans say it; other arena bytes are
 * unspecified):
 *  - flat-list schemas (every container a list or set of scalars, at most
 *    8 of them per record counting by-value struct members; no maps, no
 *    strings in containers, nothing boxed): the BLOCK RULE. Records are
 *    grouped by index in blocks of 64; block b's arrays are dense, back to
 *    back in read order (records in order, a record's arrays in wire
 *    order), each 8-byte aligned, from align8(scale x the wire start of
 *    record 64 b) — the elements of a list are one contiguous array, as the
 *    reference's std::vector is, and the block's arrays fit the wire bytes
 *    it came from (x scale);
 *  - other schemas without regions: each array at scale x the wire
 *    position of its first element (the position rule). */
uint32_t tgpu_schema_arena_scale(const tgpu_schema* schema, int protocol);

/* Canonical wire length of every record if it is fixed for `protocol`
 * (Binary with only fixed-width fields), else 0. */
uint64_t tgpu_schema_fixed_wire_size(const tgpu_schema* schema, int protocol);

/*
 * Compiles the schema's record codec for `protocol` into specialized gfx950
 * kernels now (hipRTC) — the run-time counterpart of the reference's per-type
 * code generation (thrift1 emitting T::readNoXfer / T::write,
 * deserialize_struct.whisker:19-160, serialize_struct.whisker:40-67). Without
 * this call the library compiles on the first batch of >= 64 Ki records and
 * interprets the schema below that (env TGPU_JIT=1: compile on first use,
 * TGPU_JIT=0: never). Results are identical either way.
 * Returns TGPU_OK, or TGPU_ERR_UNSUPPORTED when the schema has no canonical
 * record program for the protocol (optional fields, maps, ...) or the
 * compiler is unavailable (the interpreting kernels are used).
 */
int tgpu_schema_compile(const tgpu_schema* schema, int protocol);
/* Diagnostics: generates and compiles the kernels of the schema given by the
 * tables (as for tgpu_schema_create) for `arch` (e.g. "gfx950"; NULL =
 * gfx950) without loading them — needs no GPU. The compiler log goes to
 * log[0..log_capacity) (may be NULL). TGPU_ERR_UNSUPPORTED as for
 * tgpu_schema_compile. Nested container types need the _ex form (here a
 * field with type_index != 0 has no program). arch "" (empty): the program is
 * built and the kernel sources generated, nothing compiled (whether a schema
 * has a program, in milliseconds instead of seconds). */
int tgpu_schema_compile_check(const tgpu_struct_desc* structs, uint32_t n_structs,
                              const tgpu_field_desc* fields, uint32_t n_fields, int protocol,
                              const char* arch, char* log, uint64_t log_capacity);
/* The same with a container type table (tgpu_schema_create_ex). Schemas whose
 * lists / sets hold structs or scalar lists (and no maps or strings inside
 * containers, every field unqualified or required) compile their nested
 * record program: one decode kernel with a loop per container level. */
int tgpu_schema_compile_check_ex(const tgpu_struct_desc* structs, uint32_t n_structs,
                                 const tgpu_field_desc* fields, uint32_t n_fields,
                                 const tgpu_type_desc* types, uint32_t n_types, int protocol,
                                 const char* arch, char* log, uint64_t log_capacity);

/* The transcoder's kernels for a schema with a flat record program in both
 * protocols (tgpu_transcode_batch without materialized records): generated
 * and compiled for `arch` without a GPU, as tgpu_schema_compile_check. */
int tgpu_transcode_compile_check(const tgpu_struct_desc* structs, uint32_t n_structs,
                                 const tgpu_field_desc* fields, uint32_t n_fields,
                                 int from_protocol, int to_protocol, const char* arch, char* log,
                                 uint64_t log_capacity);

/* ---- context ---------------------------------------------------------- */
int tgpu_context_create(tgpu_context** out);
void tgpu_context_destroy(tgpu_context* ctx);
/* Pre-sizes the workspace for batches of up to n_records (so later calls do
 * no allocation and can be captured into a hipGraph). */
int tgpu_context_reserve(tgpu_context* ctx, uint64_t n_records);
/* Waits for `stream` and reports the last call's result on this context. */
int tgpu_context_wait(tgpu_context* ctx, void* stream, tgpu_status* st,
                      uint64_t* n_done, uint64_t* bytes);
/*
 * Repair counters of the last stream index on this context (the parallel
 * form of the file loop, Serializer.h:97-100; tgpu_index_stream,
 * tgpu_decode_stream, unindexed tgpu_decode_batch). Waits for `stream`.
 * out[TGPU_ISTAT_*]: chunks (LDS tiles or lane chunks) of the call; tiles the
 * speculation left partial, without a start, with a broken link to their
 * predecessor; links the ordered repair lane visited; tiles whose stored
 * record starts were re-walked. A canonical stream needs no repair: every
 * counter but the first is 0 (a diagnostic: speed, not correctness, depends
 * on it). out[TGPU_ISTAT_GENERAL]: records of the context's last decode call
 * (any kind) that left the compiled / fixed-layout fast path for the general
 * reader (0 on a canonical stream); after an encode, the records a compiled
 * nested writer left to the general writer (a recursive schema's records
 * nesting past its unrolled levels); after a transcode, the records left to
 * the general reader / writer. Returns TGPU_ERR_INVALID_ARGUMENT when
 * the context has run no index (out[TGPU_ISTAT_GENERAL] is still filled).
 */
enum {
  TGPU_ISTAT_CHUNKS = 0, TGPU_ISTAT_PARTIAL = 1, TGPU_ISTAT_NO_START = 2,
  TGPU_ISTAT_BROKEN = 3, TGPU_ISTAT_REPAIRED = 4, TGPU_ISTAT_REWALKED = 5,
  TGPU_ISTAT_GENERAL = 6, TGPU_ISTAT_COUNT = 7
};
int tgpu_index_stats(tgpu_context* ctx, void* stream, uint64_t* out);

/* ---- batch encode ----------------------------------------------------- */
/*
 * Serializes records[0..n) (stride = tgpu_schema_record_size) back to back
 * into `out` (capacity out_capacity bytes). out_offsets (device, n+1 entries,
 * may be NULL) receives each record's start offset and the total size.
 * string_base / list_base are the bases the records' spans point into.
 * If st != NULL the call waits and fills st and *out_size.
 */
int tgpu_encode_batch(tgpu_context* ctx, const tgpu_schema* schema,
                      int protocol, const void* records, uint64_t n_records,
                      const void* string_base, const void* list_base,
                      void* out, uint64_t out_capacity, uint64_t* out_offsets,
                      void* stream, tgpu_status* st, uint64_t* out_size);

/*
 * Exact wire size of each record (out_offsets, device, n+1 entries, required)
 * and of the whole batch, without writing it: the bulk form of
 * T::serializedSize<P> (serialize_struct.whisker:17-26; the reference returns
 * an upper bound with varints counted at their maximum width, this is exact).
 * Validates like encode (bool bytes, string/list sizes). list_base is
 * required when the schema has lists (Compact element widths depend on the
 * element values); string payloads are not read.
 */
int tgpu_encoded_size(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                      const void* records, uint64_t n_records,
                      const void* list_base, uint64_t* out_offsets,
                      void* stream, tgpu_status* st, uint64_t* total);

/* ---- batch decode ----------------------------------------------------- */
/*
 * Deserializes n_records records from the concatenated stream in[0..in_len).
 * offsets (device, n_records+1 entries) may be given as a record index; NULL
 * means records are read back to back from offset 0 like repeated
 * deserialize<T>(Cursor&). Records are default-initialized (zero, isset 0)
 * before reading. List elements are written to list_arena (capacity
 * list_arena_capacity bytes; required size: in_len x tgpu_schema_arena_scale
 * — in_len Binary / 8 * in_len Compact for scalar elements, 0 without
 * lists/sets/maps). Bytes of list_arena outside the records' spans are
 * unspecified (a Binary decode may copy whole wire tiles there).
 * limits may be NULL (reference defaults).
 * If st != NULL the call waits and fills st, *n_decoded (records fully
 * decoded before the first failure) and *consumed (bytes consumed by them).
 */
int tgpu_decode_batch(tgpu_context* ctx, const tgpu_schema* schema,
                      int protocol, const void* in, uint64_t in_len,
                      const uint64_t* offsets, uint64_t n_records,
                      void* records, void* list_arena,
                      uint64_t list_arena_capacity, const tgpu_limits* limits,
                      void* stream, tgpu_status* st, uint64_t* n_decoded,
                      uint64_t* consumed);

/* ---- transcoding ------------------------------------------------------ */
/*
 * Re-encodes n records of a stream from one protocol into another (Binary,
 * Compact, CompactV1 in any direction, same schema) without leaving the
 * device: each output record is byte-identical to
 * serialize<To>(deserialize<From>(record)) of the reference — the bulk form
 * of the wire-to-wire transcoder (thrift/lib/cpp2/transcode/README.md:1-20,
 * schema-driven; unknown fields are dropped as the generated codec drops
 * them). The decoded records and list elements stay in a context workspace
 * in HBM between the read and the write. in/offsets/limits as for
 * tgpu_decode_batch; out/out_offsets (n+1 entries, may be NULL) as for
 * tgpu_encode_batch. Blocking. A record the reader rejects ends the batch:
 * the records before it are transcoded (*n_done, *out_size) and st is the
 * reader's status for it; an output overflow reports the encoder's.
 */
int tgpu_transcode_batch(tgpu_context* ctx, const tgpu_schema* schema, int from_protocol,
                         int to_protocol, const void* in, uint64_t in_len,
                         const uint64_t* offsets, uint64_t n_records, void* out,
                         uint64_t out_capacity, uint64_t* out_offsets,
                         const tgpu_limits* limits, void* stream, tgpu_status* st,
                         uint64_t* n_done, uint64_t* out_size);

/* ---- host-memory batches ---------------------------------------------- */
/*
 * The same calls for data that starts and ends in HOST memory (an IOBuf's
 * bytes, a host record array): Serializer::deserialize / ::serialize over a
 * host buffer (Serializer.h:62-72, :136-148), N records at a time. The batch
 * is cut into chunks of chunk_records records (0 = 4 Mi) that are pipelined
 * over three streams (copy in, kernels, copy out overlapping), so the rate is
 * the PCIe rate. Host buffers may be pinned (fastest) or pageable (pinned in
 * place for the call). Blocking; results and status exactly as for
 * tgpu_decode_batch / tgpu_encode_batch on the whole batch.
 * Scope: tgpu_encode_host needs a fixed canonical Binary record length
 * (tgpu_schema_fixed_wire_size != 0); tgpu_decode_host also takes
 * variable-length schemas without lists (decoded resident in one pass; string
 * spans are offsets into host_in). Others -> TGPU_ERR_UNSUPPORTED.
 */
int tgpu_decode_host(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                     const void* host_in, uint64_t in_len, uint64_t n_records,
                     void* host_records, uint64_t chunk_records, const tgpu_limits* limits,
                     tgpu_status* st, uint64_t* n_decoded, uint64_t* consumed);
int tgpu_encode_host(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                     const void* host_records, uint64_t n_records, void* host_out,
                     uint64_t out_capacity, uint64_t chunk_records, tgpu_status* st,
                     uint64_t* out_size);

/*
 * Host-memory batches of ANY schema (lists, sets, maps, strings, unions):
 * one resident pass — the host buffers are copied to the device, the
 * device call runs, the outputs come back (PCIe-bound; pageable buffers are
 * pinned in place for the call). Results and status exactly as for
 * tgpu_decode_batch / tgpu_encode_batch. Decode: string spans are offsets
 * into host_in, list spans into host_arena (capacity as for the device
 * arena: in_len x tgpu_schema_arena_scale; may be NULL/0 without lists).
 * Encode: spans are relative to host_strings / host_lists; host_out_offsets
 * (n+1 entries) may be NULL. Blocking.
 */
int tgpu_decode_host_ex(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                        const void* host_in, uint64_t in_len, uint64_t n_records,
                        void* host_records, void* host_arena, uint64_t arena_capacity,
                        const tgpu_limits* limits, tgpu_status* st, uint64_t* n_decoded,
                        uint64_t* consumed);
int tgpu_encode_host_ex(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                        const void* host_records, uint64_t n_records, const void* host_strings,
                        uint64_t strings_len, const void* host_lists, uint64_t lists_len,
                        void* host_out, uint64_t out_capacity, uint64_t* host_out_offsets,
                        tgpu_status* st, uint64_t* out_size);

/*
 * Host-memory batches of any schema, chunk-pipelined. Decode: the stream
 * goes to the device in chunk_bytes pieces on a copy stream while the
 * records beginning in each piece are indexed and decoded (the piece after
 * it must be resident: a record may continue there) and the previous
 * piece's records and list-arena slice come back on a third stream; every
 * finished range of records [r0, r1) is announced through on_chunk (may be
 * NULL) while later chunks are still moving, so a caller can materialize
 * them meanwhile (host_records / host_arena as for tgpu_decode_host_ex; the
 * arena slice of a range is arena_scale x its wire bytes; under the block
 * rule a range is whole blocks of 64 records, so the arena is exactly
 * tgpu_decode_host_ex's). Any chunk that
 * does not finish cleanly (a malformed record, more records than
 * n_records, a record longer than a piece) sends the whole batch through
 * the resident pass, so results and status are exactly
 * tgpu_decode_host_ex's; on_chunk then reports [r0, n_decoded + 1).
 * chunk_bytes 0 = 64 MiB. Blocking.
 */
typedef void (*tgpu_chunk_fn)(void* user, uint64_t r0, uint64_t r1);
int tgpu_decode_host_chunks(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                            const void* host_in, uint64_t in_len, uint64_t n_records,
                            void* host_records, void* host_arena, uint64_t arena_capacity,
                            const tgpu_limits* limits, uint64_t chunk_bytes,
                            tgpu_chunk_fn on_chunk, void* user, tgpu_status* st,
                            uint64_t* n_decoded, uint64_t* consumed);

/*
 * tgpu_decode_host_chunks with flags. TGPU_HOST_PACK_LISTS: for a schema
 * whose list arena holds only scalar list / set elements (a flat record
 * program: no containers of structs or of containers, no strings inside
 * containers), each finished range's element arrays are packed, in record
 * order, at the front of that range's arena slice and the records' spans
 * point there; only the records and the packed bytes are copied back (the
 * slice is as large as its wire bytes x arena scale, config 4's elements
 * 36 % of it). Span offsets then differ from tgpu_decode_host_ex's; the
 * values they describe do not. Other schemas ignore the flag. The IOBuf
 * batch API (GpuBatchSerializer::deserializeBatch) sets it.
 */
enum { TGPU_HOST_PACK_LISTS = 1 };
int tgpu_decode_host_chunks_ex(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                               const void* host_in, uint64_t in_len, uint64_t n_records,
                               void* host_records, void* host_arena, uint64_t arena_capacity,
                               const tgpu_limits* limits, uint64_t chunk_bytes, uint32_t flags,
                               tgpu_chunk_fn on_chunk, void* user, tgpu_status* st,
                               uint64_t* n_decoded, uint64_t* consumed);
/*
 * Encode: the caller's fill(user, r0, r1, &form) provides the device form of
 * records [r0, r1) (records, and the string / list bases their spans are
 * relative to: each chunk its own) just before the chunk is needed, so the
 * caller builds chunk k+1 on the host while the device encodes chunk k;
 * reserve(user, bytes) returns where a chunk's `bytes` wire bytes go (an
 * IOBufQueue::preallocate), written in record order. The buffers fill gives
 * must stay valid until the next-but-one fill call. chunk_records 0 = 1 Mi.
 * Status as tgpu_encode_batch (records relative to the batch; the wire of
 * the records before a failing one has been handed to reserve). Blocking.
 */
typedef struct tgpu_host_form {
  const void* records;
  const void* strings;
  uint64_t strings_len;
  const void* lists;
  uint64_t lists_len;
} tgpu_host_form;
typedef int (*tgpu_fill_fn)(void* user, uint64_t r0, uint64_t r1, tgpu_host_form* form);
typedef void* (*tgpu_reserve_fn)(void* user, uint64_t bytes);
int tgpu_encode_host_chunks(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                            uint64_t n_records, uint64_t chunk_records, tgpu_fill_fn fill,
                            tgpu_reserve_fn reserve, void* user, tgpu_status* st,
                            uint64_t* out_size);
/* The same, and landed(user, r0, r1, dst, bytes) once the wire of records
 * [r0, r1) has arrived at the `dst` reserve returned (in chunk order, on the
 * calling thread, before the call returns; every chunk whose wire reserve
 * took lands, also when a later one fails). A caller that reserves pinned
 * staging moves each chunk on from there while later chunks still encode. */
typedef void (*tgpu_landed_fn)(void* user, uint64_t r0, uint64_t r1, void* dst, uint64_t bytes);
int tgpu_encode_host_chunks_ex(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                               uint64_t n_records, uint64_t chunk_records, tgpu_fill_fn fill,
                               tgpu_reserve_fn reserve, tgpu_landed_fn landed, void* user,
                               tgpu_status* st, uint64_t* out_size);

/* Pinned (page-locked) host memory: staging for the host-memory entry
 * points' records, arenas and device forms that the PCIe copies read and
 * write without the runtime's bounce buffers or a per-call hipHostRegister
 * (the C++ batch API keeps its staging in it across calls). */
int tgpu_host_alloc(uint64_t bytes, void** out);
void tgpu_host_free(void* p);

/* Exact wire size of host-memory records (tgpu_encoded_size over host
 * buffers; host_out_offsets, n+1 entries, may be NULL): what an encode into
 * an IOBufQueue preallocates. Blocking. */
int tgpu_encoded_size_host(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                           const void* host_records, uint64_t n_records, const void* host_lists,
                           uint64_t lists_len, uint64_t* host_out_offsets, tgpu_status* st,
                           uint64_t* total);

/* ---- stream index ----------------------------------------------------- */
/*
 * Record index of an unindexed stream — the bulk form of the file-reading
 * loop `while (!cursor.isAtEnd()) deserialize<T>(cursor)` over back-to-back
 * records (thrift/lib/cpp2/protocol/Serializer.h:97-100): the start of every
 * record that begins in [begin, end) of in[0..in_len). Records may run past
 * `end` up to in_len (a shard's overlap with the next shard).
 *
 * begin must be a record boundary, unless `speculative` is set: then the first
 * record start at or after begin is discovered (*first_start) — one shard of
 * a file split by bytes, whose first boundary is confirmed by the previous
 * shard's *last_end (the only exchange between shards).
 *
 * offsets (device, max_records + 1 entries) receives the starts, then the end
 * of the last record. Errors: the first record the reader rejects ends the
 * index with that record's exact reference status (st->record = its index,
 * offsets[st->record] = its start); more than max_records records ->
 * TGPU_ERR_OUTPUT_OVERFLOW with *n_records = the number found; speculative
 * call with no record start in the first chunk -> TGPU_ERR_UNSUPPORTED.
 * Blocking when st != NULL (then n_records / first_start / last_end are filled).
 */
int tgpu_index_stream(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                      const void* in, uint64_t in_len, uint64_t begin, uint64_t end,
                      int speculative, uint64_t* offsets, uint64_t max_records,
                      const tgpu_limits* limits, void* stream, tgpu_status* st,
                      uint64_t* n_records, uint64_t* first_start, uint64_t* last_end);

/*
 * Index + decode in one pass: the records that begin in [begin, end) of an
 * unindexed stream (as tgpu_index_stream, incl. a speculative shard) are
 * decoded into records[0..n) while their starts are found — the whole file
 * loop `while (!cursor.isAtEnd()) deserialize<T>(cursor)`
 * (Serializer.h:97-100) over a byte range. offsets (max_records + 1) receives
 * the starts and the end as for tgpu_index_stream; list_arena as for
 * tgpu_decode_batch (capacity in_len Binary / 8 * in_len Compact). A record
 * the reader rejects ends the range with its status and is partially
 * decoded like the reference leaves it. Blocking when st != NULL.
 */
int tgpu_decode_stream(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                       const void* in, uint64_t in_len, uint64_t begin, uint64_t end,
                       int speculative, uint64_t* offsets, uint64_t max_records,
                       void* records, void* list_arena, uint64_t list_arena_capacity,
                       const tgpu_limits* limits, void* stream, tgpu_status* st,
                       uint64_t* n_records, uint64_t* first_start, uint64_t* last_end);

/*
 * Schemaless skim: one entry per top-level field of every record, in wire
 * order — the parse loop of protocol::parseObject
 * (thrift/lib/cpp2/protocol/detail/Object.h:416-432) with each value kept as
 * its encoded bytes instead of materialized, as the masked parse stores an
 * excluded field (setMaskedDataFull, detail/FieldMaskUtil.h:373-388:
 * wireType + the bytes apache::thrift::skip passes over). Bool fields are
 * read (parseValueWithMask, FieldMaskUtil.h:441-450): Compact carries the
 * value in the field header, so its encoded value is empty and the value is
 * in `flags`.
 *   offset  absolute byte position of the value in `in` (after the header)
 *   length  bytes of the value (what skip consumed); a value of 4 GiB or
 *           more does not fit and fails the record with TGPU_ERR_UNSUPPORTED
 *   flags   TGPU_SKIM_BOOL | (value ? TGPU_SKIM_TRUE : 0) for T_BOOL
 */
typedef struct tgpu_skim_field {
  int16_t id;
  uint8_t ttype; /* wire TType (Compact types mapped to TType) */
  uint8_t flags;
  uint32_t length;
  uint64_t offset;
} tgpu_skim_field;

enum { TGPU_SKIM_BOOL = 1, TGPU_SKIM_TRUE = 2 };
/* Nested skim (tgpu_skim_batch_ex): flags bits 2-5 hold the entry's struct
 * nesting level (0 = a top-level field). */
enum { TGPU_SKIM_LEVEL_SHIFT = 2, TGPU_SKIM_LEVEL_MASK = 0x3c, TGPU_SKIM_MAX_NEST = 8 };

/*
 * Skims records [0, n) of an indexed stream (offsets: device, n + 1 entries,
 * e.g. from tgpu_index_stream with a field-less schema). fields (device,
 * 16-byte aligned, max_fields * n_records entries) is field-major: the k-th field of record i
 * is fields[k * n_records + i] (so a wavefront's k-th stores are contiguous);
 * field_counts[i] (device) receives the record's total number of fields —
 * fields past max_fields are counted but not stored, slots past the count
 * are left untouched. Errors as tgpu_decode_batch: the first record (in record order)
 * the reader rejects, or whose end disagrees with offsets[i + 1]
 * (TGPU_ERR_INDEX_MISMATCH), is reported with the reference's status; n_done
 * = records before it. Blocking when st != NULL.
 */
int tgpu_skim_batch(tgpu_context* ctx, int protocol, const void* in, uint64_t in_len,
                    const uint64_t* offsets, uint64_t n_records, tgpu_skim_field* fields,
                    uint32_t max_fields, uint32_t* field_counts, const tgpu_limits* limits,
                    void* stream, tgpu_status* st, uint64_t* n_done);
/*
 * The same, descending into struct-valued fields up to max_nest levels
 * (<= TGPU_SKIM_MAX_NEST; 0 = tgpu_skim_batch): parseObject's recursion
 * (parseValue -> parseObjectInplace, protocol/detail/Object.h:416-432) with
 * every other value kept as its encoded bytes. Entries are in pre-order (wire
 * order of the field headers): a descended struct's entry (ttype T_STRUCT,
 * offset / length of its whole encoded value, as a skip passes over it)
 * precedes its fields' entries, which carry level + 1 in flags. Depth and
 * height are checked as apache::thrift::skip would for the same struct
 * (Protocol.h:187-283: max_depth per nesting level, readStructBegin's
 * descend). field_counts count every entry, nested ones included.
 */
int tgpu_skim_batch_ex(tgpu_context* ctx, int protocol, const void* in, uint64_t in_len,
                       const uint64_t* offsets, uint64_t n_records, tgpu_skim_field* fields,
                       uint32_t max_fields, uint32_t* field_counts, uint32_t max_nest,
                       const tgpu_limits* limits, void* stream, tgpu_status* st,
                       uint64_t* n_done);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* THRIFT_GPU_H_ */
