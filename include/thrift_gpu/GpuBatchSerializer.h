/*
 * GpuBatchSerializer.h — C++ host mirror of fbthrift's
 * apache::thrift::Serializer<Reader, Writer> (thrift/lib/cpp2/protocol/
 * Serializer.h:34-224) for whole batches of same-schema records, on top of
 * the C-ABI in thrift_gpu.h. Header-only; links against libtgpu.so and the
 * HIP runtime.
 *
 *   using BinaryBatch  = GpuBatchSerializer<BinaryProtocol>;   // T_BINARY_PROTOCOL
 *   using CompactBatch = GpuBatchSerializer<CompactProtocol>;  // T_COMPACT_PROTOCOL
 *
 *   BinaryBatch ser(schema);                        // schema: GpuSchema
 *   size_t bytes = ser.serialize(d_records, n, d_out, cap, d_offsets);
 *   size_t used  = ser.deserialize(d_in, len, n, d_records);  // throws like
 *                                                            // deserialize<T>
 *
 * Errors are rethrown with the reference's exception types: a
 * TProtocolException carrying the reference's TProtocolExceptionType, or
 * std::out_of_range; a bool byte > 1 on write calls std::abort() exactly like
 * validate_bool's LOG(FATAL) (thrift/lib/cpp2/protocol/Protocol.h:126-163)
 * unless THRIFT_GPU_NO_ABORT is defined (then it throws std::logic_error).
 *
 * With THRIFT_GPU_WITH_FBTHRIFT defined (building inside an fbthrift tree),
 * the exception type is apache::thrift::protocol::TProtocolException itself
 * and the protocol tags are the real BinaryProtocolReader/Writer types.
 */
#ifndef THRIFT_GPU_GPU_BATCH_SERIALIZER_H_
#define THRIFT_GPU_GPU_BATCH_SERIALIZER_H_

#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../thrift_gpu.h"

#ifdef THRIFT_GPU_WITH_FBTHRIFT
#include <thrift/lib/cpp/protocol/TProtocolException.h>
#include <thrift/lib/cpp2/protocol/BinaryProtocol.h>
#include <thrift/lib/cpp2/protocol/CompactProtocol.h>
#endif

namespace apache::thrift::gpu {

#ifdef THRIFT_GPU_WITH_FBTHRIFT
using TProtocolException = apache::thrift::protocol::TProtocolException;
inline TProtocolException makeProtocolException(int type, const std::string& what) {
  return TProtocolException(
      static_cast<TProtocolException::TProtocolExceptionType>(type), what);
}
struct BinaryProtocol {
  using ProtocolReader = apache::thrift::BinaryProtocolReader;
  using ProtocolWriter = apache::thrift::BinaryProtocolWriter;
  static constexpr int kId = TGPU_PROTOCOL_BINARY;
};
struct CompactProtocol {
  using ProtocolReader = apache::thrift::CompactProtocolReader;
  using ProtocolWriter = apache::thrift::CompactProtocolWriter;
  static constexpr int kId = TGPU_PROTOCOL_COMPACT;
};
struct CompactV1Protocol {
  using ProtocolReader = apache::thrift::CompactV1ProtocolReader;
  using ProtocolWriter = apache::thrift::CompactV1ProtocolWriter;
  static constexpr int kId = TGPU_PROTOCOL_COMPACT_V1;
};
#else
/* Same type codes as thrift/lib/cpp/protocol/TProtocolException.h:41-51. */
class TProtocolException : public std::runtime_error {
 public:
  enum TProtocolExceptionType {
    UNKNOWN = 0,
    INVALID_DATA = 1,
    NEGATIVE_SIZE = 2,
    SIZE_LIMIT = 3,
    BAD_VERSION = 4,
    NOT_IMPLEMENTED = 5,
    MISSING_REQUIRED_FIELD = 6,
    CHECKSUM_MISMATCH = 7,
    DEPTH_LIMIT = 8,
  };
  TProtocolException(TProtocolExceptionType t, const std::string& what)
      : std::runtime_error(what), type_(t) {}
  TProtocolExceptionType getType() const { return type_; }

 private:
  TProtocolExceptionType type_;
};
inline TProtocolException makeProtocolException(int type, const std::string& what) {
  return TProtocolException(static_cast<TProtocolException::TProtocolExceptionType>(type), what);
}
/* protocolType() values: thrift/lib/cpp/protocol/TProtocolTypes.h:24-27. */
struct BinaryProtocol {
  static constexpr int kId = TGPU_PROTOCOL_BINARY;
};
struct CompactProtocol {
  static constexpr int kId = TGPU_PROTOCOL_COMPACT;
};
struct CompactV1Protocol {  /* CompactV1Protocol.h: doubles little-endian */
  static constexpr int kId = TGPU_PROTOCOL_COMPACT_V1;
};
#endif

/* tgpu runtime failure (HIP error, bad argument, capacity) — no reference
 * counterpart. */
class GpuBatchError : public std::runtime_error {
 public:
  GpuBatchError(const tgpu_status& st, const std::string& what)
      : std::runtime_error(what), status_(st) {}
  const tgpu_status& status() const { return status_; }

 private:
  tgpu_status status_;
};

/* Throws the exception the reference would have thrown for `st`. */
[[noreturn]] inline void rethrow(const tgpu_status& st) {
  const std::string what = std::string(tgpu_code_name(st.code)) + " at record " +
                           std::to_string(st.record) + ", byte " +
                           std::to_string(st.byte_offset);
  switch (st.exc_class) {
    case TGPU_EXC_OUT_OF_RANGE:
      throw std::out_of_range(st.code == TGPU_ERR_INVALID_VARINT ? "invalid varint read" : what);
    case TGPU_EXC_PROTOCOL:
      throw makeProtocolException(st.tproto_type, what);
    case TGPU_EXC_ABORT:
#ifdef THRIFT_GPU_NO_ABORT
      throw std::logic_error("invalid bool value: " + what);
#else
      std::abort();
#endif
    default:
      throw GpuBatchError(st, what);
  }
}

inline void check(int rc, const char* what) {
  if (rc != TGPU_OK) {
    tgpu_status st{};
    st.code = rc;
    tgpu_code_classify(rc, &st.exc_class, &st.tproto_type);
    throw GpuBatchError(st, std::string(what) + ": " + tgpu_code_name(rc));
  }
}

/* A field of a runtime schema (the StructInfo/FieldInfo analog). */
struct FieldSpec {
  int16_t id;
  uint8_t ttype;
  uint8_t elem_ttype = 0;  /* list/set element, map key */
  bool optional = false;
  int32_t struct_index = -1;
  uint8_t val_ttype = 0;   /* map value */
  uint8_t qualifier = 0;   /* TGPU_TERSE etc.; `optional` wins when set */
};

/* Owns a tgpu_schema. Structs are given as lists of FieldSpec (struct 0 =
 * record); the layout is computed by tgpu_layout_compute so it matches a
 * codegen'd struct with the same members (declaration order, natural
 * alignment, trailing isset bytes; strings/lists as tgpu_span). */
class GpuSchema {
 public:
  /* unions[i] marks struct i as a Thrift union (may be shorter than structs). */
  explicit GpuSchema(const std::vector<std::vector<FieldSpec>>& structs,
                     const std::vector<bool>& unions = {}) {
    for (size_t i = 0; i < structs.size(); ++i) {
      const auto& s = structs[i];
      tgpu_struct_desc d{};
      d.first_field = static_cast<uint32_t>(fields_.size());
      d.num_fields = static_cast<uint32_t>(s.size());
      d.flags = (i < unions.size() && unions[i]) ? TGPU_STRUCT_UNION : 0u;
      structs_.push_back(d);
      for (const FieldSpec& f : s) {
        tgpu_field_desc fd{};
        fd.id = f.id;
        fd.ttype = f.ttype;
        fd.elem_ttype = f.elem_ttype;
        fd.val_ttype = f.val_ttype;
        fd.qualifier = f.optional ? TGPU_OPTIONAL : f.qualifier;
        fd.struct_index = f.struct_index;
        fields_.push_back(fd);
      }
    }
    check(tgpu_layout_compute(structs_.data(), (uint32_t)structs_.size(), fields_.data(),
                              (uint32_t)fields_.size()),
          "tgpu_layout_compute");
    check(tgpu_schema_create(structs_.data(), (uint32_t)structs_.size(), fields_.data(),
                             (uint32_t)fields_.size(), &schema_),
          "tgpu_schema_create");
  }
  ~GpuSchema() { tgpu_schema_destroy(schema_); }
  GpuSchema(const GpuSchema&) = delete;
  GpuSchema& operator=(const GpuSchema&) = delete;

  const tgpu_schema* get() const { return schema_; }
  uint32_t recordSize() const { return structs_[0].size; }
  uint32_t memberOffset(uint32_t struct_index, uint32_t k) const {
    return fields_[structs_[struct_index].first_field + k].member_offset;
  }
  uint32_t issetOffset(uint32_t struct_index, uint32_t k) const {
    return fields_[structs_[struct_index].first_field + k].isset_offset;
  }

 private:
  std::vector<tgpu_struct_desc> structs_;
  std::vector<tgpu_field_desc> fields_;
  tgpu_schema* schema_ = nullptr;
};

/*
 * Serializer<Reader, Writer> for batches. Like the reference's reader/writer
 * objects, an instance is single-threaded (it owns one workspace); the static
 * reference entry points map to one instance per thread.
 */
template <class Protocol>
class GpuBatchSerializer {
 public:
  explicit GpuBatchSerializer(const GpuSchema& schema, void* stream = nullptr)
      : schema_(schema), stream_(stream) {
    check(tgpu_context_create(&ctx_), "tgpu_context_create");
  }
  ~GpuBatchSerializer() { tgpu_context_destroy(ctx_); }
  GpuBatchSerializer(const GpuBatchSerializer&) = delete;
  GpuBatchSerializer& operator=(const GpuBatchSerializer&) = delete;

  static constexpr int protocolType() { return Protocol::kId; }

  /* Limits = gflags thrift_cpp2_protocol_reader_{string,container}_limit and
   * thrift_protocol_max_depth (defaults 0, 0, 12000). */
  void setLimits(int32_t string_limit, int32_t container_limit, int32_t max_depth = 12000) {
    limits_ = tgpu_limits{string_limit, container_limit, max_depth, 0};
  }
  void setHeight(int32_t height) { limits_.height = height; }
  void reserve(uint64_t n_records) { check(tgpu_context_reserve(ctx_, n_records), "reserve"); }

  /* N x serialize(obj, &queue): returns bytes written to out (device). */
  uint64_t serialize(const void* records, uint64_t n, void* out, uint64_t capacity,
                     uint64_t* offsets = nullptr, const void* string_base = nullptr,
                     const void* list_base = nullptr) {
    tgpu_status st{};
    uint64_t size = 0;
    tgpu_encode_batch(ctx_, schema_.get(), Protocol::kId, records, n, string_base, list_base, out,
                      capacity, offsets, stream_, &st, &size);
    if (st.code != TGPU_OK) rethrow(st);
    return size;
  }

  /* Exact serialized size of each record (serializedSize analog). */
  uint64_t serializedSize(const void* records, uint64_t n, uint64_t* offsets,
                          const void* list_base = nullptr) {
    tgpu_status st{};
    uint64_t total = 0;
    tgpu_encoded_size(ctx_, schema_.get(), Protocol::kId, records, n, list_base, offsets, stream_,
                      &st, &total);
    if (st.code != TGPU_OK) rethrow(st);
    return total;
  }

  /* N x deserialize<T>(Cursor&): returns bytes consumed; throws on the first
   * failing record (records before it are fully decoded). */
  uint64_t deserialize(const void* in, uint64_t len, uint64_t n, void* records,
                       const uint64_t* offsets = nullptr, void* list_arena = nullptr,
                       uint64_t list_arena_capacity = 0) {
    tgpu_status st{};
    uint64_t done = 0, consumed = 0;
    tgpu_decode_batch(ctx_, schema_.get(), Protocol::kId, in, len, offsets, n, records,
                      list_arena, list_arena_capacity, &limits_, stream_, &st, &done, &consumed);
    if (st.code != TGPU_OK) rethrow(st);
    return consumed;
  }

  /* Host-memory forms (the reference's callers hold IOBuf / host objects,
   * Serializer.h:62-72,136-148): records and bytes stay in host memory and
   * are pipelined through the GPU in chunks (tgpu_decode_host /
   * tgpu_encode_host; fixed-length Binary record schemas). */
  uint64_t deserializeHost(const void* in, uint64_t len, uint64_t n, void* records,
                           uint64_t chunk_records = 0) {
    tgpu_status st{};
    uint64_t done = 0, consumed = 0;
    tgpu_decode_host(ctx_, schema_.get(), Protocol::kId, in, len, n, records, chunk_records,
                     &limits_, &st, &done, &consumed);
    if (st.code != TGPU_OK) rethrow(st);
    return consumed;
  }
  uint64_t serializeHost(const void* records, uint64_t n, void* out, uint64_t capacity,
                         uint64_t chunk_records = 0) {
    tgpu_status st{};
    uint64_t size = 0;
    tgpu_encode_host(ctx_, schema_.get(), Protocol::kId, records, n, out, capacity,
                     chunk_records, &st, &size);
    if (st.code != TGPU_OK) rethrow(st);
    return size;
  }
  /* Host-memory forms for any schema (tgpu_decode_host_ex /
   * tgpu_encode_host_ex): one resident pass through the GPU. */
  uint64_t deserializeHostEx(const void* in, uint64_t len, uint64_t n, void* records,
                             void* arena = nullptr, uint64_t arena_capacity = 0) {
    tgpu_status st{};
    uint64_t done = 0, consumed = 0;
    tgpu_decode_host_ex(ctx_, schema_.get(), Protocol::kId, in, len, n, records, arena,
                        arena_capacity, &limits_, &st, &done, &consumed);
    if (st.code != TGPU_OK) rethrow(st);
    return consumed;
  }
  uint64_t serializeHostEx(const void* records, uint64_t n, const void* strings,
                           uint64_t strings_len, const void* lists, uint64_t lists_len,
                           void* out, uint64_t capacity, uint64_t* out_offsets = nullptr) {
    tgpu_status st{};
    uint64_t size = 0;
    tgpu_encode_host_ex(ctx_, schema_.get(), Protocol::kId, records, n, strings, strings_len,
                        lists, lists_len, out, capacity, out_offsets, &st, &size);
    if (st.code != TGPU_OK) rethrow(st);
    return size;
  }

  /* Re-encodes n records of `in` (this serializer's protocol) into protocol
   * To (tgpu_transcode_batch): serialize<To>(deserialize<From>(record)) per
   * record without leaving the device. Returns the output size; throws on
   * the first record the reader rejects (records before it are written). */
  template <class To>
  uint64_t transcode(const void* in, uint64_t len, uint64_t n, void* out, uint64_t capacity,
                     uint64_t* out_offsets = nullptr, const uint64_t* offsets = nullptr) {
    tgpu_status st{};
    uint64_t done = 0, size = 0;
    tgpu_transcode_batch(ctx_, schema_.get(), Protocol::kId, To::kId, in, len, offsets, n, out,
                         capacity, out_offsets, &limits_, stream_, &st, &done, &size);
    if (st.code != TGPU_OK) rethrow(st);
    return size;
  }
  /* Schemaless skim of n indexed records (tgpu_skim_batch): the field loop
   * of protocol::parseObject with every value kept as its encoded bytes
   * (protocol/detail/FieldMaskUtil.h:373-388). fields: max_fields * n
   * entries, field-major (fields[k * n + i] = field k of record i); counts:
   * n. Device pointers. Throws on the first record the reader rejects. */
  void skim(const void* in, uint64_t len, const uint64_t* offsets, uint64_t n,
            tgpu_skim_field* fields, uint32_t max_fields, uint32_t* counts) {
    tgpu_status st{};
    uint64_t done = 0;
    tgpu_skim_batch(ctx_, Protocol::kId, in, len, offsets, n, fields, max_fields, counts,
                    &limits_, stream_, &st, &done);
    if (st.code != TGPU_OK) rethrow(st);
  }
  /* List arena bytes deserialize() needs for `len` input bytes. */
  uint64_t arenaBytes(uint64_t len) const {
    return len * tgpu_schema_arena_scale(schema_.get(), Protocol::kId);
  }

  /* Generates and compiles the schema's kernels now (tgpu_schema_compile):
   * the run-time counterpart of thrift1 emitting T::readNoXfer / T::write.
   * False when the schema runs on the interpreting kernels instead. */
  bool compile() { return tgpu_schema_compile(schema_.get(), Protocol::kId) == TGPU_OK; }

  /* Asynchronous forms: enqueue on the stream; collect with wait(). */
  void serializeAsync(const void* records, uint64_t n, void* out, uint64_t capacity,
                      uint64_t* offsets = nullptr, const void* string_base = nullptr,
                      const void* list_base = nullptr) {
    check(tgpu_encode_batch(ctx_, schema_.get(), Protocol::kId, records, n, string_base,
                            list_base, out, capacity, offsets, stream_, nullptr, nullptr),
          "tgpu_encode_batch");
  }
  void deserializeAsync(const void* in, uint64_t len, uint64_t n, void* records,
                        const uint64_t* offsets = nullptr, void* list_arena = nullptr,
                        uint64_t list_arena_capacity = 0) {
    check(tgpu_decode_batch(ctx_, schema_.get(), Protocol::kId, in, len, offsets, n, records,
                            list_arena, list_arena_capacity, &limits_, stream_, nullptr, nullptr,
                            nullptr),
          "tgpu_decode_batch");
  }
  /* Waits for the last async call; returns (records done, bytes). */
  std::pair<uint64_t, uint64_t> wait() {
    tgpu_status st{};
    uint64_t done = 0, bytes = 0;
    tgpu_context_wait(ctx_, stream_, &st, &done, &bytes);
    if (st.code != TGPU_OK) rethrow(st);
    return {done, bytes};
  }

 private:
  const GpuSchema& schema_;
  void* stream_;
  tgpu_context* ctx_ = nullptr;
  tgpu_limits limits_{0, 0, 12000, 0};
};

using BinaryBatchSerializer = GpuBatchSerializer<BinaryProtocol>;
using CompactBatchSerializer = GpuBatchSerializer<CompactProtocol>;
using CompactV1BatchSerializer = GpuBatchSerializer<CompactV1Protocol>;

}  // namespace apache::thrift::gpu

#endif  // THRIFT_GPU_GPU_BATCH_SERIALIZER_H_
