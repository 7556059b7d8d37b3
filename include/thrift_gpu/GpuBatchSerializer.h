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

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>
#include <condition_variable>
#include <mutex>
#include <thread>

#include <memory>

#include "../thrift_gpu.h"
#include "HostBinding.h"

#ifdef THRIFT_GPU_WITH_FBTHRIFT
#include <folly/io/IOBuf.h>
#include <folly/io/IOBufQueue.h>
#include <thrift/lib/cpp/protocol/TProtocolException.h>
#include <thrift/lib/cpp2/protocol/BinaryProtocol.h>
#include <thrift/lib/cpp2/protocol/CompactProtocol.h>
#include <thrift/lib/cpp2/protocol/CompactV1Protocol.h>
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

#ifdef THRIFT_GPU_WITH_FBTHRIFT
using IOBuf = folly::IOBuf;
using IOBufQueue = folly::IOBufQueue;
#else
/* Header-free stand-ins for the folly::IOBuf / IOBufQueue subset the batch
 * entry points use (the reference's serialize / deserialize take and fill
 * these, Serializer.h:62-72,136-148): a circular chain of byte buffers with
 * data() / length() / next() / prependChain(), and a queue that appends
 * through preallocate() / postallocate() and hands its chain over with
 * move(). The batch code is written against this subset only, so the same
 * templates instantiate with folly's types. */
class IOBuf {
 public:
  static std::unique_ptr<IOBuf> copyBuffer(const void* p, size_t n) {
    std::unique_ptr<IOBuf> b = create(n);
    if (n) std::memcpy(b->buf_.get(), p, n);
    b->length_ = n;
    return b;
  }
  /* An empty buffer of `capacity` bytes (not initialized, like folly's). */
  static std::unique_ptr<IOBuf> create(size_t capacity) {
    std::unique_ptr<IOBuf> b(new IOBuf());
    b->buf_.reset(new uint8_t[capacity ? capacity : 1]);
    b->capacity_ = capacity;
    return b;
  }
  ~IOBuf() {
    // a chain owns its other buffers (the head is owned by its holder)
    if (next_ != this) {
      IOBuf* p = next_;
      prev_->next_ = nullptr;
      while (p) {
        IOBuf* q = p->next_;
        p->next_ = p->prev_ = p;
        delete p;
        p = q;
      }
    }
  }
  const uint8_t* data() const { return buf_.get(); }
  uint8_t* writableData() { return buf_.get(); }
  size_t length() const { return length_; }
  size_t capacity() const { return capacity_; }
  /* Grows / shrinks the data length within the capacity. */
  void setLength(size_t n) { length_ = n < capacity_ ? n : capacity_; }
  IOBuf* next() { return next_; }
  const IOBuf* next() const { return next_; }
  bool isChained() const { return next_ != this; }
  /* Appends `other` (a chain) at the end of this chain. */
  void prependChain(std::unique_ptr<IOBuf> other) {
    IOBuf* o = other.release();
    IOBuf* otail = o->prev_;
    IOBuf* tail = prev_;
    tail->next_ = o;
    o->prev_ = tail;
    otail->next_ = this;
    prev_ = otail;
  }
  size_t computeChainDataLength() const {
    size_t n = 0;
    const IOBuf* b = this;
    do {
      n += b->length();
      b = b->next_;
    } while (b != this);
    return n;
  }

 private:
  IOBuf() : next_(this), prev_(this) {}
  std::unique_ptr<uint8_t[]> buf_;
  size_t length_ = 0, capacity_ = 0;
  IOBuf* next_;
  IOBuf* prev_;
};

class IOBufQueue {
 public:
  /* Writable space of at least `min` bytes at the end of the queue. */
  std::pair<void*, size_t> preallocate(size_t min, size_t newAllocationSize) {
    pending_ = IOBuf::create(std::max(min, newAllocationSize));
    return {pending_->writableData(), pending_->capacity()};
  }
  /* Commits n bytes of the last preallocate(). */
  void postallocate(size_t n) {
    pending_->setLength(n);
    if (!head_) head_ = std::move(pending_);
    else head_->prependChain(std::move(pending_));
  }
  size_t chainLength() const { return head_ ? head_->computeChainDataLength() : 0; }
  std::unique_ptr<IOBuf> move() { return std::move(head_); }
  const IOBuf* front() const { return head_.get(); }

 private:
  std::unique_ptr<IOBuf> head_, pending_;
};
#endif

/* Bytes of an IOBuf chain, in order (the bytes a Cursor over it reads). */
template <class Buf>
std::vector<uint8_t> coalesced(const Buf* head) {
  std::vector<uint8_t> out;
  if (!head) return out;
  out.reserve(head->computeChainDataLength());
  const Buf* b = head;
  do {
    out.insert(out.end(), b->data(), b->data() + b->length());
    b = b->next();
  } while (b != head);
  return out;
}

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
  uint8_t qualifier = 0;   /* TGPU_TERSE, TGPU_BOXED etc.; `optional` wins when set */
  uint32_t type_index = 0; /* 1 + nested container type (tgpu_type_desc) */
  uint16_t key_index = 0;  /* map: 1 + type node of a struct / container key */
};

/* Owns a tgpu_schema. Structs are given as lists of FieldSpec (struct 0 =
 * record); the layout is computed by tgpu_layout_compute so it matches a
 * codegen'd struct with the same members (declaration order, natural
 * alignment, trailing isset bytes; strings/lists as tgpu_span). */
class GpuSchema {
 public:
  /* unions[i] marks struct i as a Thrift union (may be shorter than structs);
     flags[i] adds tgpu_struct_flags (e.g. TGPU_STRUCT_ENFORCE_REQUIRED);
     types: nested container types referenced by FieldSpec::type_index. */
  explicit GpuSchema(const std::vector<std::vector<FieldSpec>>& structs,
                     const std::vector<bool>& unions = {},
                     const std::vector<tgpu_type_desc>& types = {},
                     const std::vector<uint32_t>& flags = {})
      : types_(types) {
    for (size_t i = 0; i < structs.size(); ++i) {
      const auto& s = structs[i];
      tgpu_struct_desc d{};
      d.first_field = static_cast<uint32_t>(fields_.size());
      d.num_fields = static_cast<uint32_t>(s.size());
      d.flags = (i < unions.size() && unions[i]) ? TGPU_STRUCT_UNION : 0u;
      if (i < flags.size()) d.flags |= flags[i];
      structs_.push_back(d);
      for (const FieldSpec& f : s) {
        tgpu_field_desc fd{};
        fd.id = f.id;
        fd.ttype = f.ttype;
        fd.elem_ttype = f.elem_ttype;
        fd.val_ttype = f.val_ttype;
        fd.qualifier = f.optional ? TGPU_OPTIONAL : f.qualifier;
        fd.struct_index = f.struct_index;
        fd.type_index = f.type_index;
        fd.key_index = f.key_index;
        fields_.push_back(fd);
      }
    }
    check(tgpu_layout_compute(structs_.data(), (uint32_t)structs_.size(), fields_.data(),
                              (uint32_t)fields_.size()),
          "tgpu_layout_compute");
    check(tgpu_schema_create_ex(structs_.data(), (uint32_t)structs_.size(), fields_.data(),
                                (uint32_t)fields_.size(), types_.data(),
                                (uint32_t)types_.size(), &schema_),
          "tgpu_schema_create_ex");
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
  SchemaTables tables() const { return SchemaTables{structs_.data(), fields_.data(), types_.data()}; }

 private:
  std::vector<tgpu_type_desc> types_;
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

  /* deserialize over an IOBuf chain into codegen'd objects: N x
   * Serializer::deserialize<T>(Cursor&) (Serializer.h:62-72,97-100) with the
   * records materialized into T (std::string / std::vector members filled
   * with COPY semantics, Protocol.h:406-454) through `binding`. out[0..n)
   * are default-constructed T. Returns bytes consumed; throws like the
   * reference on the first failing record, the records before it set (the
   * failing one partially, as the reference leaves it); an exception a
   * binding hook throws reaches the caller too.
   * The device pass is chunk-pipelined (tgpu_decode_host_chunks) into this
   * serializer's pinned staging; every finished range of records is cut into
   * blocks that the host pool's materialize_threads() workers turn into
   * objects while later chunks cross PCIe and decode. */
  template <class T>
  uint64_t deserializeBatch(const IOBuf* buf, T* out, uint64_t n, const HostStruct& binding) {
    const uint8_t* in = nullptr;
    uint64_t len = 0;
    if (buf && !buf->isChained()) {
      in = buf->data();
      len = buf->length();
    } else if (buf) {  // a chain: its bytes in order, into pinned staging
      len = buf->computeChainDataLength();
      uint8_t* dst = in_.get(len + 16);
      const IOBuf* b = buf;
      uint64_t at = 0;
      do {
        std::memcpy(dst + at, b->data(), b->length());
        at += b->length();
        b = b->next();
      } while (b != buf);
      in = dst;
    }
    const uint32_t S = schema_.recordSize();
    uint8_t* recs = recs_.get(n * S + 16);
    const uint64_t acap = len * tgpu_schema_arena_scale(schema_.get(), Protocol::kId);
    uint8_t* arena = acap ? arena_.get(acap + 16) : nullptr;
    struct Feed {
      HostPool::Group g;
      SchemaTables tables;
      const uint8_t *recs, *in, *arena;
      uint32_t S;
      const HostStruct* binding;
      T* out;
    } feed{{}, schema_.tables(), recs, in, arena, S, &binding, out};
    auto on_chunk = [](void* u, uint64_t r0, uint64_t r1) {
      Feed& f = *static_cast<Feed*>(u);
      materializeAsync(f.g, f.tables, f.recs, r0, r1, f.S, f.in, f.arena, *f.binding, f.out,
                       sizeof(T));
    };
    tgpu_status st{};
    uint64_t done = 0, consumed = 0;
    // (list elements packed at each range's arena slice: only the records and
    // the elements cross PCIe back; the binding reads through the spans)
    tgpu_decode_host_chunks_ex(ctx_, schema_.get(), Protocol::kId, in, len, n, recs, arena, acap,
                               &limits_, decodeChunkBytes(len), TGPU_HOST_PACK_LISTS, on_chunk,
                               &feed, &st, &done, &consumed);
    feed.g.wait();  // every announced record materialized (or a hook's exception)
    if (st.code != TGPU_OK) rethrow(st);
    return consumed;
  }

  /* serialize of codegen'd objects appended to an IOBufQueue: N x
   * Serializer::serialize(obj, &queue) (Serializer.h:136-148). Chunk-
   * pipelined (tgpu_encode_host_chunks): while the device encodes chunk k,
   * a producer builds chunk k+1's device form in this serializer's pinned
   * slots (parts of the chunk sized, then written at their bases, on the host
   * pool's threads), and each chunk's wire lands in a preallocate() of its
   * exact size. Returns the bytes appended. */
  template <class T>
  uint64_t serializeBatch(const T* in, uint64_t n, const HostStruct& binding, IOBufQueue* out) {
    const uint64_t K = chunk_records_ ? chunk_records_ : (1ull << 20);  // records per chunk
    const uint64_t nch = (n + K - 1) / K;
    // three slots: chunk k is built into slot k % 3 once the library took
    // chunk k - 1 (fill(k - 1)): it then holds chunks k - 1 and k - 2 only
    // (the buffers of a fill stay in use until the next-but-one fill)
    struct Ctx {
      const T* in;
      const HostStruct* binding;
      SchemaTables tables;
      uint32_t S;
      uint64_t n, nch, K;
      FormSlot* slot;
      uint64_t built = 0, taken = 0;  // chunks built / handed to the library
      std::mutex mu;
      std::condition_variable cv;
      bool stop = false, failed = false;
      std::exception_ptr err;
      IOBufQueue* out;
      // the wire: each chunk's D2H lands in pinned staging (slot k % 3),
      // then the pool copies it into the queue's preallocated space
      WireStage* stage;
      uint64_t reserved = 0;
      std::vector<uint8_t*> dst;  // queue space of chunk k
      double t_build = 0, t_fill = 0, t_reserve = 0;  // TGPU_HOST_TIMING (seconds)
    } c{in, &binding, schema_.tables(), schema_.recordSize(), n, nch, K, slots_,
        0, 0, {}, {}, false, false, nullptr, out, wire_, 0, {}};
    using Clk = std::chrono::steady_clock;
    auto secs = [](Clk::time_point t) {
      return std::chrono::duration<double>(Clk::now() - t).count();
    };
    const auto t_call = Clk::now();
    std::thread producer([&c] {
      try {
        for (uint64_t k = 0; k < c.nch; ++k) {
          {
            std::unique_lock<std::mutex> lk(c.mu);
            c.cv.wait(lk, [&] { return c.stop || c.taken >= k; });
            if (c.stop) return;
          }
          const uint64_t r0 = k * c.K, r1 = std::min(c.n, r0 + c.K);
          const auto t0 = Clk::now();
          c.slot[k % 3].build(c.tables, c.S, c.in, r0, r1, sizeof(T), *c.binding);
          c.t_build += std::chrono::duration<double>(Clk::now() - t0).count();
          {
            std::lock_guard<std::mutex> lk(c.mu);
            c.built = k + 1;
          }
          c.cv.notify_all();
        }
      } catch (...) {
        std::lock_guard<std::mutex> lk(c.mu);
        c.err = std::current_exception();
        c.failed = true;
        c.cv.notify_all();
      }
    });
    auto fill = [](void* u, uint64_t r0, uint64_t, tgpu_host_form* f) -> int {
      Ctx& x = *static_cast<Ctx*>(u);
      const uint64_t k = r0 / x.K;
      const auto t0 = std::chrono::steady_clock::now();
      std::unique_lock<std::mutex> lk(x.mu);
      x.cv.wait(lk, [&] { return x.built > k || x.failed; });
      x.t_fill += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (x.built <= k) return -1;
      x.taken = k + 1;
      lk.unlock();
      x.cv.notify_all();
      const FormSlot& d = x.slot[k % 3];
      f->records = d.rec.data();
      f->strings = d.str.data();
      f->strings_len = d.slen;
      f->lists = d.lst.data();
      f->lists_len = d.llen;
      return 0;
    };
    auto reserve = [](void* u, uint64_t bytes) -> void* {
      Ctx& x = *static_cast<Ctx*>(u);
      const auto t0 = std::chrono::steady_clock::now();
      auto space = x.out->preallocate(bytes, bytes);
      x.out->postallocate(bytes);  // filled before serializeBatch returns
      x.dst.push_back(static_cast<uint8_t*>(space.first));
      WireStage& w = x.stage[x.reserved++ % 3];
      w.copies.wait();  // its previous chunk has left the staging
      uint8_t* p = w.buf.get(bytes + 16);
      x.t_reserve += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      return p;
    };
    auto landed = [](void* u, uint64_t r0, uint64_t, void* src, uint64_t bytes) {
      Ctx& x = *static_cast<Ctx*>(u);
      const uint64_t k = r0 / x.K;
      uint8_t* d = x.dst[k];
      const uint8_t* sp = static_cast<const uint8_t*>(src);
      constexpr uint64_t kPiece = 4ull << 20;  // (first touch of the queue's pages too)
      for (uint64_t a = 0; a < bytes; a += kPiece) {
        const uint64_t m = std::min(kPiece, bytes - a);
        x.stage[k % 3].copies.run([=] { std::memcpy(d + a, sp + a, m); });
      }
    };
    tgpu_status st{};
    uint64_t size = 0;
    tgpu_encode_host_chunks_ex(ctx_, schema_.get(), Protocol::kId, n, K, fill, reserve, landed,
                               &c, &st, &size);
    {
      std::lock_guard<std::mutex> lk(c.mu);
      c.stop = true;
    }
    c.cv.notify_all();
    producer.join();
    for (int k = 0; k < 3; ++k) wire_[k].copies.wait();
    if (std::getenv("TGPU_HOST_TIMING"))
      std::fprintf(stderr,
                   "serializeBatch: %.3f ms total, build %.3f ms (producer), fill wait %.3f ms, "
                   "reserve %.3f ms, %llu chunks\n",
                   secs(t_call) * 1e3, c.t_build * 1e3, c.t_fill * 1e3, c.t_reserve * 1e3,
                   (unsigned long long)nch);
    if (c.err) std::rethrow_exception(c.err);
    if (st.code != TGPU_OK) rethrow(st);
    return size;
  }

  /* Records per serializeBatch chunk (0 = 1 Mi) and wire bytes per
   * deserializeBatch piece (0 = 1/24 of the batch, 4-64 MiB). */
  void setChunkRecords(uint64_t k) { chunk_records_ = k; }
  void setChunkBytes(uint64_t b) { chunk_bytes_ = b; }

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
   * n. Device pointers. Throws on the first record the reader rejects.
   * nest > 0: the fields of struct-valued fields too, that many levels down
   * (parseObject's recursion; pre-order, the level in flags bits 2-5;
   * tgpu_skim_batch_ex). */
  void skim(const void* in, uint64_t len, const uint64_t* offsets, uint64_t n,
            tgpu_skim_field* fields, uint32_t max_fields, uint32_t* counts, uint32_t nest = 0) {
    tgpu_status st{};
    uint64_t done = 0;
    tgpu_skim_batch_ex(ctx_, Protocol::kId, in, len, offsets, n, fields, max_fields, counts, nest,
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
  uint64_t decodeChunkBytes(uint64_t len) const {
    if (chunk_bytes_) return chunk_bytes_;
    // (1/24 of the batch: config 4's 373 MB in 16 MB pieces took 11.0-11.3 ms,
    // 23 MB pieces 11.9-14.9, 8 MB 13.9-14.8; profiles/r05/ab/host_batch_pieces/)
    return std::min<uint64_t>(64ull << 20, std::max<uint64_t>(4ull << 20, len / 24));
  }
  /* Pinned host staging kept across calls (grown with 25 % slack). */
  class Pinned {
   public:
    Pinned() = default;
    Pinned(const Pinned&) = delete;
    ~Pinned() { tgpu_host_free(p_); }
    uint8_t* get(uint64_t n) {
      if (n > cap_) {
        tgpu_host_free(p_);
        p_ = nullptr;
        cap_ = 0;
        const uint64_t want = n + n / 4;
        void* q = nullptr;
        check(tgpu_host_alloc(want, &q), "tgpu_host_alloc");
        p_ = static_cast<uint8_t*>(q);
        cap_ = want;
      }
      return p_;
    }
    uint8_t* data() const { return p_; }

   private:
    uint8_t* p_ = nullptr;
    uint64_t cap_ = 0;
  };
  /* One chunk's device form in pinned memory: records, string base, list
     base. build(): the chunk's records cut into parts, each part's string /
     list bytes sized (formBytes), then every part written at its base
     (formWrite) — both passes in parallel on the host pool. */
  struct FormSlot {
    Pinned rec, str, lst;
    uint64_t slen = 0, llen = 0;
    void build(const SchemaTables& sc, uint32_t S, const void* objects, uint64_t r0, uint64_t r1,
               size_t stride, const HostStruct& hs) {
      const uint64_t m = r1 - r0;
      const uint64_t P = std::max<uint64_t>(
          1, std::min<uint64_t>(4ull * materialize_threads(), m / 2048));
      auto bound = [&](uint64_t t) { return r0 + m * t / P; };
      std::vector<std::pair<uint64_t, uint64_t>> sz(P);
      {
        HostPool::Group g;
        for (uint64_t t = 0; t < P; ++t)
          g.run([&, t] { sz[t] = formBytes(sc, objects, bound(t), bound(t + 1), stride, hs); });
        g.wait();
      }
      std::vector<detail::Sink> at(P);
      uint64_t SB = 0, LB = 0;
      for (uint64_t t = 0; t < P; ++t) {
        at[t].spos = SB;
        at[t].lpos = LB;
        SB += sz[t].first;
        LB = (LB + sz[t].second + 7) & ~7ull;
      }
      uint8_t* rp = rec.get(m * S + 16);
      uint8_t* sp = str.get(SB + 16);
      uint8_t* lp = lst.get(LB + 16);
      slen = SB;
      llen = LB;
      HostPool::Group g;
      for (uint64_t t = 0; t < P; ++t)
        g.run([&, t] {
          detail::Sink k = at[t];
          k.strings = sp;
          k.lists = lp;
          formWrite(sc, S, objects, bound(t), bound(t + 1), stride, hs,
                    rp + (bound(t) - r0) * S, k);
        });
      g.wait();
    }
  };

  const GpuSchema& schema_;
  void* stream_;
  tgpu_context* ctx_ = nullptr;
  tgpu_limits limits_{0, 0, 12000, 0};
  /* Pinned landing place of one chunk's wire and the host copies that move
     it into the queue. */
  struct WireStage {
    Pinned buf;
    HostPool::Group copies;
  };

  uint64_t chunk_records_ = 0, chunk_bytes_ = 0;
  Pinned in_, recs_, arena_;
  FormSlot slots_[3];
  WireStage wire_[3];
};

using BinaryBatchSerializer = GpuBatchSerializer<BinaryProtocol>;
using CompactBatchSerializer = GpuBatchSerializer<CompactProtocol>;
using CompactV1BatchSerializer = GpuBatchSerializer<CompactV1Protocol>;

}  // namespace apache::thrift::gpu

#endif  // THRIFT_GPU_GPU_BATCH_SERIALIZER_H_
