// Host-object batch rate (bench.py --host-batch): serializeBatch of
// codegen'd C++ objects into an IOBufQueue and deserializeBatch of the IOBuf
// back into objects (include/thrift_gpu/GpuBatchSerializer.h) — the calls a
// drop-in caller of Serializer<R,W>::serialize / deserialize makes
// (thrift/lib/cpp2/protocol/Serializer.h:62-72,136-148), with the objects'
// std::string / std::vector members filled with COPY semantics
// (Protocol.h:406-454). Workloads: BASELINE config 3 (Compact {4 x i32,
// 2 x string}) and config 4 (Binary {i64, list<i32>, inner {3 x double}}).
//
// Beside it, the CPU rate of a hand-written reader/writer of the same
// objects in the generated code's shape (serialize_struct.whisker /
// deserialize_struct.whisker fast path: fields in order, one record after
// another), single-threaded: what one core of the reference's generated
// code does for these types (an estimate: the reference itself needs folly
// and cannot be built here).
//
// Usage: host_batch_bench <config 3|4> <records> <reps>; prints one JSON line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#define THRIFT_GPU_NO_ABORT 1
#include "thrift_gpu/GpuBatchSerializer.h"

using namespace apache::thrift::gpu;
using Clock = std::chrono::steady_clock;

template <class T, class M>
uint32_t off(M T::*m) {
  static const T t{};
  return (uint32_t)((const char*)&(t.*m) - (const char*)&t);
}
template <class T>
int32_t isset_at(int k) {
  return (int32_t)(off(&T::isset) + k);
}
static double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

// ---- config 3: struct Mixed { 1..4: i32; 5, 6: string } (Compact) ----------
struct Mixed {
  int32_t a = 0, b = 0, c = 0, d = 0;
  std::string e, f;
  uint8_t isset[6] = {};
  bool operator==(const Mixed& o) const {
    return a == o.a && b == o.b && c == o.c && d == o.d && e == o.e && f == o.f &&
           std::memcmp(isset, o.isset, 6) == 0;
  }
};
// ---- config 4: struct Inner { 1..3: double }; struct Nested { 1: i64;
//      2: list<i32>; 3: Inner } (Binary) ----------------------------------------
struct Inner {
  double x = 0, y = 0, z = 0;
  uint8_t isset[3] = {};
  bool operator==(const Inner& o) const {
    return x == o.x && y == o.y && z == o.z && std::memcmp(isset, o.isset, 3) == 0;
  }
};
struct Nested {
  int64_t k = 0;
  std::vector<int32_t> l;
  Inner in;
  uint8_t isset[3] = {};
  bool operator==(const Nested& o) const {
    return k == o.k && l == o.l && in == o.in && std::memcmp(isset, o.isset, 3) == 0;
  }
};

static HostStruct mixedB, innerB, nestedB;
static const HostType innerT = structType(&innerB);
static const HostType i32ListT = listType<std::vector<int32_t>>(scalarType<int32_t>());

static void bind() {
  mixedB.fields = {{scalarType<int32_t>(), off(&Mixed::a), isset_at<Mixed>(0)},
                   {scalarType<int32_t>(), off(&Mixed::b), isset_at<Mixed>(1)},
                   {scalarType<int32_t>(), off(&Mixed::c), isset_at<Mixed>(2)},
                   {scalarType<int32_t>(), off(&Mixed::d), isset_at<Mixed>(3)},
                   {stringType(), off(&Mixed::e), isset_at<Mixed>(4)},
                   {stringType(), off(&Mixed::f), isset_at<Mixed>(5)}};
  innerB.fields = {{scalarType<double>(), off(&Inner::x), isset_at<Inner>(0)},
                   {scalarType<double>(), off(&Inner::y), isset_at<Inner>(1)},
                   {scalarType<double>(), off(&Inner::z), isset_at<Inner>(2)}};
  nestedB.fields = {{scalarType<int64_t>(), off(&Nested::k), isset_at<Nested>(0)},
                    {&i32ListT, off(&Nested::l), isset_at<Nested>(1)},
                    {&innerT, off(&Nested::in), isset_at<Nested>(2)}};
}

static Mixed gen_mixed(std::mt19937_64& r) {
  Mixed m;
  auto v = [&]() {  // 1..5-byte varints, as BASELINE config 3
    const int b = 1 + (int)(r() % 5);
    const uint64_t hi = b == 5 ? 0xffffffffull : (1ull << (7 * b)) - 1;
    const uint64_t lo = b == 1 ? 0 : 1ull << (7 * (b - 1));
    const uint32_t z = (uint32_t)(lo + r() % (hi - lo + 1));
    return (int32_t)((z >> 1) ^ -(int32_t)(z & 1));
  };
  m.a = v(), m.b = v(), m.c = v(), m.d = v();
  for (std::string* s : {&m.e, &m.f}) {
    s->resize(r() % 33);
    for (auto& ch : *s) ch = (char)r();
  }
  std::memset(m.isset, 1, 6);
  return m;
}
static Nested gen_nested(std::mt19937_64& r) {
  Nested n;
  n.k = (int64_t)r();
  n.l.resize(r() % 17);
  for (auto& x : n.l) x = (int32_t)r();
  n.in.x = (double)(int64_t)r() / 7.0;
  n.in.y = (double)(int64_t)r() / 11.0;
  n.in.z = (double)(int64_t)r() / 13.0;
  std::memset(n.in.isset, 1, 3);
  std::memset(n.isset, 1, 3);
  return n;
}

// ---- the generated code's shape, one core -----------------------------------
// An appender in the shape of folly's QueueAppender: a capacity check per
// write, uninitialized storage grown geometrically.
struct Out {
  std::unique_ptr<uint8_t[]> buf;
  size_t cap = 0, len = 0;
  void reserve(size_t n) {
    if (n <= cap) return;
    std::unique_ptr<uint8_t[]> nb(new uint8_t[n]);
    if (len) std::memcpy(nb.get(), buf.get(), len);
    buf = std::move(nb);
    cap = n;
  }
  uint8_t* room(size_t k) {
    if (len + k > cap) reserve(std::max(2 * cap, len + k + (64 << 10)));
    uint8_t* q = buf.get() + len;
    len += k;
    return q;
  }
  void u8(uint8_t v) { *room(1) = v; }
  void be(uint64_t v, int n) {
    uint8_t* q = room(n);
    for (int k = 0; k < n; ++k) q[k] = (uint8_t)(v >> (8 * (n - 1 - k)));
  }
  void varint(uint64_t v) {
    uint8_t* q = room(10);
    int k = 0;
    while (v >= 0x80) {
      q[k++] = (uint8_t)(v | 0x80);
      v >>= 7;
    }
    q[k++] = (uint8_t)v;
    len -= 10 - k;
  }
  void bytes(const std::string& s) { std::memcpy(room(s.size()), s.data(), s.size()); }
  const uint8_t* data() const { return buf.get(); }
  bool same(const std::vector<uint8_t>& b) const {
    return len == b.size() && std::memcmp(buf.get(), b.data(), len) == 0;
  }
};
struct In {
  const uint8_t* p;
  const uint8_t* e;
  uint8_t u8() {
    if (p >= e) throw std::out_of_range("underflow");
    return *p++;
  }
  uint64_t be(int n) {
    if (e - p < n) throw std::out_of_range("underflow");
    uint64_t v = 0;
    for (int k = 0; k < n; ++k) v = (v << 8) | *p++;
    return v;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 70; s += 7) {
      const uint8_t x = u8();
      v |= (uint64_t)(x & 0x7f) << s;
      if (!(x & 0x80)) return v;
    }
    throw std::out_of_range("invalid varint");
  }
  void bytes(std::string& s, uint64_t n) {
    if ((uint64_t)(e - p) < n) throw std::out_of_range("underflow");
    s.assign((const char*)p, n);
    p += n;
  }
};
static uint32_t zz(int32_t v) { return ((uint32_t)v << 1) ^ (uint32_t)(v >> 31); }
static int32_t unzz(uint32_t v) { return (int32_t)((v >> 1) ^ -(int32_t)(v & 1)); }

static void write_mixed(Out& o, const Mixed& m) {  // Compact, fields 1..6 in order
  for (int32_t v : {m.a, m.b, m.c, m.d}) {
    o.u8(0x15);
    o.varint(zz(v));
  }
  for (const std::string* s : {&m.e, &m.f}) {
    o.u8(0x18);
    o.varint(s->size());
    o.bytes(*s);
  }
  o.u8(0);
}
static void read_mixed(In& in, Mixed& m) {
  int32_t* ints[4] = {&m.a, &m.b, &m.c, &m.d};
  for (int k = 0; k < 4; ++k) {
    if (in.u8() != 0x15) throw std::runtime_error("slow path");
    *ints[k] = unzz((uint32_t)in.varint());
  }
  for (std::string* s : {&m.e, &m.f}) {
    if (in.u8() != 0x18) throw std::runtime_error("slow path");
    in.bytes(*s, in.varint());
  }
  if (in.u8() != 0) throw std::runtime_error("slow path");
  std::memset(m.isset, 1, 6);
}
static void write_nested(Out& o, const Nested& n) {  // Binary
  o.u8(10), o.be(1, 2), o.be((uint64_t)n.k, 8);
  o.u8(15), o.be(2, 2), o.u8(8), o.be(n.l.size(), 4);
  for (int32_t x : n.l) o.be((uint32_t)x, 4);
  o.u8(12), o.be(3, 2);
  for (int k = 0; k < 3; ++k) {
    const double d = k == 0 ? n.in.x : k == 1 ? n.in.y : n.in.z;
    uint64_t bits;
    std::memcpy(&bits, &d, 8);
    o.u8(4), o.be(k + 1, 2), o.be(bits, 8);
  }
  o.u8(0);
  o.u8(0);
}
static void read_nested(In& in, Nested& n) {
  if (in.u8() != 10 || in.be(2) != 1) throw std::runtime_error("slow path");
  n.k = (int64_t)in.be(8);
  if (in.u8() != 15 || in.be(2) != 2 || in.u8() != 8) throw std::runtime_error("slow path");
  const uint32_t len = (uint32_t)in.be(4);
  n.l.resize(len);
  for (auto& x : n.l) x = (int32_t)in.be(4);
  if (in.u8() != 12 || in.be(2) != 3) throw std::runtime_error("slow path");
  for (int k = 0; k < 3; ++k) {
    if (in.u8() != 4 || in.be(2) != (uint64_t)(k + 1)) throw std::runtime_error("slow path");
    const uint64_t bits = in.be(8);
    std::memcpy(k == 0 ? &n.in.x : k == 1 ? &n.in.y : &n.in.z, &bits, 8);
  }
  if (in.u8() != 0 || in.u8() != 0) throw std::runtime_error("slow path");
  std::memset(n.in.isset, 1, 3);
  std::memset(n.isset, 1, 3);
}

template <class Ser, class T, class Gen, class W, class R>
static int run(int config, const GpuSchema& schema, const HostStruct& binding, uint64_t n,
               int reps, Gen gen, W write, R read) {
  std::mt19937_64 r(0x1729 + config);
  std::vector<T> src;
  src.reserve(n);
  for (uint64_t i = 0; i < n; ++i) src.push_back(gen(r));
  Ser ser(schema);
  ser.compile();
  // (A/B: records per serializeBatch chunk; default the serializer's)
  if (const char* e = std::getenv("HB_CHUNK_RECORDS")) ser.setChunkRecords(std::strtoull(e, nullptr, 10));
  // (A/B: wire bytes per deserializeBatch piece; default 1/16 of the batch)
  if (const char* e = std::getenv("HB_CHUNK_BYTES")) ser.setChunkBytes(std::strtoull(e, nullptr, 10));
  double ser_ms = 1e30, de_ms = 1e30;
  uint64_t wire = 0;
  std::vector<uint8_t> bytes;
  for (int rep = 0; rep < reps; ++rep) {
    IOBufQueue q;
    auto t0 = Clock::now();
    wire = ser.serializeBatch(src.data(), n, binding, &q);
    ser_ms = std::min(ser_ms, ms_since(t0));
    if (rep == 0) bytes = coalesced(q.front());
  }
  auto buf = IOBuf::copyBuffer(bytes.data(), bytes.size());
  std::vector<T> back;
  for (int rep = 0; rep < reps; ++rep) {
    back.assign(n, T{});
    auto t0 = Clock::now();
    ser.deserializeBatch(buf.get(), back.data(), n, binding);
    de_ms = std::min(de_ms, ms_since(t0));
  }
  for (uint64_t i = 0; i < n; ++i)
    if (!(back[i] == src[i])) {
      std::fprintf(stderr, "mismatch at record %llu\n", (unsigned long long)i);
      return 1;
    }
  // the host side alone: materialize() of device-form records decoded once
  // (the resident pass) into fresh objects, and the device pass alone
  // (deserializeHostEx into pinned records / arena, nothing materialized)
  double mat_ms = 1e30, dev_ms = 1e30;
  {
    const uint32_t S = schema.recordSize();
    const uint64_t acap = bytes.size() * tgpu_schema_arena_scale(schema.get(), Ser::protocolType());
    void *recs = nullptr, *ar = nullptr;
    check(tgpu_host_alloc(n * S + 16, &recs), "tgpu_host_alloc");
    check(tgpu_host_alloc(acap + 16, &ar), "tgpu_host_alloc");
    for (int rep = 0; rep < reps; ++rep) {
      auto t0 = Clock::now();
      ser.deserializeHostEx(buf->data(), bytes.size(), n, recs, acap ? ar : nullptr, acap);
      dev_ms = std::min(dev_ms, ms_since(t0));
    }
    for (int rep = 0; rep < reps; ++rep) {
      back.assign(n, T{});
      auto t0 = Clock::now();
      materialize(schema.tables(), (const uint8_t*)recs, n, S, buf->data(), (const uint8_t*)ar,
                  binding, back.data(), sizeof(T));
      mat_ms = std::min(mat_ms, ms_since(t0));
    }
    tgpu_host_free(recs);
    tgpu_host_free(ar);
  }
  // the generated code's shape, one core (and its bytes must match)
  Out o;
  o.reserve(wire);
  auto t0 = Clock::now();
  for (const T& x : src) write(o, x);
  const double cw = ms_since(t0);
  if (!o.same(bytes)) {
    std::fprintf(stderr, "CPU writer bytes differ\n");
    return 1;
  }
  std::vector<T> cb(n);
  std::vector<uint64_t> ends(n);
  t0 = Clock::now();
  In in{o.data(), o.data() + o.len};
  for (uint64_t i = 0; i < n; ++i) {
    read(in, cb[i]);
    ends[i] = (uint64_t)(in.p - o.data());
  }
  const double cr = ms_since(t0) ;
  // the same reader / writer on materialize_threads() host threads, each on
  // a contiguous record range: the writer's parts concatenated into one
  // buffer (the copy timed too); the reader given every part's first record
  // start (an index the reference's file loop does not have — its best case)
  const unsigned TT = materialize_threads();
  auto part = [&](unsigned t) { return std::make_pair(n * t / TT, n * (t + 1) / TT); };
  double cwT = 1e30, crT = 1e30;
  for (int rep = 0; rep < reps; ++rep) {
    std::vector<Out> parts(TT);
    std::unique_ptr<uint8_t[]> joined;
    std::vector<uint64_t> base(TT + 1, 0);
    auto t1 = Clock::now();
    {
      std::vector<std::thread> th;
      for (unsigned t = 0; t < TT; ++t)
        th.emplace_back([&, t] {
          auto [b, e] = part(t);
          parts[t].reserve((e - b) * (wire / n + 16));
          for (uint64_t i = b; i < e; ++i) write(parts[t], src[i]);
        });
      for (auto& x : th) x.join();
      for (unsigned t = 0; t < TT; ++t) base[t + 1] = base[t] + parts[t].len;
      joined.reset(new uint8_t[base[TT]]);
      th.clear();
      for (unsigned t = 0; t < TT; ++t)
        th.emplace_back([&, t] {
          std::memcpy(joined.get() + base[t], parts[t].data(), parts[t].len);
        });
      for (auto& x : th) x.join();
    }
    cwT = std::min(cwT, ms_since(t1));
    if (base[TT] != bytes.size() || std::memcmp(joined.get(), bytes.data(), bytes.size()) != 0) {
      std::fprintf(stderr, "threaded CPU writer bytes differ\n");
      return 1;
    }
    std::vector<T> cbT(n);
    t1 = Clock::now();
    {
      std::vector<std::thread> th;
      for (unsigned t = 0; t < TT; ++t)
        th.emplace_back([&, t] {
          auto [b, e] = part(t);
          In pin{o.data() + (b ? ends[b - 1] : 0), o.data() + (e ? ends[e - 1] : 0)};
          for (uint64_t i = b; i < e; ++i) read(pin, cbT[i]);
        });
      for (auto& x : th) x.join();
    }
    crT = std::min(crT, ms_since(t1));
    for (uint64_t i = 0; i < n; i += 997)
      if (!(cbT[i] == src[i])) {
        std::fprintf(stderr, "threaded CPU reader mismatch at %llu\n", (unsigned long long)i);
        return 1;
      }
  }
  const double gib = (double)wire / (1ull << 30);
  std::printf(
      "{\"config\": %d, \"records\": %llu, \"wire_bytes\": %llu, \"reps\": %d, "
      "\"serializeBatch_ms\": %.3f, \"deserializeBatch_ms\": %.3f, "
      "\"serializeBatch_GiBps\": %.3f, \"deserializeBatch_GiBps\": %.3f, "
      "\"serializeBatch_ns_per_record\": %.2f, \"deserializeBatch_ns_per_record\": %.2f, "
      "\"cpu_generated_shape_1core\": {\"write_ms\": %.3f, \"read_ms\": %.3f, "
      "\"write_GiBps\": %.3f, \"read_GiBps\": %.3f}, "
      "\"cpu_generated_shape_threads\": {\"threads\": %u, \"write_ms\": %.3f, "
      "\"read_ms\": %.3f, \"write_GiBps\": %.3f, \"read_GiBps\": %.3f, "
      "\"note\": \"reader given each thread's first record start\"}, "
      "\"materialize_only_ms\": %.3f, \"device_pass_resident_ms\": %.3f, "
      "\"materialize_threads\": %u}\n",
      config, (unsigned long long)n, (unsigned long long)wire, reps, ser_ms, de_ms,
      gib / (ser_ms / 1e3), gib / (de_ms / 1e3), ser_ms * 1e6 / n, de_ms * 1e6 / n, cw, cr,
      gib / (cw / 1e3), gib / (cr / 1e3), TT, cwT, crT, gib / (cwT / 1e3), gib / (crT / 1e3),
      mat_ms, dev_ms, materialize_threads());
  return 0;
}

int main(int argc, char** argv) {
  const int config = argc > 1 ? std::atoi(argv[1]) : 3;
  const uint64_t n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (4ull << 20);
  const int reps = argc > 3 ? std::atoi(argv[3]) : 3;
  bind();
  try {
    if (config == 3) {
      GpuSchema schema({{{1, TGPU_T_I32}, {2, TGPU_T_I32}, {3, TGPU_T_I32}, {4, TGPU_T_I32},
                         {5, TGPU_T_STRING}, {6, TGPU_T_STRING}}});
      return run<CompactBatchSerializer, Mixed>(config, schema, mixedB, n, reps, gen_mixed,
                                                write_mixed, read_mixed);
    }
    GpuSchema schema({{{1, TGPU_T_I64}, {2, TGPU_T_LIST, TGPU_T_I32}, {3, TGPU_T_STRUCT, 0, false, 1}},
                      {{1, TGPU_T_DOUBLE}, {2, TGPU_T_DOUBLE}, {3, TGPU_T_DOUBLE}}});
    return run<BinaryBatchSerializer, Nested>(config, schema, nestedB, n, reps, gen_nested,
                                              write_nested, read_nested);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 2;
  }
}
