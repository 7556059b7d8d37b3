// The IOBuf-facing batch API of the C++ host mirror (GpuBatchSerializer.h):
// serializeBatch of codegen'd objects (std::string / std::vector / std::map /
// std::set / nested structs, bound by HostBinding.h) appended to an IOBufQueue,
// deserializeBatch from a split IOBuf chain back into objects (COPY semantics,
// Protocol.h:406-454).
//
// Parity anchor independent of the device writer: a plain Binary writer over
// the same objects, following the reference's field / list / map / set
// headers (BinaryProtocol-inl.h:31-140: type byte + big-endian i16 id;
// element type + i32 size; key type + value type + i32 size). The Compact
// stream must equal the device transcode of that Binary stream.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

#define THRIFT_GPU_NO_ABORT 1
#include "thrift_gpu/GpuBatchSerializer.h"

using namespace apache::thrift::gpu;

// What thrift1 generates (members + isset bytes), for
//   struct Item { 1: i32 id; 2: string name; 3: list<i16> tags;
//                 4: optional double score; }
//   struct Record { 1: i64 key; 2: list<Item> items; 3: map<i32, Item> by_id;
//                   4: string note; 5: list<list<i32>> grid;
//                   6: set<string> labels;
//                   7: map<string, list<string>> index; }
struct Item {
  int32_t id = 0;
  std::string name;
  std::vector<int16_t> tags;
  double score = 0;
  uint8_t isset[4] = {};
  bool operator==(const Item& o) const {
    return id == o.id && name == o.name && tags == o.tags &&
           std::memcmp(isset, o.isset, 4) == 0 && (!isset[3] || score == o.score);
  }
};
struct Record {
  int64_t key = 0;
  std::vector<Item> items;
  std::map<int32_t, Item> by_id;
  std::string note;
  std::vector<std::vector<int32_t>> grid;
  std::set<std::string> labels;
  std::map<std::string, std::vector<std::string>> index;
  uint8_t isset[7] = {};
  bool operator==(const Record& o) const {
    return key == o.key && items == o.items && by_id == o.by_id && note == o.note &&
           grid == o.grid && labels == o.labels && index == o.index &&
           std::memcmp(isset, o.isset, 7) == 0;
  }
};

template <class T, class M>
uint32_t off(M T::*m) {
  static const T t{};
  return (uint32_t)((const char*)&(t.*m) - (const char*)&t);
}
template <class T>
int32_t isset_at(int k) {
  return (int32_t)(off(&T::isset) + k);
}

#define CHECK(x)                                                       \
  do {                                                                 \
    if (!(x)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #x); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

// ---- bindings (what thrift1 would emit per type) ------------------------------
static HostStruct itemB, recordB;
static const HostType itemT = structType(&itemB);
static const HostType i16ListT = listType<std::vector<int16_t>>(scalarType<int16_t>());
static const HostType i32ListT = listType<std::vector<int32_t>>(scalarType<int32_t>());
static const HostType strListT = listType<std::vector<std::string>>(stringType());
static const HostType itemsT = listType<std::vector<Item>>(&itemT);
static const HostType byIdT = mapType<std::map<int32_t, Item>>(scalarType<int32_t>(), &itemT);
static const HostType gridT = listType<std::vector<std::vector<int32_t>>>(&i32ListT);
static const HostType labelsT = setType<std::set<std::string>>(stringType());
static const HostType indexT =
    mapType<std::map<std::string, std::vector<std::string>>>(stringType(), &strListT);

static void bind() {
  itemB.fields = {{scalarType<int32_t>(), off(&Item::id), isset_at<Item>(0)},
                  {stringType(), off(&Item::name), isset_at<Item>(1)},
                  {&i16ListT, off(&Item::tags), isset_at<Item>(2)},
                  {scalarType<double>(), off(&Item::score), isset_at<Item>(3)}};
  recordB.fields = {{scalarType<int64_t>(), off(&Record::key), isset_at<Record>(0)},
                    {&itemsT, off(&Record::items), isset_at<Record>(1)},
                    {&byIdT, off(&Record::by_id), isset_at<Record>(2)},
                    {stringType(), off(&Record::note), isset_at<Record>(3)},
                    {&gridT, off(&Record::grid), isset_at<Record>(4)},
                    {&labelsT, off(&Record::labels), isset_at<Record>(5)},
                    {&indexT, off(&Record::index), isset_at<Record>(6)}};
}

static GpuSchema makeSchema() {
  std::vector<FieldSpec> record = {
      {1, TGPU_T_I64},
      {2, TGPU_T_LIST, TGPU_T_STRUCT, false, 1},
      {3, TGPU_T_MAP, TGPU_T_I32, false, 1, TGPU_T_STRUCT},
      {4, TGPU_T_STRING},
      {5, TGPU_T_LIST, TGPU_T_LIST, false, -1, 0, 0, 1},
      {6, TGPU_T_SET, TGPU_T_STRING},
      {7, TGPU_T_MAP, TGPU_T_STRING, false, -1, TGPU_T_LIST, 0, 2}};
  std::vector<FieldSpec> item = {{1, TGPU_T_I32},
                                 {2, TGPU_T_STRING},
                                 {3, TGPU_T_LIST, TGPU_T_I16},
                                 {4, TGPU_T_DOUBLE, 0, true}};
  std::vector<tgpu_type_desc> types(2);
  types[0] = tgpu_type_desc{TGPU_T_LIST, TGPU_T_I32, 0, 0, -1, 0, 0};
  types[1] = tgpu_type_desc{TGPU_T_LIST, TGPU_T_STRING, 0, 0, -1, 0, 0};
  return GpuSchema({record, item}, {}, types);
}

// ---- deterministic objects -----------------------------------------------------
struct Gen {
  std::mt19937_64 r;
  explicit Gen(uint64_t seed) : r(seed) {}
  uint64_t below(uint64_t n) { return n ? r() % n : 0; }
  std::string str(int maxlen) {
    std::string s(below(maxlen + 1), '\0');
    for (auto& c : s) c = (char)r();
    return s;
  }
  Item item() {
    Item it;
    it.id = (int32_t)r();
    it.name = str(12);
    for (uint64_t k = below(20); k--;) it.tags.push_back((int16_t)r());
    std::memset(it.isset, 1, 3);
    if (below(3)) {
      it.score = (double)(int64_t)r() / 3.0;
      it.isset[3] = 1;
    }
    return it;
  }
  Record record() {
    Record rec;
    rec.key = (int64_t)r();
    for (uint64_t k = below(6); k--;) rec.items.push_back(item());
    for (uint64_t k = below(4); k--;) rec.by_id.emplace((int32_t)below(1000), item());
    rec.note = str(40);
    for (uint64_t k = below(5); k--;) {
      rec.grid.emplace_back();
      for (uint64_t j = below(18); j--;) rec.grid.back().push_back((int32_t)r());
    }
    for (uint64_t k = below(5); k--;) rec.labels.insert(str(6));
    for (uint64_t k = below(3); k--;) {
      auto& v = rec.index[str(5)];
      for (uint64_t j = below(4); j--;) v.push_back(str(7));
    }
    std::memset(rec.isset, 1, 7);
    return rec;
  }
};

// ---- plain Binary writer (the parity anchor) -----------------------------------
struct BinWriter {
  std::vector<uint8_t> b;
  void u8(uint8_t v) { b.push_back(v); }
  void be(uint64_t v, int n) {
    for (int k = n - 1; k >= 0; --k) b.push_back((uint8_t)(v >> (8 * k)));
  }
  void field(uint8_t t, int16_t id) {
    u8(t);
    be((uint16_t)id, 2);
  }
  void str(const std::string& s) {
    be((uint32_t)s.size(), 4);
    b.insert(b.end(), s.begin(), s.end());
  }
  void item(const Item& it) {
    field(TGPU_T_I32, 1);
    be((uint32_t)it.id, 4);
    field(TGPU_T_STRING, 2);
    str(it.name);
    field(TGPU_T_LIST, 3);
    u8(TGPU_T_I16);
    be(it.tags.size(), 4);
    for (int16_t t : it.tags) be((uint16_t)t, 2);
    if (it.isset[3]) {
      uint64_t bits;
      std::memcpy(&bits, &it.score, 8);
      field(TGPU_T_DOUBLE, 4);
      be(bits, 8);
    }
    u8(0);
  }
  void record(const Record& r) {
    field(TGPU_T_I64, 1);
    be((uint64_t)r.key, 8);
    field(TGPU_T_LIST, 2);
    u8(TGPU_T_STRUCT);
    be(r.items.size(), 4);
    for (const auto& it : r.items) item(it);
    field(TGPU_T_MAP, 3);
    u8(TGPU_T_I32);
    u8(TGPU_T_STRUCT);
    be(r.by_id.size(), 4);
    for (const auto& kv : r.by_id) {
      be((uint32_t)kv.first, 4);
      item(kv.second);
    }
    field(TGPU_T_STRING, 4);
    str(r.note);
    field(TGPU_T_LIST, 5);
    u8(TGPU_T_LIST);
    be(r.grid.size(), 4);
    for (const auto& row : r.grid) {
      u8(TGPU_T_I32);
      be(row.size(), 4);
      for (int32_t v : row) be((uint32_t)v, 4);
    }
    field(TGPU_T_SET, 6);
    u8(TGPU_T_STRING);
    be(r.labels.size(), 4);
    for (const auto& s : r.labels) str(s);
    field(TGPU_T_MAP, 7);
    u8(TGPU_T_STRING);
    u8(TGPU_T_LIST);
    be(r.index.size(), 4);
    for (const auto& kv : r.index) {
      str(kv.first);
      u8(TGPU_T_STRING);
      be(kv.second.size(), 4);
      for (const auto& s : kv.second) str(s);
    }
    u8(0);
  }
};

// A chain of `pieces` IOBufs holding bytes (split at uneven points).
static std::unique_ptr<IOBuf> chain(const std::vector<uint8_t>& bytes, int pieces) {
  std::unique_ptr<IOBuf> head;
  size_t at = 0;
  for (int p = 0; p < pieces; ++p) {
    const size_t end = p == pieces - 1 ? bytes.size() : bytes.size() * (p + 1) * (p + 2) /
                                                            ((size_t)pieces * (pieces + 1));
    auto b = IOBuf::copyBuffer(bytes.data() + at, end - at);
    at = end;
    if (!head) head = std::move(b);
    else head->prependChain(std::move(b));
  }
  return head;
}

static std::vector<uint8_t> bytesOf(const IOBuf* head) { return coalesced(head); }

int main() {
  bind();
  GpuSchema schema = makeSchema();
  const uint64_t n = 20000;
  std::vector<Record> src;
  Gen g(0x5eed);
  for (uint64_t i = 0; i < n; ++i) src.push_back(g.record());

  BinWriter ref;
  std::vector<uint64_t> ends;
  for (const auto& r : src) {
    ref.record(r);
    ends.push_back(ref.b.size());
  }

  // Binary: serializeBatch appends exactly the reference bytes to a queue
  // that already holds data; deserializeBatch reads them back from a chain.
  BinaryBatchSerializer bin(schema);
  IOBufQueue q;
  auto pre = q.preallocate(3, 3);
  std::memcpy(pre.first, "abc", 3);
  q.postallocate(3);
  const uint64_t wrote = bin.serializeBatch(src.data(), n, recordB, &q);
  CHECK(wrote == ref.b.size());
  std::vector<uint8_t> qb = bytesOf(q.front());
  CHECK(qb.size() == 3 + ref.b.size());
  CHECK(std::memcmp(qb.data(), "abc", 3) == 0);
  CHECK(std::memcmp(qb.data() + 3, ref.b.data(), ref.b.size()) == 0);

  for (int pieces : {1, 7, 64}) {
    auto c = chain(ref.b, pieces);
    std::vector<Record> back(n);
    CHECK(bin.deserializeBatch(c.get(), back.data(), n, recordB) == ref.b.size());
    for (uint64_t i = 0; i < n; ++i) CHECK(back[i] == src[i]);
  }

  // Compact: the device transcode of the Binary stream, and round trip.
  CompactBatchSerializer cmp(schema);
  IOBufQueue cq;
  const uint64_t cbytes = cmp.serializeBatch(src.data(), n, recordB, &cq);
  std::vector<uint8_t> cb = bytesOf(cq.front());
  CHECK(cb.size() == cbytes);
  {
    uint8_t *d_b = nullptr, *d_c = nullptr;
    CHECK(hipMalloc(&d_b, ref.b.size()) == hipSuccess);
    CHECK(hipMalloc(&d_c, ref.b.size() * 2) == hipSuccess);
    CHECK(hipMemcpy(d_b, ref.b.data(), ref.b.size(), hipMemcpyHostToDevice) == hipSuccess);
    const uint64_t t = bin.transcode<CompactProtocol>(d_b, ref.b.size(), n, d_c,
                                                      ref.b.size() * 2);
    CHECK(t == cbytes);
    std::vector<uint8_t> tb(t);
    CHECK(hipMemcpy(tb.data(), d_c, t, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(tb == cb);
    (void)hipFree(d_b);
    (void)hipFree(d_c);
  }
  {
    auto c = chain(cb, 5);
    std::vector<Record> back(n);
    CHECK(cmp.deserializeBatch(c.get(), back.data(), n, recordB) == cbytes);
    for (uint64_t i = 0; i < n; ++i) CHECK(back[i] == src[i]);
  }

  // A stream cut inside record k: std::out_of_range (cursor underflow), the
  // records before it materialized.
  {
    const uint64_t k = 12345;
    std::vector<uint8_t> cut(ref.b.begin(), ref.b.begin() + (ends[k - 1] + ends[k]) / 2);
    auto c = chain(cut, 3);
    std::vector<Record> back(n);
    bool threw = false;
    try {
      bin.deserializeBatch(c.get(), back.data(), n, recordB);
    } catch (const std::out_of_range&) {
      threw = true;
    }
    CHECK(threw);
    for (uint64_t i = 0; i < k; ++i) CHECK(back[i] == src[i]);
  }
  // Many chunks both ways (serializeBatch: 2,500 records per chunk = 8
  // chunks, every slot reused; deserializeBatch: 64 KiB pieces), the bytes
  // still exactly the reference's; then a stream cut in a late piece: the
  // pipeline's resident fallback returns the records before the cut with
  // their lists (the arena copied back from the failing record's start).
  {
    BinaryBatchSerializer many(schema);
    many.setChunkRecords(2500);
    many.setChunkBytes(64 << 10);
    IOBufQueue mq;
    CHECK(many.serializeBatch(src.data(), n, recordB, &mq) == ref.b.size());
    CHECK(bytesOf(mq.front()) == ref.b);
    for (int pieces : {1, 9}) {
      auto c = chain(ref.b, pieces);
      std::vector<Record> back(n);
      CHECK(many.deserializeBatch(c.get(), back.data(), n, recordB) == ref.b.size());
      for (uint64_t i = 0; i < n; ++i) CHECK(back[i] == src[i]);
    }
    const uint64_t k = 17001;
    std::vector<uint8_t> cut(ref.b.begin(), ref.b.begin() + (ends[k - 1] + ends[k]) / 2);
    auto c = chain(cut, 1);
    std::vector<Record> back(n);
    bool threw = false;
    try {
      many.deserializeBatch(c.get(), back.data(), n, recordB);
    } catch (const std::out_of_range&) {
      threw = true;
    }
    CHECK(threw);
    for (uint64_t i = 0; i < k; ++i) CHECK(back[i] == src[i]);
  }
  std::printf("host objects ok\n");
  return 0;
}
