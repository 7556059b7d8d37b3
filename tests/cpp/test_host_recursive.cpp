// Recursive structs and struct map keys through the C++ host mirror
// (GpuBatchSerializer.h + HostBinding.h): a linked list of boxed nodes
// (std::unique_ptr members, what cpp.ref / thrift.box generate) and a map
// keyed by a struct (std::map<Point, std::string>, Point with operator<).
//
// Parity anchor: a plain Binary writer over the same objects following the
// reference's headers (BinaryProtocol-inl.h:31-140) and the generated write of
// a ref field (serialize_field.whisker:32-50: a null unqualified ref is an
// empty struct). serializeBatch must produce exactly those bytes and
// deserializeBatch must give the objects back.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <vector>

#define THRIFT_GPU_NO_ABORT 1
#include "thrift_gpu/GpuBatchSerializer.h"

using namespace apache::thrift::gpu;

// struct Point { 1: i32 x; 2: i32 y; }
// struct Node { 1: i64 v; 2: optional Node next (thrift.box);
//               3: Point at (cpp.ref); 4: map<Point, string> names; }
struct Point {
  int32_t x = 0, y = 0;
  uint8_t isset[2] = {};
  bool operator<(const Point& o) const { return x != o.x ? x < o.x : y < o.y; }
  bool operator==(const Point& o) const { return x == o.x && y == o.y; }
};
struct Node {
  int64_t v = 0;
  std::unique_ptr<Node> next;
  std::unique_ptr<Point> at;
  std::map<Point, std::string> names;
  uint8_t isset[4] = {};
  bool operator==(const Node& o) const {
    if (v != o.v || names != o.names || isset[1] != o.isset[1]) return false;
    if (!!next != !!o.next || (next && !(*next == *o.next))) return false;
    return !!at == !!o.at && (!at || *at == *o.at);
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

static HostStruct pointB, nodeB;
static const HostType pointT = structType(&pointB);
static const HostType nextT = boxType<std::unique_ptr<Node>>(&nodeB);
static const HostType atT = boxType<std::unique_ptr<Point>>(&pointB);
static const HostType namesT = mapType<std::map<Point, std::string>>(&pointT, stringType());

static void bind() {
  pointB.fields = {{scalarType<int32_t>(), off(&Point::x), isset_at<Point>(0)},
                   {scalarType<int32_t>(), off(&Point::y), isset_at<Point>(1)}};
  nodeB.fields = {{scalarType<int64_t>(), off(&Node::v), isset_at<Node>(0)},
                  {&nextT, off(&Node::next), isset_at<Node>(1)},
                  {&atT, off(&Node::at), isset_at<Node>(2)},
                  {&namesT, off(&Node::names), isset_at<Node>(3)}};
}

static GpuSchema makeSchema() {
  FieldSpec next{2, TGPU_T_STRUCT, 0, false, 0};
  next.qualifier = TGPU_OPTIONAL_BOXED;
  FieldSpec at{3, TGPU_T_STRUCT, 0, false, 1};
  at.qualifier = TGPU_BOXED;
  FieldSpec names{4, TGPU_T_MAP, TGPU_T_STRUCT, false, -1, TGPU_T_STRING};
  names.key_index = 1;
  std::vector<FieldSpec> node = {{1, TGPU_T_I64}, next, at, names};
  std::vector<FieldSpec> point = {{1, TGPU_T_I32}, {2, TGPU_T_I32}};
  std::vector<tgpu_type_desc> types(1);
  types[0] = tgpu_type_desc{TGPU_T_STRUCT, 0, 0, 0, 1, 0, 0};  // the key: Point
  return GpuSchema({node, point}, {}, types);
}

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
  void point(const Point& p) {
    field(TGPU_T_I32, 1);
    be((uint32_t)p.x, 4);
    field(TGPU_T_I32, 2);
    be((uint32_t)p.y, 4);
    u8(0);
  }
  void node(const Node& n) {
    field(TGPU_T_I64, 1);
    be((uint64_t)n.v, 8);
    if (n.isset[1]) {
      field(TGPU_T_STRUCT, 2);
      node(*n.next);
    }
    field(TGPU_T_STRUCT, 3);
    if (n.at) point(*n.at);
    else u8(0);  // a null ref: writeStructBegin, writeFieldStop, writeStructEnd
    field(TGPU_T_MAP, 4);
    u8(TGPU_T_STRUCT);
    u8(TGPU_T_STRING);
    be(n.names.size(), 4);
    for (const auto& kv : n.names) {
      point(kv.first);
      be((uint32_t)kv.second.size(), 4);
      b.insert(b.end(), kv.second.begin(), kv.second.end());
    }
    u8(0);
  }
};

static Node make(std::mt19937_64& r, int depth) {
  Node n;
  n.v = (int64_t)r();
  std::memset(n.isset, 1, 4);
  n.isset[1] = depth > 0;
  if (depth > 0) n.next = std::make_unique<Node>(make(r, depth - 1));
  if (r() % 3) {
    n.at = std::make_unique<Point>();
    n.at->x = (int32_t)(r() % 100);
    n.at->y = (int32_t)(r() % 100);
    std::memset(n.at->isset, 1, 2);
  }
  for (uint64_t k = r() % 4; k--;) {
    Point p;
    p.x = (int32_t)(r() % 10);
    p.y = (int32_t)(r() % 10);
    std::memset(p.isset, 1, 2);
    n.names.emplace(p, std::string(r() % 6, (char)('a' + r() % 26)));
  }
  return n;
}

int main() {
  bind();
  GpuSchema schema = makeSchema();
  std::mt19937_64 r(0xbeef);
  const uint64_t n = 3000;
  std::vector<Node> src;
  for (uint64_t i = 0; i < n; ++i) src.push_back(make(r, i == 7 ? 500 : (int)(r() % 12)));
  BinWriter ref;
  for (const auto& x : src) ref.node(x);

  BinaryBatchSerializer bin(schema);
  IOBufQueue q;
  CHECK(bin.serializeBatch(src.data(), n, nodeB, &q) == ref.b.size());
  std::vector<uint8_t> qb = coalesced(q.front());
  CHECK(qb == ref.b);

  std::vector<Node> back(n);
  auto buf = IOBuf::copyBuffer(ref.b.data(), ref.b.size());
  CHECK(bin.deserializeBatch(buf.get(), back.data(), n, nodeB) == ref.b.size());
  for (uint64_t i = 0; i < n; ++i) {
    // a null `at` is written as an empty struct and read back as an empty one
    if (!src[i].at) {
      CHECK(back[i].at && back[i].at->x == 0 && back[i].at->y == 0);
      back[i].at.reset();
    }
    for (Node *a = &src[i], *b = &back[i]; a->next; a = a->next.get(), b = b->next.get()) {
      CHECK(b->next);
      if (!a->next->at) {
        CHECK(b->next->at);
        b->next->at.reset();
      }
    }
    CHECK(back[i] == src[i]);
  }
  std::printf("host recursive ok\n");
  return 0;
}
