// Host-only check of HostBinding.h's one-copy list path (no GPU, no
// library): a list<i16> schema field bound to std::vector<int32_t> must take
// the per-element path on both decode (readStruct) and encode (writeStruct):
// the one-copy path reads / writes sizeof(E) bytes per element and would
// misread the 2-byte device elements. A width-matched
// binding (list<i32> -> std::vector<int32_t>) keeps the one-copy path and
// gives the same values. A schema type WIDER than the bound element
// (list<i64> -> std::vector<int32_t>) takes the per-element
// path too and never copies more than 4 bytes into / out of an element:
// decode keeps the low bytes, encode sign-extends (built with
// -fsanitize=address, so an overrun fails the run).
#include <cstdio>
#include <cstring>
#include <vector>

#include "thrift_gpu/HostBinding.h"

using namespace apache::thrift::gpu;

#define CHECK(x)                                                   \
  do {                                                             \
    if (!(x)) {                                                    \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #x); \
      return 1;                                                    \
    }                                                              \
  } while (0)

struct Rec {
  std::vector<int32_t> v;
  uint8_t isset[1];
};

static int run(uint8_t elem_tt, uint32_t ew) {
  // one struct { 1: list<elem_tt> v } — device record: span @0, isset @16
  tgpu_struct_desc s{0, 1, 24, 8, 0};
  tgpu_field_desc f{};
  f.id = 1;
  f.ttype = TGPU_T_LIST;
  f.elem_ttype = elem_tt;
  f.member_offset = 0;
  f.isset_offset = 16;
  f.struct_index = -1;
  const SchemaTables sc{&s, &f, nullptr};
  static const HostType vT = listType<std::vector<int32_t>>(scalarType<int32_t>());
  HostStruct hs;
  hs.fields = {{&vT, offsetof(Rec, v), (int32_t)offsetof(Rec, isset)}};

  // decode: 5 elements of ew bytes in the arena
  const int32_t want[5] = {-3, 7, 300, -32768, 32767};
  std::vector<uint8_t> arena(64, 0xee);
  for (int i = 0; i < 5; ++i) {
    const int64_t w64 = want[i];  // (little-endian: the low ew bytes of the value)
    std::memcpy(arena.data() + 8 + i * ew, &w64, ew);
  }
  uint8_t dev[24] = {};
  detail::storeSpan(dev, 8, 5);
  dev[16] = 1;
  Rec r{};
  detail::readStruct(sc, 0, dev, detail::Sources{nullptr, arena.data()}, hs, (uint8_t*)&r);
  CHECK(r.isset[0] == 1 && r.v.size() == 5);
  for (int i = 0; i < 5; ++i) CHECK(r.v[i] == want[i]);

  // encode: the device form's element array holds ew bytes per element
  std::vector<uint8_t> lists(5 * ew, 0), out(24, 0);
  detail::Sink k;
  detail::writeStruct<true>(sc, 0, (const uint8_t*)&r, hs, k, nullptr);
  CHECK(k.lpos == 5 * ew);
  detail::Sink sink;
  sink.lists = lists.data();
  detail::writeStruct<false>(sc, 0, (const uint8_t*)&r, hs, sink, out.data());
  const tgpu_span sp = detail::loadSpan(out.data());
  CHECK(sp.length == 5);
  for (int i = 0; i < 5; ++i) {
    int64_t x = 0;
    std::memcpy(&x, lists.data() + sp.offset + i * ew, ew);
    if (ew == 2) x = (int16_t)x;
    if (ew == 4) x = (int32_t)x;
    CHECK(x == want[i]);
  }
  return 0;
}

int main() {
  if (run(TGPU_T_I16, 2)) return 1;  // width mismatch: per-element path
  if (run(TGPU_T_I32, 4)) return 1;  // matched: the one-copy path
  if (run(TGPU_T_I64, 8)) return 1;  // schema wider than the element: per element, in bounds
  std::printf("binding width ok\n");
  return 0;
}
