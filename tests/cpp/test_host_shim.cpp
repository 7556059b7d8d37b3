// Exercises the C++ host mirror (include/thrift_gpu/GpuBatchSerializer.h) on
// the GPU: a codegen-layout struct round trip and the exception types of the
// reference (TProtocolException{INVALID_DATA}, std::out_of_range).
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstring>
#include <vector>

#define THRIFT_GPU_NO_ABORT 1
#include "thrift_gpu/GpuBatchSerializer.h"

using namespace apache::thrift::gpu;

// What thrift1 would generate for `struct Flat { 1: i64 f1; ... 8: i64 f8; }`
// (members in declaration order, then isset_bitset<8> = 8 bytes).
struct Flat {
  int64_t f[8];
  uint8_t isset[8];
};
static_assert(sizeof(Flat) == 72 && offsetof(Flat, isset) == 64, "codegen layout");

struct WithBool {  // { 1: i64 a; 2: bool b; 3: i32 c; }
  int64_t a;
  uint8_t b;
  uint8_t pad[3];
  int32_t c;
  uint8_t isset[3];
  uint8_t pad2[5];
};
static_assert(sizeof(WithBool) == 24, "codegen layout");

#define CHECK(x)                                                   \
  do {                                                             \
    if (!(x)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #x); \
      return 1;                                                    \
    }                                                              \
  } while (0)

template <class T>
T* dev_alloc(size_t n) {
  T* p = nullptr;
  if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) std::abort();
  return p;
}

int main() {
  const uint64_t n = 100000;
  GpuSchema flat({{{1, TGPU_T_I64}, {2, TGPU_T_I64}, {3, TGPU_T_I64}, {4, TGPU_T_I64},
                   {5, TGPU_T_I64}, {6, TGPU_T_I64}, {7, TGPU_T_I64}, {8, TGPU_T_I64}}});
  CHECK(flat.recordSize() == sizeof(Flat));
  CHECK(flat.issetOffset(0, 0) == offsetof(Flat, isset));
  std::vector<Flat> h(n);
  for (uint64_t i = 0; i < n; ++i) {
    for (int k = 0; k < 8; ++k) h[i].f[k] = (int64_t)(i * 0x9E3779B97F4A7C15ull + k);
    std::memset(h[i].isset, 1, 8);
  }
  Flat* d_rec = dev_alloc<Flat>(n);
  Flat* d_back = dev_alloc<Flat>(n);
  uint8_t* d_wire = dev_alloc<uint8_t>(n * 89);
  CHECK(hipMemcpy(d_rec, h.data(), n * sizeof(Flat), hipMemcpyHostToDevice) == hipSuccess);

  for (int proto = 0; proto < 2; ++proto) {
    uint64_t bytes = 0, used = 0;
    if (proto == 0) {
      BinaryBatchSerializer ser(flat);
      bytes = ser.serialize(d_rec, n, d_wire, n * 89);
      CHECK(bytes == n * 89);
      used = ser.deserialize(d_wire, bytes, n, d_back);
    } else {
      CompactBatchSerializer ser(flat);
      bytes = ser.serialize(d_rec, n, d_wire, n * 89);
      used = ser.deserialize(d_wire, bytes, n, d_back);
    }
    CHECK(used == bytes);
    std::vector<Flat> back(n);
    CHECK(hipMemcpy(back.data(), d_back, n * sizeof(Flat), hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(std::memcmp(back.data(), h.data(), n * sizeof(Flat)) == 0);
  }

  // Host-memory forms (tgpu_encode_host / tgpu_decode_host): same bytes as
  // the device-resident calls, records round-trip through host memory.
  {
    BinaryBatchSerializer ser(flat);
    std::vector<uint8_t> hw(n * 89), dw(n * 89);
    CHECK(ser.serializeHost(h.data(), n, hw.data(), hw.size(), 10000) == n * 89);
    CHECK(ser.serialize(d_rec, n, d_wire, n * 89) == n * 89);
    CHECK(hipMemcpy(dw.data(), d_wire, n * 89, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(hw == dw);
    std::vector<Flat> back(n);
    CHECK(ser.deserializeHost(hw.data(), hw.size(), n, back.data(), 10000) == n * 89);
    CHECK(std::memcmp(back.data(), h.data(), n * sizeof(Flat)) == 0);
    ser.compile();  // fixed-layout schema: compiled or interpreted, same results
  }

  // Transcoding (tgpu_transcode_batch): Binary -> Compact equals the Compact
  // serializer's bytes, and Compact -> Binary gives the original stream back.
  {
    BinaryBatchSerializer bin(flat);
    CompactBatchSerializer cmp(flat);
    const uint64_t bbytes = bin.serialize(d_rec, n, d_wire, n * 89);
    uint8_t* d_c1 = dev_alloc<uint8_t>(n * 89 * 2);
    uint8_t* d_c2 = dev_alloc<uint8_t>(n * 89 * 2);
    uint8_t* d_b2 = dev_alloc<uint8_t>(n * 89);
    const uint64_t cbytes = bin.transcode<CompactProtocol>(d_wire, bbytes, n, d_c1, n * 178);
    CHECK(cmp.serialize(d_rec, n, d_c2, n * 178) == cbytes);
    std::vector<uint8_t> c1(cbytes), c2(cbytes), b1(bbytes), b2(bbytes);
    CHECK(hipMemcpy(c1.data(), d_c1, cbytes, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(hipMemcpy(c2.data(), d_c2, cbytes, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(c1 == c2);
    CHECK(cmp.transcode<BinaryProtocol>(d_c1, cbytes, n, d_b2, n * 89) == bbytes);
    CHECK(hipMemcpy(b1.data(), d_wire, bbytes, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(hipMemcpy(b2.data(), d_b2, bbytes, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(b1 == b2);
    CHECK(bin.arenaBytes(1000) == 0);  // no lists or maps
    (void)hipFree(d_c1);
    (void)hipFree(d_c2);
    (void)hipFree(d_b2);
  }

  // Schemaless skim (tgpu_skim_batch): field k of record i is an i64 whose
  // 8 value bytes follow its 3-byte header at i * 89 + 11 k.
  {
    BinaryBatchSerializer bin(flat);
    CHECK(bin.serialize(d_rec, n, d_wire, n * 89) == n * 89);
    std::vector<uint64_t> ho(n + 1);
    for (uint64_t i = 0; i <= n; ++i) ho[i] = i * 89;
    uint64_t* d_offs = dev_alloc<uint64_t>(n + 1);
    tgpu_skim_field* d_f = dev_alloc<tgpu_skim_field>(8 * n);
    uint32_t* d_cnt = dev_alloc<uint32_t>(n);
    CHECK(hipMemcpy(d_offs, ho.data(), (n + 1) * 8, hipMemcpyHostToDevice) == hipSuccess);
    bin.skim(d_wire, n * 89, d_offs, n, d_f, 8, d_cnt);
    std::vector<tgpu_skim_field> f(8 * n);
    std::vector<uint32_t> cnt(n);
    CHECK(hipMemcpy(f.data(), d_f, 8 * n * sizeof(tgpu_skim_field), hipMemcpyDeviceToHost) ==
          hipSuccess);
    CHECK(hipMemcpy(cnt.data(), d_cnt, n * 4, hipMemcpyDeviceToHost) == hipSuccess);
    for (uint64_t i = 0; i < n; i += 997) {
      CHECK(cnt[i] == 8);
      for (int k = 0; k < 8; ++k) {
        const tgpu_skim_field& e = f[k * n + i];
        CHECK(e.id == k + 1 && e.ttype == TGPU_T_I64 && e.length == 8);
        CHECK(e.offset == i * 89 + 11 * k + 3);
      }
    }
    (void)hipFree(d_offs);
    (void)hipFree(d_f);
    (void)hipFree(d_cnt);
  }

  // Binary readBool: a byte >= 2 throws TProtocolException(INVALID_DATA)
  // (BinaryProtocol-inl.h:489-495; BinaryProtocolTest.cpp:30-41).
  GpuSchema wb({{{1, TGPU_T_I64}, {2, TGPU_T_BOOL}, {3, TGPU_T_I32}}});
  CHECK(wb.recordSize() == sizeof(WithBool));
  std::vector<WithBool> hb(1000);
  for (size_t i = 0; i < hb.size(); ++i) {
    hb[i] = WithBool{};
    hb[i].a = (int64_t)i;
    hb[i].b = i & 1;
    hb[i].c = (int32_t)(i * 7);
    std::memset(hb[i].isset, 1, 3);
  }
  WithBool* d_wb = dev_alloc<WithBool>(hb.size());
  WithBool* d_wb2 = dev_alloc<WithBool>(hb.size());
  CHECK(hipMemcpy(d_wb, hb.data(), hb.size() * sizeof(WithBool), hipMemcpyHostToDevice) ==
        hipSuccess);
  BinaryBatchSerializer bser(wb);
  const uint64_t L = 3 + 8 + 3 + 1 + 3 + 4 + 1;  // 23
  const uint64_t wbytes = bser.serialize(d_wb, hb.size(), d_wire, hb.size() * L);
  CHECK(wbytes == hb.size() * L);
  const uint8_t two = 2;
  CHECK(hipMemcpy(d_wire + 417 * L + 11 + 3, &two, 1, hipMemcpyHostToDevice) == hipSuccess);
  bool threw = false;
  try {
    bser.deserialize(d_wire, wbytes, hb.size(), d_wb2);
  } catch (const TProtocolException& e) {
    threw = e.getType() == TProtocolException::INVALID_DATA;
  }
  CHECK(threw);
  // Truncated stream: std::out_of_range (folly cursor underflow).
  threw = false;
  try {
    bser.deserialize(d_wire, 416 * L + 5, 417, d_wb2);
  } catch (const std::out_of_range&) {
    threw = true;
  }
  CHECK(threw);
  // Writing an invalid bool: the reference aborts; with THRIFT_GPU_NO_ABORT a
  // logic_error carries the same diagnosis.
  hb[5].b = 7;
  CHECK(hipMemcpy(d_wb, hb.data(), hb.size() * sizeof(WithBool), hipMemcpyHostToDevice) ==
        hipSuccess);
  threw = false;
  try {
    bser.serialize(d_wb, hb.size(), d_wire, hb.size() * L);
  } catch (const std::logic_error&) {
    threw = true;
  }
  CHECK(threw);
  std::printf("host shim ok\n");
  return 0;
}
