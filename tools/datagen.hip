// Device-side record generators for bench.py configs 3 and 4, following the
// spec of tests/golden/datagen.py (gen_mixed / gen_nested: counter-based
// splitmix64, seed 0x1729) so that a bench batch's first records equal the
// golden generator's. Built into tools/build/libtgpu_datagen.so.
//
// Layouts (tgpu_layout_compute, see fbthrift_amd/schema.py):
//   mixed  (S=56): i32 f1..f4 @0..12, span f5 @16, span f6 @32, isset[6] @48
//   nested (S=64): i64 @0, span(list<i32>) @8, Inner{3 x f64, isset[3]} @24,
//                  isset[3] @56
// tgpu_gen_mixed / tgpu_gen_nested: strings of record i live in a 64-byte slot
// at string_base + 64 i (+32 for field 6); list elements in a 64-byte slot at
// list_base + 64 i. The _packed forms (bench.py) store the same bytes back to
// back in record order (field 5 then 6; a record's list after the previous
// record's): the layout a columnar caller hands over, and the one the decode
// leaves (string views into one contiguous stream). Both fit n * 64 bytes.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

namespace {

__device__ inline uint64_t sm64(uint64_t seed, uint64_t index) {
  uint64_t z = seed + (index + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Span {
  uint64_t off;
  uint32_t len;
  uint32_t reserved;
};

__global__ void gen_mixed_kernel(uint64_t seed, uint64_t first, uint64_t n, uint8_t* recs,
                                 uint8_t* strings) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t i = first + t;
  uint8_t* r = recs + t * 56;
  for (int k = 0; k < 4; ++k) {
    const uint64_t a = sm64(seed, 16 * i + 2 * k), b2 = sm64(seed, 16 * i + 2 * k + 1);
    const uint64_t b = 1 + a % 5;
    const uint64_t lo = b == 1 ? 0 : 1ull << (7 * (b - 1));
    const uint64_t hi = b == 5 ? 0xFFFFFFFFull : (1ull << (7 * b)) - 1;
    const uint32_t z = (uint32_t)(lo + b2 % (hi - lo + 1));
    const int32_t v = (int32_t)((z >> 1) ^ (0u - (z & 1)));
    *(int32_t*)(r + 4 * k) = v;
  }
  for (int k = 0; k < 2; ++k) {
    const uint32_t len = (uint32_t)(sm64(seed, 16 * i + 8 + k) % 33);
    uint64_t* slot = (uint64_t*)(strings + t * 64 + 32 * k);
    for (int w = 0; w < 4; ++w) slot[w] = sm64(seed ^ 0x5EED, (2 * i + k) * 4 + w);
    Span s{t * 64 + 32 * k, len, 0};
    *(Span*)(r + 16 + 16 * k) = s;
  }
  *(uint64_t*)(r + 48) = 0x0000010101010101ull;  // isset[6] + 2 pad bytes
}

__device__ inline uint32_t mixed_len(uint64_t seed, uint64_t i, int k) {
  return (uint32_t)(sm64(seed, 16 * i + 8 + k) % 33);
}
__device__ inline uint32_t nested_len(uint64_t seed, uint64_t i) {
  return (uint32_t)(sm64(seed, 32 * i + 1) % 17);
}

// payload bytes of record t (first + t): mixed strings, nested i32 elements
__global__ void payload_len_kernel(uint64_t seed, uint64_t first, uint64_t n, int nested,
                                   uint64_t* out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t i = first + t;
  out[t] = nested ? 4ull * nested_len(seed, i) : mixed_len(seed, i, 0) + mixed_len(seed, i, 1);
}

// the same records as gen_mixed_kernel, strings packed at base[t]
__global__ void gen_mixed_packed_kernel(uint64_t seed, uint64_t first, uint64_t n, uint8_t* recs,
                                        uint8_t* strings, const uint64_t* base) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t i = first + t;
  uint8_t* r = recs + t * 56;
  uint64_t off = base[t];
  for (int k = 0; k < 2; ++k) {
    const uint32_t len = mixed_len(seed, i, k);
    for (uint32_t b = 0; b < len; ++b)
      strings[off + b] = (uint8_t)(sm64(seed ^ 0x5EED, (2 * i + k) * 4 + b / 8) >> (8 * (b % 8)));
    Span s{off, len, 0};
    *(Span*)(r + 16 + 16 * k) = s;
    off += len;
  }
}

// the same records as gen_nested_kernel, list elements packed at base[t]
__global__ void gen_nested_packed_kernel(uint64_t seed, uint64_t first, uint64_t n, uint8_t* recs,
                                         uint8_t* lists, const uint64_t* base) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t i = first + t;
  uint8_t* r = recs + t * 64;
  const uint32_t len = nested_len(seed, i);
  int32_t* e = (int32_t*)(lists + base[t]);
  for (uint32_t j = 0; j < len; ++j) e[j] = (int32_t)(uint32_t)sm64(seed, 32 * i + 2 + j);
  Span s{base[t], len, 0};
  *(Span*)(r + 8) = s;
}

__device__ inline uint64_t finite_bits(uint64_t b) {
  if (((b >> 52) & 0x7FF) == 0x7FF) b &= ~(1ull << 62);
  return b;
}

__global__ void gen_nested_kernel(uint64_t seed, uint64_t first, uint64_t n, uint8_t* recs,
                                  uint8_t* lists) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t i = first + t;
  uint8_t* r = recs + t * 64;
  *(uint64_t*)r = sm64(seed, 32 * i);
  const uint32_t len = (uint32_t)(sm64(seed, 32 * i + 1) % 17);
  int32_t* slot = (int32_t*)(lists + t * 64);
  for (uint32_t j = 0; j < 16; ++j) slot[j] = j < len ? (int32_t)(uint32_t)sm64(seed, 32 * i + 2 + j) : 0;
  Span s{t * 64, len, 0};
  *(Span*)(r + 8) = s;
  for (int k = 0; k < 3; ++k) *(uint64_t*)(r + 24 + 8 * k) = finite_bits(sm64(seed, 32 * i + 20 + k));
  *(uint64_t*)(r + 48) = 0x0000000000010101ull;  // Inner isset[3] + pad
  *(uint64_t*)(r + 56) = 0x0000000000010101ull;  // isset[3] + pad
}

}  // namespace

extern "C" int tgpu_gen_mixed(uint64_t seed, uint64_t first, uint64_t n, void* recs,
                              void* strings, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(gen_mixed_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, seed, first, n, (uint8_t*)recs, (uint8_t*)strings);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int tgpu_gen_nested(uint64_t seed, uint64_t first, uint64_t n, void* recs,
                               void* lists, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(gen_nested_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, seed, first, n, (uint8_t*)recs, (uint8_t*)lists);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

namespace {
// slot generator, then the payloads moved to their packed positions (an
// exclusive scan of the per-record payload bytes)
int gen_packed(bool nested, uint64_t seed, uint64_t first, uint64_t n, void* recs, void* side,
               hipStream_t st) {
  if (n == 0) return 0;
  const dim3 g((uint32_t)((n + 255) / 256)), b(256);
  if (nested)
    hipLaunchKernelGGL(gen_nested_kernel, g, b, 0, st, seed, first, n, (uint8_t*)recs,
                       (uint8_t*)side);
  else
    hipLaunchKernelGGL(gen_mixed_kernel, g, b, 0, st, seed, first, n, (uint8_t*)recs,
                       (uint8_t*)side);
  uint64_t* lens = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  if (hipMallocAsync((void**)&lens, 2 * n * sizeof(uint64_t), st) != hipSuccess) return 1;
  uint64_t* base = lens + n;
  hipLaunchKernelGGL(payload_len_kernel, g, b, 0, st, seed, first, n, nested ? 1 : 0, lens);
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tb, lens, base, n, st) != hipSuccess ||
      hipMallocAsync(&tmp, tb, st) != hipSuccess ||
      hipcub::DeviceScan::ExclusiveSum(tmp, tb, lens, base, n, st) != hipSuccess)
    return 1;
  if (nested)
    hipLaunchKernelGGL(gen_nested_packed_kernel, g, b, 0, st, seed, first, n, (uint8_t*)recs,
                       (uint8_t*)side, base);
  else
    hipLaunchKernelGGL(gen_mixed_packed_kernel, g, b, 0, st, seed, first, n, (uint8_t*)recs,
                       (uint8_t*)side, base);
  const hipError_t e = hipGetLastError();
  (void)hipFreeAsync(tmp, st);
  (void)hipFreeAsync(lens, st);
  return e == hipSuccess ? 0 : 1;
}
}  // namespace

extern "C" int tgpu_gen_mixed_packed(uint64_t seed, uint64_t first, uint64_t n, void* recs,
                                     void* strings, void* stream) {
  return gen_packed(false, seed, first, n, recs, strings, (hipStream_t)stream);
}

extern "C" int tgpu_gen_nested_packed(uint64_t seed, uint64_t first, uint64_t n, void* recs,
                                      void* lists, void* stream) {
  return gen_packed(true, seed, first, n, recs, lists, (hipStream_t)stream);
}
