// Measured HBM ceiling for the roofline: streaming copies (bytes moved = read
// + write) in a few shapes; bench.py reports the best. Also the PMC
// calibration copies (16- and 8-byte lanes) used by tools/pmc_summary.py.
// Built into tools/build/libcopyceil.so.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename V, bool kNT, int kUnroll>
__global__ __launch_bounds__(256) void copy_t(const V* __restrict__ src, V* __restrict__ dst,
                                              uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * kUnroll;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 * kUnroll + threadIdx.x; base < n;
       base += stride) {
    V v[kUnroll];
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      const uint64_t i = base + (uint64_t)k * 256;
      if (i < n) v[k] = kNT ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      const uint64_t i = base + (uint64_t)k * 256;
      if (i < n) {
        if (kNT)
          __builtin_nontemporal_store(v[k], dst + i);
        else
          dst[i] = v[k];
      }
    }
  }
}

// The calibration kernels keep distinct names for the PMC summary.
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ src,
                                                    u32x4* __restrict__ dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16;
       i += (uint64_t)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}
__global__ __launch_bounds__(256) void copy8_kernel(const unsigned long long* __restrict__ src,
                                                     unsigned long long* __restrict__ dst,
                                                     uint64_t n8) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n8;
       i += (uint64_t)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

extern "C" int copy_calibrate(const void* src, void* dst, uint64_t bytes) {
  hipLaunchKernelGGL(copy_kernel, dim3(2048), dim3(256), 0, 0, (const u32x4*)src,
                           (u32x4*)dst, bytes / 16);
  hipLaunchKernelGGL(copy8_kernel, dim3(2048), dim3(256), 0, 0,
                           (const unsigned long long*)src, (unsigned long long*)dst, bytes / 8);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

static void launch_variant(int variant, const void* src, void* dst, uint64_t bytes) {
  const uint64_t n16 = bytes / 16;
  const u32x4* s = (const u32x4*)src;
  u32x4* d = (u32x4*)dst;
  const uint32_t full1 = (uint32_t)((n16 + 255) / 256), full4 = (uint32_t)((n16 + 1023) / 1024);
  switch (variant) {
    case 0: hipLaunchKernelGGL((copy_t<u32x4, true, 4>), dim3(2048), dim3(256), 0, 0, s, d, n16); break;
    case 1: hipLaunchKernelGGL((copy_t<u32x4, false, 4>), dim3(2048), dim3(256), 0, 0, s, d, n16); break;
    case 2: hipLaunchKernelGGL((copy_t<u32x4, true, 1>), dim3(full1), dim3(256), 0, 0, s, d, n16); break;
    case 3: hipLaunchKernelGGL((copy_t<u32x4, false, 1>), dim3(full1), dim3(256), 0, 0, s, d, n16); break;
    case 4: hipLaunchKernelGGL((copy_t<u32x4, true, 4>), dim3(full4), dim3(256), 0, 0, s, d, n16); break;
    case 5: hipLaunchKernelGGL((copy_t<u32x4, false, 4>), dim3(full4), dim3(256), 0, 0, s, d, n16); break;
    case 6: hipLaunchKernelGGL((copy_t<u32x4, false, 8>), dim3(4096), dim3(256), 0, 0, s, d, n16); break;
    default: hipLaunchKernelGGL((copy_t<u32x4, false, 2>), dim3(8192), dim3(256), 0, 0, s, d, n16); break;
  }
}

// Average time of `iters` launches of copy variant `variant` (0..7) over `bytes`.
extern "C" int copy_ceiling_run(int variant, const void* src, void* dst, uint64_t bytes,
                                int iters, float* ms_per_iter) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch_variant(variant, src, dst, bytes);
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < iters; ++i) launch_variant(variant, src, dst, bytes);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  *ms_per_iter = ms / iters;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
