// glds_probe.hip — does an LDS-DMA (global_load_lds_dwordx4) write land in LDS
// after the issuing waves' `s_waitcnt vmcnt(0)` + `s_barrier`?
//
// Each workgroup stages a tile of `tile` bytes of a large buffer into LDS
// (whole waves by LDS-DMA, the last partial wave through registers: the
// staging of the stream index), passes __syncthreads(), and every thread
// hashes its words of the tile twice: right after the barrier and again after
// a second barrier. Threads whose two hashes differ saw the tile change after
// the staging barrier. mode 0: LDS-DMA; 1: register staging; 2: LDS-DMA, then
// each wave reads back its own last DMA'd vector (ds_read + lgkmcnt(0))
// before the barrier; 3: LDS-DMA, then s_sleep before the first hash; 4:
// LDS-DMA with heavy LDS traffic (bank-conflicting ds_or) by every wave after
// its DMAs are issued and again after the barrier, as in the stream index's
// tiles; 5: mode 4's traffic with register staging.
// Built into tools/build/libglds_probe.so; bench/diagnostic only.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr uint32_t kT = 256;
constexpr uint32_t kMaxTile = 20 * 1024;

__global__ __launch_bounds__(kT) void probe_kernel(const uint8_t* __restrict__ src, uint64_t len,
                                                   uint32_t tile, uint32_t stride, int mode,
                                                   unsigned long long* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kMaxTile + 32];
  __shared__ uint32_t busy[2048];
  const uint64_t lo = (uint64_t)blockIdx.x * stride;  // (stride < tile: tiles overlap)
  if (lo >= len) return;
  const uint32_t bytes = (uint32_t)min((uint64_t)tile, len - lo);
  const uint32_t nvec = (bytes + 15) >> 4;
  const uint4* g = (const uint4*)(src + lo);
  const uint32_t whole = (mode == 1 || mode == 5) ? 0u : (nvec & ~63u);
  const uint32_t wave = threadIdx.x >> 6;
  uint32_t last = ~0u;
  for (uint32_t k = 0; k * kT < whole; ++k) {
    const uint32_t w0 = k * kT + wave * 64;
    if (w0 < whole) {
      __builtin_amdgcn_global_load_lds((const void*)(g + w0 + (threadIdx.x & 63)),
                                       (__attribute__((address_space(3))) void*)(lds + (size_t)w0 * 16),
                                       16, 0, 0);
      last = w0 + (threadIdx.x & 63);
    }
  }
  for (uint32_t i = whole + threadIdx.x; i < nvec; i += kT) ((uint4*)lds)[i] = g[i];
  if (mode >= 4)  // LDS traffic (32-way bank conflicts) while the DMAs are in flight
    for (uint32_t r = 0; r < 64; ++r) atomicOr(&busy[((threadIdx.x * 32) + r) & 2047], r);
  if (mode == 2 && last != ~0u) {
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0) (all counters)
    const uint32_t v = ((volatile uint32_t*)lds)[last * 4];
    if (v == 0x12345678u && bytes == 1) out[3] = v;  // (keeps the read)
  }
  __syncthreads();
  if (mode == 3) __builtin_amdgcn_s_sleep(10);
  if (mode >= 4)
    for (uint32_t r = 0; r < 64; ++r) atomicOr(&busy[((threadIdx.x * 32) + r * 7) & 2047], r);
  const uint32_t nw = bytes >> 2;
  uint32_t h0 = 0, h1 = 0, hg = 0;
  for (uint32_t d = threadIdx.x; d < nw; d += kT) h0 ^= ((volatile uint32_t*)lds)[d] * (d | 1);
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < nw; d += kT) {
    h1 ^= ((volatile uint32_t*)lds)[d] * (d | 1);
    hg ^= ((const uint32_t*)(src + lo))[d] * (d | 1);
  }
  if (h0 != h1) atomicAdd(&out[0], 1ull);  // threads that saw the tile change
  if (h0 != hg) atomicAdd(&out[1], 1ull);  // ... whose first read differs from HBM
  if (h1 != hg) atomicAdd(&out[2], 1ull);  // ... whose second read differs from HBM
}
}  // namespace

// Runs the probe over [0, len) of src `reps` times; out[0..3) summed.
// refresh != NULL: before every launch the buffer is rewritten from refresh
// (a device copy: the probe then reads bytes another kernel just wrote, as the
// stream index reads the encoder's output)
extern "C" int glds_probe_run(const void* src, uint64_t len, uint32_t tile, uint32_t stride,
                              int mode, int reps, const void* refresh,
                              unsigned long long* host_out) {
  if (tile > kMaxTile || tile % 16) return 1;
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 4 * sizeof(unsigned long long)) != hipSuccess) return 2;
  hipMemset(d, 0, 4 * sizeof(unsigned long long));
  const uint64_t blocks = (len + stride - 1) / stride;
  for (int r = 0; r < reps; ++r) {
    if (refresh) (void)hipMemcpyAsync((void*)src, refresh, len, hipMemcpyDeviceToDevice, 0);
    hipLaunchKernelGGL(probe_kernel, dim3((uint32_t)blocks), dim3(kT), 0, 0, (const uint8_t*)src,
                       len, tile, stride, mode, d);
  }
  const hipError_t e = hipMemcpy(host_out, d, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  hipFree(d);
  return e == hipSuccess ? 0 : 3;
}
