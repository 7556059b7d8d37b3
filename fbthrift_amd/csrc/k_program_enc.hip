// k_program_enc.hip — compiled-program encode of variable-length records
// (BASELINE configs 3 and 4 encode), plus the multi-block scan of per-tile
// byte counts shared with the general encoder.
//
// The schema's VProgram (tgpu_api.cpp build_program) is the canonical wire
// form the generated T::write emits for an all-unqualified schema: fields in
// declaration order (serialize_struct.whisker:40-67), each header
// (BinaryProtocol-inl.h:41-67 / CompactProtocol-inl.h:133-180) then its value
// (BinaryProtocol-inl.h:120-222 / CompactProtocol-inl.h:252-373).
//
// One record per lane, 256-record tiles (bodies in tgpu_prog_kernels.h):
//   1. program_size_kernel — record tile HBM -> LDS; each lane sizes its
//      record; sizes -> out_offsets[i]; tile sum -> block_sums[t];
//      validation failures (validate_bool, > INT32_MAX sizes) -> first_fail.
//   2. scan_tiles_* — exclusive scan of the tile sums (tile stream offsets).
//   3. program_write_kernel — record tile -> LDS again, block scan of the
//      sizes, records emitted into a zero-filled LDS output tile a dword at a
//      time, coalesced 16-byte stores; out_offsets receives every start.
// tgpu_encoded_size stops after 2.
#include <cstdlib>
#include <cstring>

#include "tgpu_prog_kernels.h"

namespace tgpu {
namespace {

using prog::block_exscan256;
using prog::kET;
using prog::kOutCap;

__global__ __launch_bounds__(kET) void program_size_kernel(EncodeArgs a,
                                                           const VProgram* __restrict__ P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ unsigned long long part[4];
  prog::size_tile(a, prog::DynProg{P}, a.rec_size, smem, part);
}

__global__ __launch_bounds__(kET) void program_write_kernel(EncodeArgs a,
                                                            const VProgram* __restrict__ P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ prog::EncodeShared sm;
  prog::write_tile(a, prog::DynProg{P}, a.rec_size, smem, sm);
}

// ---- scan of per-tile sums (exclusive, in place; total -> res, offs[n]) ----
constexpr uint32_t kScanChunk = 2048;  // sums per workgroup (8 per thread)

__global__ __launch_bounds__(256) void scan_tiles_reduce(const unsigned long long* __restrict__ sums,
                                                         uint64_t nb,
                                                         unsigned long long* __restrict__ part) {
  __shared__ unsigned long long wp[4];
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanChunk;
  unsigned long long s = 0;
  for (uint32_t j = 0; j < kScanChunk / 256; ++j) {
    const uint64_t k = b0 + j * 256 + threadIdx.x;
    if (k < nb) s += sums[k];
  }
  unsigned long long total;
  (void)block_exscan256(s, wp, &total);
  if (threadIdx.x == 0) part[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void scan_tiles_top(unsigned long long* part, uint64_t np,
                                                       unsigned long long* total1,
                                                       uint64_t* total2) {
  __shared__ unsigned long long sm[1024];
  const uint64_t per = (np + 1023) / 1024;
  const uint64_t b = threadIdx.x * per, e = min(np, b + per);
  unsigned long long s = 0;
  for (uint64_t k = b; k < e; ++k) s += part[k];
  sm[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const unsigned long long y = threadIdx.x >= (unsigned)o ? sm[threadIdx.x - o] : 0;
    __syncthreads();
    sm[threadIdx.x] += y;
    __syncthreads();
  }
  unsigned long long run = sm[threadIdx.x] - s;
  for (uint64_t k = b; k < e; ++k) {
    const unsigned long long v = part[k];
    part[k] = run;
    run += v;
  }
  if (threadIdx.x == 1023) {
    if (total1) *total1 = sm[1023];
    if (total2) *total2 = sm[1023];
  }
}

__global__ __launch_bounds__(256) void scan_tiles_apply(unsigned long long* __restrict__ sums,
                                                        uint64_t nb,
                                                        const unsigned long long* __restrict__ part) {
  __shared__ unsigned long long wp[4];
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanChunk + threadIdx.x * (kScanChunk / 256);
  unsigned long long v[kScanChunk / 256];
  unsigned long long s = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanChunk / 256; ++j) {
    v[j] = b0 + j < nb ? sums[b0 + j] : 0;
    s += v[j];
  }
  unsigned long long total;
  unsigned long long run = part[blockIdx.x] + block_exscan256(s, wp, &total);
#pragma unroll
  for (uint32_t j = 0; j < kScanChunk / 256; ++j) {
    if (b0 + j < nb) sums[b0 + j] = run;
    run += v[j];
  }
}

}  // namespace

hipError_t launch_scan_tiles(unsigned long long* sums, uint64_t nb, unsigned long long* part,
                             unsigned long long* total1, uint64_t* total2, hipStream_t stream) {
  const uint64_t np = (nb + kScanChunk - 1) / kScanChunk;
  hipLaunchKernelGGL(scan_tiles_reduce, dim3((uint32_t)np), dim3(256), 0, stream, sums, nb, part);
  hipLaunchKernelGGL(scan_tiles_top, dim3(1), dim3(1024), 0, stream, part, np, total1, total2);
  hipLaunchKernelGGL(scan_tiles_apply, dim3((uint32_t)np), dim3(256), 0, stream, sums, nb, part);
  return hipGetLastError();
}

uint64_t scan_tiles_parts(uint64_t nb) { return (nb + kScanChunk - 1) / kScanChunk; }

bool program_encode_fits(uint32_t rec_size) {
  return kET * rec_size + 32 <= 32 * 1024;  // record tile + 24 KiB output tile <= 64 KiB LDS
}

// LDS of the compiled write kernel's element stage: prog::kElemStage, or a
// "#define TGPU_ELEM_STAGE n" in TGPU_JIT_DEFINES (A/B runs, tools/kbench_jit.py)
static uint32_t elem_stage_bytes() {
  uint32_t n = prog::kElemStage;
  if (const char* d = getenv("TGPU_JIT_DEFINES")) {
    if (const char* k = strstr(d, "TGPU_ELEM_STAGE")) n = (uint32_t)strtoul(k + 15, nullptr, 10);
  }
  return n;
}

// The single-pass compiled encode (write_tile_one) only under
// TGPU_ENCODE_ONEPASS=1: measured slower than the size pass + tile scan +
// write pass on configs 3 and 4
static bool encode_onepass() {
  const char* s = getenv("TGPU_ENCODE_ONEPASS");
  return s && *s == '1';
}

hipError_t launch_program_encode(const EncodeArgs& a, const VProgram* d_prog,
                                 unsigned long long* part, bool size_only, hipStream_t stream,
                                 const JitKernels* jit) {
  if (a.n == 0) return hipSuccess;
  const uint64_t tiles = (a.n + kET - 1) / kET;
  const uint32_t rt = prog::enc_record_region(a.rec_size);
  hipError_t e;
  if (jit) {
    // the compiled write pass sizes its own records (tile sums suffice)
    EncodeArgs x = a;
    x.recompute = size_only ? 0u : 1u;
    if (!size_only && encode_onepass() && jit_has(jit, 2) && !x.fixed_len) {
      // one pass (tgpu_prog_kernels.h write_tile_one): block_sums become the
      // tiles' look-back status words
      e = hipMemsetAsync(a.block_sums, 0, tiles * sizeof(unsigned long long), stream);
      if (e != hipSuccess) return e;
      return jit_launch_encode(jit, false, x, tiles,
                               (x.out_cap ? x.out_cap : kOutCap) + 32 + elem_stage_bytes(), stream,
                               2);
    }
    e = jit_launch_encode(jit, false, x, tiles, rt, stream);
    if (e == hipSuccess)
      e = launch_scan_tiles(a.block_sums, tiles, part, &a.res->total_bytes, a.offs + a.n, stream);
    if (e != hipSuccess || size_only) return e;
    return jit_launch_encode(jit, true, x, tiles,
                             (x.out_cap ? x.out_cap : kOutCap) + 32 + elem_stage_bytes(), stream);
  } else {
    hipLaunchKernelGGL(program_size_kernel, dim3((uint32_t)tiles), dim3(kET), rt, stream, a,
                       d_prog);
    e = hipGetLastError();
  }
  if (e == hipSuccess)
    e = launch_scan_tiles(a.block_sums, tiles, part, &a.res->total_bytes, a.offs + a.n, stream);
  if (e != hipSuccess || size_only) return e;
  const uint32_t lds = rt + kOutCap + 32;
  hipLaunchKernelGGL(program_write_kernel, dim3((uint32_t)tiles), dim3(kET), lds, stream, a,
                     d_prog);
  return hipGetLastError();
}

hipError_t launch_program_write_fixed(const EncodeArgs& a, const VProgram* d_prog,
                                      hipStream_t stream, const JitKernels* jit) {
  if (a.n == 0) return hipSuccess;
  const uint64_t tiles = (a.n + kET - 1) / kET;
  const uint32_t rt = prog::enc_record_region(a.rec_size);
  if (jit) return jit_launch_encode(jit, true, a, tiles, kOutCap + 32, stream);
  hipLaunchKernelGGL(program_write_kernel, dim3((uint32_t)tiles), dim3(kET), rt + kOutCap + 32,
                     stream, a, d_prog);
  return hipGetLastError();
}

}  // namespace tgpu
