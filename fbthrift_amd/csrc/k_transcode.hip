// k_transcode.hip — the wire-to-wire transcoder's launch sequence
// (tgpu_xcode.h) and its general-reader / general-writer kernels for the
// records the programs cannot take:
//   xc_one (program pair, single pass: decode, size, look back, emit) — done
//   unless it listed records; otherwise, or without the single pass:
//   xc_size (program pair)  -> general decode of the listed records into the
//   record workspace (+ deep pass) -> xc_irr_size (their target sizes, added
//   to the tiles' sums) -> tile scan -> xc_write (program pair; holes for the
//   listed records) -> xc_irr_write (general writer into the holes) ->
//   xc_finish (status: the first record whose read or write failed).
// The program pair is the schema compiler's (JIT_XCODE) or, below its
// batch threshold / without hipRTC, the AOT DynProg instantiation here.
#include <algorithm>
#include <cstdlib>

#include "tgpu_device.h"
#include "tgpu_xcode.h"

namespace tgpu {
namespace {

using prog::kPT;

__global__ __launch_bounds__(kPT) void xc_size_kernel(XcodeArgs x, const VProgram* __restrict__ ps,
                                                      const VProgram* __restrict__ pd, uint32_t S,
                                                      uint32_t wire_cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ unsigned long long part[4];
  prog::xc_size_tile<prog::DynProg, prog::DynProg, 0>(x, prog::DynProg{ps}, prog::DynProg{pd}, S,
                                                      wire_cap, smem, part);
}

__global__ __launch_bounds__(kPT) void xc_write_kernel(XcodeArgs x, const VProgram* __restrict__ ps,
                                                       const VProgram* __restrict__ pd, uint32_t S,
                                                       uint32_t wire_cap, uint32_t ocap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ prog::EncodeShared sm;
  prog::xc_write_tile<prog::DynProg, prog::DynProg, 0>(x, prog::DynProg{ps}, prog::DynProg{pd}, S,
                                                       wire_cap, ocap, smem, sm);
}

__global__ __launch_bounds__(kPT) void xc_one_kernel(XcodeArgs x, const VProgram* __restrict__ ps,
                                                     const VProgram* __restrict__ pd, uint32_t S,
                                                     uint32_t wire_cap, uint32_t ocap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ prog::EncodeShared sm;
  prog::xc_one_tile<prog::DynProg, prog::DynProg, 0>(x, prog::DynProg{ps}, prog::DynProg{pd}, S,
                                                     wire_cap, ocap, smem, sm);
}

// The listed records' target sizes (decoded by the general reader into
// e.recs): e.offs[r] = size, added to the tile's sum before the scan. A
// record at or past the first read failure is not written (size 0).
template <int P>
__global__ __launch_bounds__(256) void xc_irr_size_kernel(EncodeArgs e, const uint64_t* __restrict__ irr,
                                                          const unsigned long long* nirr) {
  const uint64_t m = *nirr;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) {
    const uint64_t r = irr[k];
    if (r >= e.res->first_fail) {
      e.offs[r] = 0;
      continue;
    }
    dev::Writer w{nullptr, 0, 0, 0, 0};
    dev::write_record<P>(w, e.sc, e.recs + r * e.rec_size, e.sbase, e.lbase);
    if (!w.ok()) {
      atomicMin(&e.res->first_fail, (unsigned long long)r);
      e.offs[r] = 0;
      continue;
    }
    e.offs[r] = w.pos;
    atomicAdd(&e.block_sums[r / kPT], (unsigned long long)w.pos);
  }
}

// The listed records written into the holes the write pass left for them.
template <int P>
__global__ __launch_bounds__(256) void xc_irr_write_kernel(EncodeArgs e, const uint64_t* __restrict__ irr,
                                                           const unsigned long long* nirr) {
  const uint64_t m = *nirr;
  const uint64_t f = e.res->first_fail;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) {
    const uint64_t r = irr[k];
    if (r >= f) continue;
    dev::Writer w{e.out, e.offs[r], e.cap, 0, 0};
    dev::write_record<P>(w, e.sc, e.recs + r * e.rec_size, e.sbase, e.lbase);
  }
}

// Status: the first failing record — a read failure (re-read for its exact
// code and input byte offset, decode_finish_kernel's rule) or an output that
// does not fit (TGPU_ERR_OUTPUT_OVERFLOW at its output start); the records
// before it are written, total_bytes = their output bytes.
template <int P>
__global__ void xc_finish_kernel(XcodeArgs x) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DevResult* res = x.d.res;
  const uint64_t f = res->first_fail;
  if (f < x.d.n) {
    const dev::Reader r = dev::decode_record<P>(x.d, f, 0);
    const uint64_t start = x.e.offs[f];
    res->code = r.ok() ? TGPU_ERR_OUTPUT_OVERFLOW : r.err;
    res->fail_offset = r.ok() ? start : r.err_off;
    res->n_records = f;
    res->total_bytes = start;
  } else {
    res->code = 0;
    res->n_records = x.d.n;
  }
}

uint32_t list_grid(uint64_t n) {
  const uint64_t b = (n + 255) / 256;
  const uint64_t cap = 4ull * kScratchGrid;
  return (uint32_t)(b < cap ? (b ? b : 1) : cap);
}

}  // namespace

// LDS of the two tile passes: the source wire tile (program_decode_wire_cap's
// occupancy rule for the decode's tile), the record tile (AOT pair) and, in
// the write pass, the output tile.
uint32_t program_decode_wire_cap(const DecodeArgs& a, uint32_t rec_size, uint64_t span_bytes,
                                 bool regrec, uint32_t extra);

hipError_t launch_xcode(const XcodeArgs& x, int from, int to, const VProgram* d_ps,
                        const VProgram* d_pd, hipStream_t s, const JitKernels* jit) {
  const uint64_t n = x.d.n;
  if (n == 0) return hipSuccess;
  const uint32_t S = x.d.rec_size;
  const bool rr = jit && jit_has(jit, 2);  // records in registers (S <= 128, S % 8 == 0)
  const uint32_t rt = rr ? 0u : prog::xc_rec_region(S, 0);
  uint32_t cap = program_decode_wire_cap(x.d, S, 0, rr, 0);
  // output tile: the encoder's 24 KiB (a record past it goes to HBM
  // directly), or — sized with the wire tile for the most workgroups per CU
  // that hold 1.04 x the mean tile of each (x.out_mean: the host's estimate)
  // — what that residency leaves. (Config 3, Compact -> Binary: 16 KiB wire +
  // 24 KiB output + the static LDS crossed 40 KiB, 3 workgroups per CU.)
  uint32_t ocap = prog::kOutCap;
  if (x.out_mean) {
    const double in_tile = (double)x.d.in_len / (double)n * kPT;
    const double want_w = 1.04 * in_tile + 256.0, max_w = 1.12 * in_tile + 512.0;
    const double want_o = std::min(1.04 * (double)x.out_mean * kPT + 256.0, (double)prog::kOutCap);
    // (no w that holds both: the sizes above)
    const int64_t cu_lds = device_lds_per_cu();
    for (uint32_t w = 8; w >= 1; --w) {
      const int64_t budget = cu_lds / w - 256 - (int64_t)rt;  // (static LDS, slack)
      const uint32_t rw = prog::decode_wire_region((uint32_t)want_w);
      // the largest wire cap within the staging rounds the tile needs (at
      // least 4 KiB); the fit is checked on the region that cap really takes
      uint32_t c = std::min<uint32_t>((uint32_t)max_w, rw - 32) & ~15u;
      c = std::max(c, std::min<uint32_t>((uint32_t)want_w, rw - 32) & ~15u);
      c = std::max<uint32_t>(c, 4096);
      const int64_t room = budget - (int64_t)prog::decode_wire_region(c) - 32;
      if ((double)room < want_o || room < (int64_t)kMinXcodeOut) continue;
      cap = c;
      ocap = (uint32_t)std::min<int64_t>(prog::kOutCap, room) & ~15u;
      break;
    }
  }
  if (lds_per_block_limit() && prog::decode_wire_region(cap) + rt + ocap + 32 >
                                   lds_per_block_limit()) {
    // (a device with less LDS than the sizes above: the encoder's own tile
    // sizes, or whatever the block limit leaves of them)
    const int64_t room = (int64_t)lds_per_block_limit() -
                         (int64_t)prog::decode_wire_region(cap) - (int64_t)rt - 32;
    ocap = (uint32_t)std::max<int64_t>(std::min<int64_t>(room, prog::kOutCap), 0) & ~15u;
  }
  if (const char* v = getenv("TGPU_XC_OCAP"))  // (A/B)
    if (*v) ocap = (uint32_t)atoi(v) & ~15u;
  const uint32_t lds_a = prog::decode_wire_region(cap) + rt;
  const uint32_t lds_c = lds_a + ocap + 32;
  const uint64_t tiles = (n + kPT - 1) / kPT;
  hipError_t e;
  XcodeArgs y = x;  // (the two-pass kernels: gated behind a single pass)
  y.gate = x.xstat ? x.xstat + tiles : nullptr;
  if (x.xstat) {
    // single pass; the kernels below it find nothing to do unless it listed
    // records or a wait passed its bound (the gate word)
    e = hipMemsetAsync(x.xstat, 0, (tiles + 1) * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    if (jit && jit_has(jit, rr ? 5 : 4)) {
      e = jit_launch_xcode(jit, rr ? 5 : 4, x, tiles, cap, ocap, lds_c, s);
    } else {
      hipLaunchKernelGGL(xc_one_kernel, dim3((uint32_t)tiles), dim3(kPT), lds_c, s, x, d_ps, d_pd,
                         S, cap, ocap);
      e = hipGetLastError();
    }
  } else if (jit) {
    e = jit_launch_xcode(jit, rr ? 2 : 0, x, tiles, cap, ocap, lds_a, s);
  } else {
    hipLaunchKernelGGL(xc_size_kernel, dim3((uint32_t)tiles), dim3(kPT), lds_a, s, x, d_ps, d_pd, S,
                       cap);
    e = hipGetLastError();
  }
  if (e != hipSuccess) return e;
  // the listed records: general reader into the record workspace (deep pass
  // for a skip nested past the private frames), then their target sizes
  DecodeArgs d = x.d;
  d.check_index = 1;
  e = launch_general_decode_list(d, from, x.irr, x.nirr, s);
  if (e == hipSuccess) e = launch_deep_decode(d, from, s);
  if (e != hipSuccess) return e;
  const uint32_t g = list_grid(n);
  TGPU_BY_PROTOCOL(to, hipLaunchKernelGGL(xc_irr_size_kernel<P_>, dim3(g), dim3(256), 0, s, x.e,
                                          x.irr, x.nirr));
  e = hipGetLastError();
  if (e == hipSuccess)
    e = launch_scan_tiles(x.e.block_sums, tiles, x.e.scan_part, &x.d.res->total_bytes,
                          x.want_offs ? x.e.offs + n : nullptr, s);
  if (e != hipSuccess) return e;
  if (jit) {
    e = jit_launch_xcode(jit, rr ? 3 : 1, y, tiles, cap, ocap, lds_c, s);
  } else {
    hipLaunchKernelGGL(xc_write_kernel, dim3((uint32_t)tiles), dim3(kPT), lds_c, s, y, d_ps, d_pd,
                       S, cap, ocap);
    e = hipGetLastError();
  }
  if (e != hipSuccess) return e;
  TGPU_BY_PROTOCOL(to, hipLaunchKernelGGL(xc_irr_write_kernel<P_>, dim3(g), dim3(256), 0, s, x.e,
                                          x.irr, x.nirr));
  TGPU_BY_PROTOCOL(from, hipLaunchKernelGGL(xc_finish_kernel<P_>, dim3(1), dim3(64), 0, s, x));
  return hipGetLastError();
}

}  // namespace tgpu
