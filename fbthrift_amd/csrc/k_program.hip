// k_program.hip — compiled-program decode of variable-length records over an
// indexed stream (BASELINE configs 3 and 4: Compact {4 x i32, 2 x string},
// Binary {i64, list<i32>, Inner{3 x double}}).
//
// The host compiles the schema into a VProgram: the canonical wire form of a
// record as the generated readNoXfer's fast path expects it (one expected
// header per field in declaration order; advanceToNextField,
// BinaryProtocol-inl.h:586-621 / CompactProtocol-inl.h:811-872), followed by
// each value's encoding. Here one lane runs the program over one record:
//   * a workgroup stages its tile's bytes [offs[r0], offs[r0+256]) HBM -> LDS
//     with coalesced 16-byte loads (any tile larger than kWireCap falls back);
//   * each lane reads its record from LDS through 8-byte windows (aligned
//     dword reads + v_alignbyte), decodes varints branch-free (7-bit group
//     compaction of the window), and writes the record into an LDS record
//     tile (strings become zero-copy views; list elements go to the arena);
//   * the record tile goes LDS -> HBM with coalesced 16-byte stores.
// A record that deviates from the canonical form in any way (other field
// order, unknown/missing fields, long-form varints past the fast window,
// limits, sizes, truncation, index mismatch) is NOT decided here: its index is
// appended to a list and the general decoder (full readNoXfer semantics,
// tgpu_device.h) decodes it, so results and errors are exactly the reference's.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "tgpu_device.h"
#include "tgpu_prog_kernels.h"

namespace tgpu {
namespace {

using prog::kPT;

__global__ __launch_bounds__(kPT) void program_decode_kernel(DecodeArgs a,
                                                             const VProgram* __restrict__ pp,
                                                             uint32_t S, uint32_t wire_cap,
                                                             uint64_t* __restrict__ irr,
                                                             unsigned long long* __restrict__ nirr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  prog::decode_tile(a, prog::DynProg{pp}, S, wire_cap, irr, nirr, smem);
}

template <int Pr>
__global__ __launch_bounds__(256) void general_decode_list_kernel(DecodeArgs a,
                                                                  const uint64_t* __restrict__ list,
                                                                  const unsigned long long* nlist) {
  const uint64_t m = *nlist;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) {
    const uint64_t i = list[k];
    const dev::Reader r = dev::decode_record<Pr>(a, i, -1);
    if (!r.ok()) dev::defer_or_fail(r, a.deep, &a.res->first_fail, i);
  }
}

}  // namespace

// LDS wire tile of the indexed decode, sized for occupancy: the kernel is
// latency-bound, so the cap is the largest that still lets the most
// workgroups share a CU while holding a tile of >= 1.04 x the batch's mean
// tile + 256 B (the rare larger tile takes the general decoder); within that,
// at most 1.12 x mean + 512 B. (A/B on MI355X, tools/kbench_prog.py: config 3
// 1.64 -> 1.45 ms going from the old fixed 1.3 x mean + 1 KiB to 5
// workgroups/CU.) TGPU_PROG_DECODE="factor,pad" overrides the upper bound.
// span_bytes: the wire bytes of the n records (0: a.in_len).
int64_t device_lds_per_cu() {
  static const int64_t v = [] {
    int dev = 0, x = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&x, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) ==
            hipSuccess &&
        x > 0)
      return (int64_t)x;
    return (int64_t)163840;
  }();
  return v;
}
uint32_t lds_per_block_limit() {
  static const uint32_t v = [] {
    int dev = 0, x = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&x, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess &&
        x > 0)
      return (uint32_t)x;
    return 0u;
  }();
  return v;
}

uint32_t program_decode_wire_cap(const DecodeArgs& a, uint32_t rec_size, uint64_t span_bytes,
                                 bool regrec, uint32_t extra) {
  double factor = 1.12, pad = 512.0;
  if (const char* e = getenv("TGPU_PROG_DECODE")) sscanf(e, "%lf,%lf", &factor, &pad);
  const double span = (double)(span_bytes ? span_bytes : a.in_len);
  const double mean = span / (double)(a.n ? a.n : 1) * kPT;
  const double lo = 1.04 * mean + 256.0, hi = std::max(factor * mean + pad, lo);
  const uint32_t rt = (regrec ? 0u : prog::decode_rtile_bytes(rec_size)) + extra;
  const double cu = (double)device_lds_per_cu();
  double cap = hi;
  for (uint32_t w = 8; w >= 1; --w) {
    // wire bytes that fit w workgroups (the region is whole 4 KiB staging rounds)
    const double room = std::floor((cu / w - rt) / 4096.0) * 4096.0 - 32.0;
    if (room >= lo) {
      cap = std::min(room, hi);
      break;
    }
  }
  cap = cap < 4096.0 ? 4096.0 : (cap > 40960.0 ? 40960.0 : cap);
  return ((uint32_t)cap) & ~15u;
}

uint32_t program_decode_lds(uint32_t wire_cap, uint32_t rec_size, bool regrec = false,
                            uint32_t extra = 0) {
  return prog::decode_wire_region(wire_cap) + (regrec ? 0u : prog::decode_rtile_bytes(rec_size)) +
         extra;
}

hipError_t launch_program_decode(const DecodeArgs& a, const VProgram* d_prog, uint32_t rec_size,
                                 uint64_t* irregular, unsigned long long* n_irregular,
                                 hipStream_t stream, const JitKernels* jit, uint64_t span_bytes) {
  if (a.n == 0) return hipSuccess;
  // the block rule: compiled Binary programs with lists pack their blocks
  // in the decode tile (pack_wave, no extra LDS); the library's interpreting
  // kernel leaves the packing to arena_pack_kernel
  DecodeArgs b = a;
  if (!jit || !b.pack_flags || !b.pack_k) b.pack_flags = nullptr, b.pack_k = 0;
  const uint32_t extra = 0;
  uint32_t cap = program_decode_wire_cap(b, rec_size, span_bytes, false, extra);
  const uint64_t tiles = (a.n + kPT - 1) / kPT;
  uint32_t lds = program_decode_lds(cap, rec_size, false, extra);
  // Records in registers (entry 2) where the LDS record tile holds the tile
  // down to 3 workgroups per CU or fewer, dropping it fits more, and records
  // are whole 64-byte halves of a cache line: config 4 (S 64) 1.86 -> 1.69 ms
  // (3 -> 5 workgroups); config 2's S 72 records at the same residency
  // measured slower (indexed 2.15 -> 2.39 ms: per-lane stores straddling
  // lines), and at 5 workgroups (config 3) the per-lane record stores cost
  // more than the residency gains (1.46 -> 1.78 ms).
  // TGPU_DECODE_REGREC=0 / 1 forces it off / on (A/B).
  if (jit && jit_has(jit, 2)) {
    const char* v = getenv("TGPU_DECODE_REGREC");
    const uint32_t cap2 = program_decode_wire_cap(b, rec_size, span_bytes, true, extra);
    const uint32_t lds2 = program_decode_lds(cap2, rec_size, true, extra);
    const uint32_t cu = (uint32_t)device_lds_per_cu();
    const uint32_t w1 = cu / lds, w2 = cu / lds2;
    const bool rr = v ? v[0] == '1' : (rec_size % 64 == 0 && w1 <= 3 && w2 > w1);
    if (rr)
      return jit_launch_decode(jit, b, tiles, cap2, lds2, irregular, n_irregular, stream, 2);
  }
  if (jit) return jit_launch_decode(jit, b, tiles, cap, lds, irregular, n_irregular, stream);
  hipLaunchKernelGGL(program_decode_kernel, dim3((uint32_t)tiles), dim3(kPT), lds, stream, b,
                     d_prog, rec_size, cap, irregular, n_irregular);
  return hipGetLastError();
}

// The strided tail decode's tile: records up to L + 32 bytes (a second
// stride of appended fields), within the program decode's 40 KiB wire tile
// beside the record tile — sized so 3 workgroups share a CU where the record
// tile allows (the persistent grid fills the CUs once).
uint32_t stream_tail_wire_cap(uint32_t rec_size, uint32_t L) {
  const uint32_t rt = (kPT * rec_size + 16 + 15) & ~15u;
  if (rt + 8192 > 163840) return 0;
  const uint32_t room = (163840 - rt) / 4096 * 4096 - 32;
  const uint32_t want = kPT * (L + 32) + 16;
  return std::min<uint32_t>(std::min<uint32_t>(room, want), 40960) & ~15u;
}

uint64_t stream_tail_max_stride(uint32_t rec_size, uint32_t L) {
  const uint32_t cap = stream_tail_wire_cap(rec_size, L);
  return cap > 16 ? (cap - 16) / kPT : 0;
}

hipError_t launch_stream_tail_decode(const DecodeArgs& a, uint32_t rec_size, uint32_t L,
                                     uint64_t* irr, unsigned long long* nirr, hipStream_t stream,
                                     const JitKernels* J, int device) {
  const uint32_t cap = stream_tail_wire_cap(rec_size, L);
  if (!cap || !jit_has(J, 1)) return hipSuccess;
  const uint32_t lds = program_decode_lds(cap, rec_size);
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      cus <= 0)
    cus = 256;
  // persistent: the workgroups one pass of the CUs holds (they loop over the
  // tail's tiles; with no tail every one returns at once)
  const uint64_t grid = (uint64_t)cus * std::max<uint32_t>(1, 163840 / lds);
  return jit_launch_decode(J, a, grid, cap, lds, irr, nirr, stream, 1);
}

hipError_t launch_general_decode_list(const DecodeArgs& a, int protocol, const uint64_t* list,
                                      const unsigned long long* n_list, hipStream_t stream) {
  // (a grid-stride loop over the list: few workgroups keep the general
  // reader's scratch backing small, k_index.hip SCRATCH_KERNEL; 4 x
  // kScratchGrid still covers a list of every record at a quarter wave per CU)
  const uint64_t b = (a.n + 255) / 256;
  const uint64_t cap = 4ull * kScratchGrid;
  const uint32_t g = (uint32_t)(b < cap ? (b ? b : 1) : cap);
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(general_decode_list_kernel<P_>, dim3(g), dim3(256), 0,
                       stream, a, list, n_list));
  return hipGetLastError();
}

}  // namespace tgpu
