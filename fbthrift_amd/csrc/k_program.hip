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

#include "tgpu_program.h"

namespace tgpu {
namespace {

constexpr uint32_t kPT = 256;               // records per tile = threads per workgroup
constexpr uint32_t kWireCap = 26 * 1024;    // default LDS bytes for one tile's wire bytes

template <bool kSProg, bool kDirect>
__global__ __launch_bounds__(kPT) void program_decode_kernel(DecodeArgs a,
                                                             const VProgram* __restrict__ pp,
                                                             uint32_t S, uint32_t wire_cap,
                                                             uint64_t* __restrict__ irr,
                                                             unsigned long long* __restrict__ nirr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* wire = smem;                                   // wire_cap + 32
  uint8_t* rtile = smem + wire_cap + 32;                  // kPT * S (+16), unless kDirect
  VProgram* P = (VProgram*)(rtile + (kDirect ? 0u : ((kPT * S + 16 + 15) & ~15u)));

  const uint64_t r0 = (uint64_t)blockIdx.x * kPT;
  const uint32_t nrec = (uint32_t)min((uint64_t)kPT, a.n - r0);
  const uint64_t t0 = a.offs[r0], t1 = a.offs[r0 + nrec];
  const bool tile_ok = t1 >= t0 && t1 <= a.in_len && (t1 - t0) + 16 <= wire_cap;
  uint32_t sh = 0;
  if (tile_ok) {
    const uint8_t* g = a.in + t0;
    sh = (uint32_t)((uintptr_t)g & 15);
    const uint4* src = (const uint4*)(g - sh);
    const uint32_t nvec = (uint32_t)((t1 - t0) + sh + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nvec; i += kPT) ((uint4*)wire)[i] = src[i];
  }
  uint8_t* gout = a.recs + r0 * S;
  const uint32_t osh = (uint32_t)((uintptr_t)gout & 15);
  if (!kDirect) {
    const uint4 z = {0u, 0u, 0u, 0u};
    const uint32_t nz = (kPT * S + osh + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nz; i += kPT) ((uint4*)rtile)[i] = z;
  }
  if (!kSProg)
    for (uint32_t i = threadIdx.x; i < (uint32_t)(sizeof(VProgram) / 16); i += kPT)
      ((uint4*)P)[i] = ((const uint4*)pp)[i];
  __syncthreads();

  const uint32_t r = threadIdx.x;
  if (r < nrec) {
    // kDirect: the lane default-initializes its record in HBM and the program
    // stores members straight there (no LDS record tile: higher occupancy)
    uint8_t* rec = kDirect ? gout + r * S : rtile + osh + r * S;
    if (kDirect) {
      if ((((uintptr_t)rec | S) & 7) == 0) {
        for (uint32_t b = 0; b < S; b += 8) *(unsigned long long*)(rec + b) = 0;
      } else if ((((uintptr_t)rec | S) & 3) == 0) {
        for (uint32_t b = 0; b < S; b += 4) *(uint32_t*)(rec + b) = 0;
      } else {
        for (uint32_t b = 0; b < S; ++b) rec[b] = 0;
      }
    }
    bool ok = tile_ok;
    if (ok) {
      const uint64_t s = a.offs[r0 + r], e = a.offs[r0 + r + 1];
      ok = s >= t0 && e >= s && e <= t1;
      if (ok) {
        const prog::Ctx c{t0 - sh, a.arena, a.arena_cap, a.string_limit, a.container_limit};
        const prog::LdsSrc src{(const uint32_t*)wire};
        uint32_t p = (uint32_t)(s - t0) + sh;
        const uint32_t pe = (uint32_t)(e - t0) + sh;
        if (kSProg)
          ok = prog::run_program<true>(pp, src, c, p, pe, rec) && p == pe;
        else
          ok = prog::run_program<true>((const VProgram*)P, src, c, p, pe, rec) && p == pe;
      }
    }
    if (!ok) {
      const unsigned long long k = atomicAdd(nirr, 1ull);
      irr[k] = r0 + r;
    }
  }
  if (kDirect) return;
  __syncthreads();
  // record tile -> HBM
  const uint32_t end = osh + nrec * S;
  const uint32_t nvec = (end + 15) >> 4;
  for (uint32_t i = threadIdx.x; i < nvec; i += kPT) {
    const uint32_t lo = i << 4, hi = lo + 16;
    uint8_t* base = gout - osh;
    if (lo >= osh && hi <= end) {
      ((uint4*)base)[i] = ((const uint4*)rtile)[i];
    } else {
      for (uint32_t b = (lo < osh ? osh : lo); b < (hi < end ? hi : end); ++b) base[b] = rtile[b];
    }
  }
}

template <int Pr>
__global__ __launch_bounds__(256) void general_decode_list_kernel(DecodeArgs a,
                                                                  const uint64_t* __restrict__ list,
                                                                  const unsigned long long* nlist) {
  const uint64_t m = *nlist;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) {
    const uint64_t i = list[k];
    uint8_t* rec = a.recs + i * a.rec_size;
    for (uint32_t b = 0; b < a.rec_size; ++b) rec[b] = 0;
    const uint64_t start = a.offs[i];
    dev::Reader r;
    r.p = a.in;
    r.pos = start;
    r.end = a.in_len;
    r.height = (int64_t)(a.height ? a.height : a.max_depth) + 1;
    r.string_limit = a.string_limit;
    r.container_limit = a.container_limit;
    r.max_depth = a.max_depth;
    r.err = 0;
    r.err_off = 0;
    r.has_bool = false;
    r.bool_val = false;
    if (start > a.in_len || (a.check_index && a.offs[i + 1] < start)) {
      r.fail(TGPU_ERR_INDEX_MISMATCH, start);
    } else {
      dev::read_record<Pr>(r, a.sc, rec, a.arena, a.arena_cap);
      if (r.ok() && a.check_index && r.pos != a.offs[i + 1]) r.fail(TGPU_ERR_INDEX_MISMATCH, r.pos);
    }
    if (!r.ok()) atomicMin(&a.res->first_fail, (unsigned long long)i);
  }
}

}  // namespace

// Variant (A/B tuning, env TGPU_PROG_DECODE="sprog,capmode"): sprog = read the
// program through the scalar cache instead of an LDS copy; capmode 1 = size
// the LDS wire tile from the batch's mean record length (in_len / n) instead
// of the fixed kWireCap.
// Defaults = A/B winners (profiles/r01_kbench_prog.log): scalar-cache
// program, mean-sized wire tile, LDS record tile (direct HBM stores of
// 56-byte records are 1.9x slower: partial-line writes).
struct ProgVariant {
  int sprog = 1, capmode = 1, direct = 0;
};
static ProgVariant prog_variant() {
  ProgVariant v;
  if (const char* e = getenv("TGPU_PROG_DECODE"))
    sscanf(e, "%d,%d,%d", &v.sprog, &v.capmode, &v.direct);
  return v;
}

hipError_t launch_program_decode(const DecodeArgs& a, const VProgram* d_prog, uint32_t rec_size,
                                 uint64_t* irregular, unsigned long long* n_irregular,
                                 hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  const ProgVariant v = prog_variant();
  uint32_t cap = kWireCap;
  if (v.capmode) {
    // mean tile + 30 % + 1 KiB headroom (capmode 2: + 12 % + 512 B); tiles
    // beyond it take the general decoder
    const double mean = (double)a.in_len / (double)a.n;
    const double want = v.capmode == 1 ? 1.3 * kPT * mean + 1024.0 : 1.12 * kPT * mean + 512.0;
    cap = (uint32_t)(want < 4096.0 ? 4096.0 : (want > 40960.0 ? 40960.0 : want));
    cap = (cap + 15) & ~15u;
  }
  const uint32_t rt = v.direct ? 0u : (kPT * rec_size + 16 + 15) & ~15u;
  const uint32_t lds = cap + 32 + rt + (v.sprog ? 0 : (uint32_t)sizeof(VProgram));
  const dim3 grid((uint32_t)((a.n + kPT - 1) / kPT)), block(kPT);
  if (v.sprog && v.direct)
    hipLaunchKernelGGL((program_decode_kernel<true, true>), grid, block, lds, stream, a, d_prog,
                       rec_size, cap, irregular, n_irregular);
  else if (v.sprog)
    hipLaunchKernelGGL((program_decode_kernel<true, false>), grid, block, lds, stream, a, d_prog,
                       rec_size, cap, irregular, n_irregular);
  else if (v.direct)
    hipLaunchKernelGGL((program_decode_kernel<false, true>), grid, block, lds, stream, a, d_prog,
                       rec_size, cap, irregular, n_irregular);
  else
    hipLaunchKernelGGL((program_decode_kernel<false, false>), grid, block, lds, stream, a, d_prog,
                       rec_size, cap, irregular, n_irregular);
  return hipGetLastError();
}

hipError_t launch_general_decode_list(const DecodeArgs& a, int protocol, const uint64_t* list,
                                      const unsigned long long* n_list, hipStream_t stream) {
  const uint64_t b = (a.n + 255) / 256;
  const uint32_t g = (uint32_t)(b < 2048 ? (b ? b : 1) : 2048);
  if (protocol == TGPU_PROTOCOL_BINARY)
    hipLaunchKernelGGL(general_decode_list_kernel<TGPU_PROTOCOL_BINARY>, dim3(g), dim3(256), 0,
                       stream, a, list, n_list);
  else
    hipLaunchKernelGGL(general_decode_list_kernel<TGPU_PROTOCOL_COMPACT>, dim3(g), dim3(256), 0,
                       stream, a, list, n_list);
  return hipGetLastError();
}

}  // namespace tgpu
