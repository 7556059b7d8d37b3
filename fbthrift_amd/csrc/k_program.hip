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

#include "tgpu_device.h"

namespace tgpu {
namespace {

constexpr uint32_t kPT = 256;               // records per tile = threads per workgroup
constexpr uint32_t kWireCap = 26 * 1024;    // default LDS bytes for one tile's wire bytes

__device__ __forceinline__ uint64_t win8(const uint32_t* w32, uint32_t p) {
  const uint32_t d = p >> 2, s = p & 3;
  const uint32_t W0 = w32[d], W1 = w32[d + 1], W2 = w32[d + 2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(W1, W0, s);
  const uint32_t hi = __builtin_amdgcn_alignbyte(W2, W1, s);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t bswap_n(uint64_t x, uint32_t width) {
  // the first `width` bytes of x (little-endian packed) as a big-endian number
  const uint64_t b = __builtin_bswap64(x);
  return width == 8 ? b : (b >> (64 - 8 * width));
}

// LEB128 at p (VarintUtils-inl.h:94-134): up to 8 bytes from one window,
// 9-10 byte i64 varints byte-wise. Returns false (irregular) on anything the
// fast path does not take (past `end`, more than ceil(bits/7) bytes).
__device__ __forceinline__ bool read_varint(const uint32_t* w32, uint32_t& p, uint32_t end,
                                            uint32_t bits, uint64_t& v) {
  const uint64_t w = win8(w32, p);
  const uint64_t stop = ~w & 0x8080808080808080ull;
  if (stop) {
    const uint32_t len = ((uint32_t)__builtin_ctzll(stop) >> 3) + 1;
    if (p + len > end || (bits == 32 && len > 5)) return false;
    uint64_t x = (len == 8 ? w : (w & ((1ull << (8 * len)) - 1))) & 0x7f7f7f7f7f7f7f7full;
    x = ((x & 0x7f007f007f007f00ull) >> 1) | (x & 0x007f007f007f007full);
    x = ((x & 0x3fff00003fff0000ull) >> 2) | (x & 0x00003fff00003fffull);
    x = ((x & 0x0fffffff00000000ull) >> 4) | (x & 0x000000000fffffffull);
    v = bits == 32 ? (x & 0xffffffffull) : x;
    p += len;
    return true;
  }
  if (bits == 32) return false;
  // i64 varint of 9 or 10 bytes: 8 continuation bytes so far
  uint64_t x = 0;
  for (uint32_t i = 0; i < 10; ++i) {
    if (p + i >= end) return false;
    const uint64_t b = (win8(w32, p + i) & 0xff);
    x |= (b & 0x7f) << (7 * i);
    if (!(b & 0x80)) {
      v = x;
      p += i + 1;
      return true;
    }
  }
  return false;
}

__device__ __forceinline__ void store_n(uint8_t* dst, uint64_t v, uint32_t width) {
  switch (width) {
    case 8: *(uint64_t*)dst = v; break;
    case 4: *(uint32_t*)dst = (uint32_t)v; break;
    case 2: *(uint16_t*)dst = (uint16_t)v; break;
    default: *dst = (uint8_t)v; break;
  }
}

__device__ __forceinline__ uint64_t unzigzag(uint64_t z, uint32_t bits) {
  if (bits == 32) {
    const uint32_t n = (uint32_t)z;
    return (uint64_t)(int64_t)(int32_t)((n >> 1) ^ (0u - (n & 1)));
  }
  return (z >> 1) ^ (0ull - (z & 1));
}

struct Ctx {
  const uint32_t* w32;   // LDS wire tile
  uint64_t gbase;        // stream offset of LDS byte 0
  uint8_t* arena;
  uint64_t arena_cap;
  int32_t string_limit, container_limit;
};

// Runs the program over [p, end) (LDS positions); writes into rec (LDS).
// PP: the program in LDS (VProgram*) or in HBM read through the scalar cache
// (const VProgram* __restrict__ kernel argument).
template <class PP>
__device__ bool run_program(PP P, const Ctx& c, uint32_t p, uint32_t end, uint8_t* rec) {
  const bool compact = P->protocol == TGPU_PROTOCOL_COMPACT;
  const uint32_t n_ops = P->n_ops;
  for (uint32_t k = 0; k < n_ops; ++k) {
    const VOp op = P->ops[k];
    switch (op.kind) {
      case VOP_CONST: {
        if (p + op.hdr_len > end) return false;
        const uint32_t lo = (uint32_t)win8(c.w32, p);
        const uint32_t mask = op.hdr_len >= 4 ? 0xffffffffu : ((1u << (8 * op.hdr_len)) - 1);
        if ((lo ^ op.hdr) & mask) return false;
        p += op.hdr_len;
        break;
      }
      case VOP_CBOOL: {
        if (p + op.hdr_len > end) return false;
        const uint32_t lo = (uint32_t)win8(c.w32, p);
        const uint32_t mask = (op.hdr_len >= 4 ? 0xffffffffu : ((1u << (8 * op.hdr_len)) - 1)) & ~0xfu;
        const uint32_t ct = lo & 0xf;
        if (((lo ^ op.hdr) & mask) || (ct != 1 && ct != 2)) return false;
        rec[op.member] = ct == 1 ? 1 : 0;
        p += op.hdr_len;
        break;
      }
      case VOP_FIXED: {
        if (p + op.width > end) return false;
        const uint64_t v = bswap_n(win8(c.w32, p), op.width);
        if (op.is_bool && v > 1) return false;  // readBool throws: general path
        store_n(rec + op.member, v, op.width);
        p += op.width;
        break;
      }
      case VOP_VARINT: {
        uint64_t z;
        if (!read_varint(c.w32, p, end, op.bits, z)) return false;
        store_n(rec + op.member, unzigzag(z, op.bits), op.width);
        break;
      }
      case VOP_STRING: {
        int64_t len;
        if (compact) {
          uint64_t z;
          if (!read_varint(c.w32, p, end, 32, z)) return false;
          len = (int32_t)(uint32_t)z;
        } else {
          if (p + 4 > end) return false;
          len = (int32_t)(uint32_t)bswap_n(win8(c.w32, p), 4);
          p += 4;
        }
        if (len < 0 || (c.string_limit > 0 && len > c.string_limit) || p + len > end) return false;
        tgpu_span* sp = (tgpu_span*)(rec + op.member);
        sp->offset = len ? c.gbase + p : 0;
        sp->length = (uint32_t)len;
        sp->reserved = 0;
        p += (uint32_t)len;
        break;
      }
      case VOP_LIST: {
        int64_t n;
        if (compact) {
          if (p + 1 > end) return false;
          const uint32_t b = (uint32_t)(win8(c.w32, p) & 0xff);
          const uint32_t ct = b & 0xf;
          const bool ok_ct = op.elem_ttype == TGPU_T_BOOL ? (ct == 1 || ct == 2) : ct == op.elem_ct;
          if (!ok_ct) return false;
          ++p;
          n = b >> 4;
          if (n == 15) {
            uint64_t z;
            if (!read_varint(c.w32, p, end, 32, z)) return false;
            n = (int32_t)(uint32_t)z;
          }
        } else {
          if (p + 5 > end) return false;
          const uint64_t w = win8(c.w32, p);
          if ((w & 0xff) != op.elem_ttype) return false;
          n = (int32_t)(uint32_t)bswap_n(w >> 8, 4);
          p += 5;
        }
        if (n < 0 || (c.container_limit && n > c.container_limit) || n > (int64_t)(end - p))
          return false;
        const uint64_t scale = compact ? 8 : 1;
        const uint64_t aoff = scale * (c.gbase + p);
        const uint32_t es = op.width;
        if (n && (!c.arena || aoff + (uint64_t)n * es > c.arena_cap)) return false;
        for (int64_t i = 0; i < n; ++i) {
          uint64_t v;
          if (op.elem_kind == VEL_VARINT) {
            uint64_t z;
            if (!read_varint(c.w32, p, end, op.bits, z)) return false;
            v = unzigzag(z, op.bits);
          } else {
            const uint32_t wb = op.elem_kind == VEL_BOOL ? 1 : es;
            if (p + wb > end) return false;
            v = bswap_n(win8(c.w32, p), wb);
            if (op.elem_kind == VEL_BOOL) {
              if (compact) v = v == 1;
              else if (v > 1) return false;
            }
            p += wb;
          }
          store_n(c.arena + aoff + (uint64_t)i * es, v, es);
        }
        tgpu_span* sp = (tgpu_span*)(rec + op.member);
        sp->offset = n ? aoff : 0;
        sp->length = (uint32_t)n;
        sp->reserved = 0;
        break;
      }
      case VOP_ISSET:
        break;
      default:
        return false;
    }
    if (op.isset != 0xffff) rec[op.isset] = 1;
  }
  return p == end;
}

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
        Ctx c{(const uint32_t*)wire, t0 - sh, a.arena, a.arena_cap, a.string_limit,
              a.container_limit};
        if (kSProg)
          ok = run_program(pp, c, (uint32_t)(s - t0) + sh, (uint32_t)(e - t0) + sh, rec);
        else
          ok = run_program((const VProgram*)P, c, (uint32_t)(s - t0) + sh,
                           (uint32_t)(e - t0) + sh, rec);
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
