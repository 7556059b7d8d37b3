// k_index.hip — record index of an unindexed stream: the bulk form of the
// reference's file-reading loop `while (!cursor.isAtEnd()) deserialize<T>(c)`
// (Serializer.h:97-100), which is sequential because record k+1 starts where
// record k's readNoXfer stopped. Here the dependency is broken by speculation:
//
//   1. index_spec_kernel — one lane per chunk of `chunk` bytes. The lane tries
//      candidate starts (chunk 0 of a non-speculative call: `begin` only) and
//      accepts the first from which records parse back to back to the chunk's
//      end, the first record in the canonical form (tgpu_program.h) and the
//      rest canonical or, failing that, read by the general reader (exact
//      readNoXfer consumption, tgpu_device.h). Result per chunk: s (first
//      start), e (first start at or past the chunk's end), cnt (records).
//   2. index_flag_kernel + scan + index_list_kernel — chunks whose link is
//      broken (s[j] != e[j-1], or nothing accepted) in ascending order.
//   3. index_fix_kernel — one lane walks the broken links in order from the
//      true start, re-parses each with the general reader and follows the
//      cascade until the chain agrees again; the first reader error ends the
//      stream exactly where the reference would throw.
//   4. scan of the per-chunk counts, index_emit_kernel writes every start
//      (one lane per chunk, re-walking its chain), index_finish_kernel writes
//      the end, the status and (decode) pads the index to the requested count.
// Speculation only decides speed: every chunk the result uses was either
// parsed from its verified true start or is linked to one by s[j] == e[j-1].
#include "tgpu_program.h"

namespace tgpu {
namespace {

constexpr uint64_t kNo = ~0ull;        // no start found / unset
constexpr uint64_t kErr = ~0ull - 1;   // chain ended in a reader error
constexpr uint64_t kPartial = ~0ull - 2;  // program stopped: general reader continues
constexpr uint64_t kLanesValid = ~0ull - 3;  // pf: the tile's per-lane results are current
constexpr uint32_t kPosCap = 0x7fffff00u;

__device__ __forceinline__ dev::Reader reader_at(const IndexArgs& a, uint64_t pos) {
  dev::Reader r;
  r.p = a.in;
  r.pos = pos;
  r.end = a.in_len;
  r.height = (int64_t)(a.height ? a.height : a.max_depth) + 1;
  r.string_limit = a.string_limit;
  r.container_limit = a.container_limit;
  r.max_depth = a.max_depth;
  r.err = 0;
  r.err_off = 0;
  r.has_bool = false;
  r.bool_val = false;
  return r;
}

struct Chain {
  uint64_t end;    // first record start >= hi (or the failing record's start)
  uint64_t count;  // records parsed
  int32_t code;    // reader error (0: none)
  uint64_t err_off;
};

// Records back to back from p while p < hi. canonical_first: the first record
// must match the program (speculation); returns false if it does not.
// emit: record starts written to emit[0..) (at most emit_cap).
template <int P>
__device__ bool chain(const IndexArgs& a, uint64_t p, uint64_t hi, bool canonical_first,
                      uint8_t* scratch, Chain& out, uint64_t* emit, uint64_t emit_cap,
                      uint64_t max_count) {
  out.count = 0;
  out.code = 0;
  out.err_off = 0;
  const prog::Ctx pc{0, nullptr, 0, a.string_limit, a.container_limit};
  while (p < hi && out.count < max_count) {
    uint64_t q = 0;
    bool ok = false;
    if (a.prog && p < a.in_len) {
      const uint64_t avail = a.in_len - p;
      const prog::HbmSrc src{a.in + p, (uint32_t)(avail < kPosCap ? avail : kPosCap)};
      uint32_t rel = 0;
      ok = prog::run_program<false>(a.prog, src, pc, rel, src.avail, nullptr);
      q = p + rel;
    }
    if (!ok) {
      // speculation: a candidate start must open with a canonical record
      // (schemas without a program: any record the reader accepts)
      if (canonical_first && out.count == 0 && a.prog) return false;
      dev::Reader r = reader_at(a, p);
      dev::read_record<P>(r, a.sc, scratch, nullptr, kDiscardArena);
      if (!r.ok()) {
        if (canonical_first && out.count == 0) return false;
        out.code = r.err;
        out.err_off = r.err_off;
        out.end = p;
        return true;
      }
      q = r.pos;
    }
    if (emit && out.count < emit_cap) emit[out.count] = p;
    ++out.count;
    p = q;
  }
  out.end = p;
  return true;
}

// Program-only chain (light: no general reader, so the speculation and emit
// kernels keep a small register footprint): records back to back from p while
// p < hi and fewer than max_count; stops early (*stuck) at the first record
// the program does not take, p then being that record's start.
__device__ __forceinline__ uint64_t prog_chain(const IndexArgs& a, uint64_t& p, uint64_t hi,
                                               uint64_t max_count, uint64_t* emit,
                                               uint64_t emit_cap, bool& stuck) {
  const prog::Ctx pc{0, nullptr, 0, a.string_limit, a.container_limit};
  uint64_t count = 0;
  stuck = false;
  while (p < hi && count < max_count) {
    if (p >= a.in_len) {
      stuck = true;
      break;
    }
    const uint64_t avail = a.in_len - p;
    const prog::HbmSrc src{a.in + p, (uint32_t)(avail < kPosCap ? avail : kPosCap)};
    uint32_t rel = 0;
    if (!prog::run_program<false>(a.prog, src, pc, rel, src.avail, nullptr)) {
      stuck = true;
      break;
    }
    if (emit && count < emit_cap) emit[count] = p;
    ++count;
    p += rel;
  }
  return count;
}

__device__ __forceinline__ uint64_t chunk_lo(const IndexArgs& a, uint64_t j) {
  return a.begin + j * a.chunk;
}
__device__ __forceinline__ uint64_t chunk_hi(const IndexArgs& a, uint64_t j) {
  const uint64_t h = a.begin + (j + 1) * a.chunk;
  return h < a.end ? h : a.end;
}

// Speculation, program-only (schemas with a program). A chain the program
// cannot finish is accepted as partial (e = kPartial, pf = where it stopped)
// when at least its first record was canonical; index_cont_kernel finishes it.
__global__ __launch_bounds__(256) void index_spec_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n_chunks) return;
  const uint64_t lo = chunk_lo(a, j), hi = chunk_hi(a, j);
  bool stuck;
  if (j == 0 && !a.speculative) {
    uint64_t p = a.begin;
    a.cnt[0] = prog_chain(a, p, hi, kNo, nullptr, 0, stuck);
    a.s[0] = a.begin;
    a.e[0] = stuck ? kPartial : p;
    a.pf[0] = p;
    return;
  }
  const uint64_t w = j == 0 ? a.chunk : a.window;  // a shard's first record may start late
  const uint64_t last = lo + w < hi ? lo + w : hi;
  // candidates are the positions holding the program's first header byte,
  // found 8 bytes per load (zero-byte test on w ^ broadcast(h0))
  const uint64_t h0 = a.prog->ops[0].kind == VOP_CONST ? (a.prog->ops[0].hdr & 0xff) : 0x100;
  const prog::HbmSrc src{a.in + lo, (uint32_t)(a.in_len - lo < kPosCap ? a.in_len - lo : kPosCap)};
  for (uint64_t base = lo; base < last; base += 8) {
    uint64_t m;
    if (h0 < 0x100) {
      const uint64_t x = src.win8((uint32_t)(base - lo)) ^ (h0 * 0x0101010101010101ull);
      m = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
    } else {
      m = 0x8080808080808080ull;  // CBOOL first: every position is a candidate
    }
    while (m) {
      const uint64_t cand = base + ((uint32_t)__builtin_ctzll(m) >> 3);
      m &= m - 1;
      if (cand >= last) break;
      uint64_t p = cand;
      const uint64_t c = prog_chain(a, p, hi, kNo, nullptr, 0, stuck);
      if (c == 0) continue;  // the candidate's first record is not canonical
      a.s[j] = cand;
      a.e[j] = stuck ? kPartial : p;
      a.pf[j] = p;
      a.cnt[j] = c;
      return;
    }
  }
  a.s[j] = kNo;
  a.e[j] = kNo;
  a.cnt[j] = 0;
}

// Finishes partial chains with the general reader (program first per record).
// A reader error rejects a speculated start (kNo: the repair pass decides);
// from a verified start (chunk 0 of a non-speculative call) it is final (kErr).
template <int P>
__global__ __launch_bounds__(256) void index_cont_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n_chunks || a.e[j] != kPartial) return;
  Chain c;
  chain<P>(a, a.pf[j], chunk_hi(a, j), false, a.scratch + j * a.rec_size, c, nullptr, 0, kNo);
  if (c.code) {
    if (j == 0 && !a.speculative) {
      a.e[0] = kErr;
    } else {
      a.s[j] = kNo;
      a.e[j] = kNo;
      a.cnt[j] = 0;
    }
    return;
  }
  a.e[j] = c.end;
  a.cnt[j] += c.count;
  a.pf[j] = 0;
}

// Speculation for schemas without a program: any record the general reader
// accepts may open a chain.
template <int P>
__global__ __launch_bounds__(256) void index_spec_general_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n_chunks) return;
  uint8_t* scratch = a.scratch + j * a.rec_size;
  const uint64_t lo = chunk_lo(a, j), hi = chunk_hi(a, j);
  Chain c;
  if (j == 0 && !a.speculative) {
    chain<P>(a, a.begin, hi, false, scratch, c, nullptr, 0, kNo);
    a.s[0] = a.begin;
    a.e[0] = c.code ? kErr : c.end;
    a.cnt[j] = c.count;
    return;
  }
  const uint64_t w = j == 0 ? a.chunk : a.window;
  const uint64_t last = lo + w < hi ? lo + w : hi;
  for (uint64_t cand = lo; cand < last; ++cand) {
    if (chain<P>(a, cand, hi, true, scratch, c, nullptr, 0, kNo) && c.code == 0) {
      a.s[j] = cand;
      a.e[j] = c.end;
      a.cnt[j] = c.count;
      return;
    }
  }
  a.s[j] = kNo;
  a.e[j] = kNo;
  a.cnt[j] = 0;
}

// ---- LDS tiles (schemas with a program) --------------------------------------
// A chunk is a tile of kTile bytes handled by one workgroup: the tile (plus
// kOver bytes for the records that straddle its end) is staged in LDS with
// coalesced 16-byte loads; lane k speculates the first record start in its
// kSub-byte slice and chains to the slice's end; the lanes' links are then
// repaired inside the workgroup (lane k restarts from lane k-1's end until
// no lane changes), so the tile behaves like one chunk of the lane path:
// (first start, end, count). A tile any lane could not finish with the
// program is handed to the general-reader kernels whole (kPartial).
constexpr uint32_t kTileLanes = 256;
constexpr uint32_t kSub = 64;
constexpr uint32_t kTile = kTileLanes * kSub;
constexpr uint32_t kOver = 4096;
constexpr uint32_t kTileLds = kTile + kOver + 32;

// LDS window with HBM fallback past the staged bytes (positions relative to
// the 16-byte aligned tile base)
struct TileSrc {
  const uint32_t* w32;
  uint32_t lds_len;
  prog::HbmSrc g;
  __device__ __forceinline__ uint64_t win8(uint32_t p) const {
    if (p + 12 <= lds_len) return prog::LdsSrc{w32}.win8(p);
    return g.win8(p);
  }
};

struct TileLane {
  uint32_t s, e, c;  // first start, end, count (tile-relative); s == kNoPos: none
  bool stuck;
};
constexpr uint32_t kNoPos = 0xffffffffu;

// Cheap rejection of a candidate start before running the program: the byte
// after the first header's value must be the second header (first ops
// CONST, VARINT|FIXED, CONST — every schema whose first two fields are
// unqualified scalars). Never rejects a canonical record start.
__device__ __forceinline__ bool quick_reject(const VProgram* __restrict__ P, const TileSrc& src,
                                             uint32_t cand) {
  if (P->n_ops < 3 || P->ops[0].kind != VOP_CONST || P->ops[2].kind != VOP_CONST) return false;
  const uint32_t h0len = P->ops[0].hdr_len;
  const VOp v = P->ops[1];
  const uint64_t w = src.win8(cand + h0len);
  uint32_t len;
  if (v.kind == VOP_VARINT) {
    const uint64_t stop = ~w & 0x8080808080808080ull;
    if (!stop) return false;
    len = ((uint32_t)__builtin_ctzll(stop) >> 3) + 1;
  } else if (v.kind == VOP_FIXED) {
    len = v.width;
  } else {
    return false;
  }
  if (len >= 8) return false;
  return ((w >> (8 * len)) & 0xff) != (P->ops[2].hdr & 0xff);
}

// chain of canonical records from x while position < hi (tile-relative)
__device__ __forceinline__ void tile_chain(const VProgram* __restrict__ P, const TileSrc& src,
                                           const prog::Ctx& pc, uint32_t x, uint32_t hi,
                                           uint32_t end, TileLane& L, uint64_t* emit) {
  L.s = x;
  L.c = 0;
  L.stuck = false;
  uint32_t p = x;
  while (p < hi) {
    uint32_t q = p;
    if (!prog::run_program<false>(P, src, pc, q, end, nullptr)) {
      L.stuck = true;
      break;
    }
    if (emit) emit[L.c] = p;
    ++L.c;
    p = q;
  }
  L.e = p;
}

// Stages the tile, speculates and repairs the lanes' chains. entry: the
// tile's known first start (tile-relative; kNoPos: speculate lane 0 too).
// Returns false when the tile needs the general reader. *first: the tile's
// first record start (kNoPos: none).
__device__ __forceinline__ bool tile_resolve(const IndexArgs& a, uint64_t j, uint8_t* lds, uint32_t entry,
                             TileLane& L, uint32_t& sh, uint32_t& first, uint32_t* E,
                             int* flag) {
  const uint64_t lo = chunk_lo(a, j);
  const uint64_t hi_abs = chunk_hi(a, j);
  const uint8_t* g = a.in + lo;
  sh = (uint32_t)((uintptr_t)g & 15);
  const uint8_t* gb = g - sh;
  const uint64_t avail64 = a.in_len - lo + sh;
  const uint32_t avail = (uint32_t)(avail64 < kPosCap ? avail64 : kPosCap);
  const uint32_t staged = avail < kTile + kOver + 16 ? avail : kTile + kOver + 16;
  const uint32_t nvec = (staged + 15) >> 4;
  for (uint32_t i = threadIdx.x; i < nvec; i += kTileLanes)
    ((uint4*)lds)[i] = ((const uint4*)gb)[i];
  __syncthreads();
  const TileSrc src{(const uint32_t*)lds, staged & ~3u, prog::HbmSrc{gb, avail}};
  const prog::Ctx pc{0, nullptr, 0, a.string_limit, a.container_limit};
  const uint32_t thi = sh + (uint32_t)(hi_abs - lo);  // tile end (relative)
  const uint32_t k = threadIdx.x;
  const uint32_t sub_lo = sh + k * kSub;
  const uint32_t sub_hi = sub_lo + kSub < thi ? sub_lo + kSub : thi;
  L.s = kNoPos;
  L.e = kNoPos;
  L.c = 0;
  L.stuck = false;
  if (k == 0 && entry != kNoPos) {
    tile_chain(a.prog, src, pc, entry, sub_hi > entry ? sub_hi : entry, avail, L, nullptr);
    if (entry >= sub_hi) {  // the entry lies past lane 0's slice
      L.s = entry;
      L.e = entry;
    }
  } else if (sub_lo < thi) {
    // candidates: bytes equal to the first header byte that survive
    // quick_reject (divergent but cheap); the chain from a candidate runs
    // outside the search so all lanes of the wave run it together
    const uint32_t h0 = a.prog->ops[0].kind == VOP_CONST ? (a.prog->ops[0].hdr & 0xff) : 0x100;
    // bytes of the slice equal to h0, all eight 8-byte groups loaded at once
    uint64_t mk[kSub / 8];
#pragma unroll
    for (uint32_t i = 0; i < kSub / 8; ++i) {
      const uint32_t base = sub_lo + 8 * i;
      uint64_t m = 0;
      if (base < sub_hi) {
        m = 0x8080808080808080ull;
        if (h0 < 0x100) {
          const uint64_t x = src.win8(base) ^ (h0 * 0x0101010101010101ull);
          m = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
        }
      }
      mk[i] = m;
    }
    uint32_t from = sub_lo;
    bool need = true;
    while (need) {
      uint32_t cand = kNoPos;
#pragma unroll
      for (uint32_t i = 0; i < kSub / 8; ++i) {
        uint64_t m = mk[i];
        while (m && cand == kNoPos) {
          const uint32_t c = sub_lo + 8 * i + ((uint32_t)__builtin_ctzll(m) >> 3);
          m &= m - 1;
          if (c < from || c >= sub_hi) continue;
          if (quick_reject(a.prog, src, c)) continue;
          cand = c;
        }
      }
      if (cand == kNoPos) break;  // no record start in this slice
      TileLane t;
      tile_chain(a.prog, src, pc, cand, sub_hi, avail, t, nullptr);
      if (t.c) {
        L = t;
        need = false;
      } else {
        from = cand + 1;
      }
    }
  }
  // the tile's first start: the first lane that found one
  __shared__ uint32_t first_lane;
  if (k == 0) first_lane = kTileLanes;
  __syncthreads();
  if (L.s != kNoPos) atomicMin(&first_lane, k);
  __syncthreads();
  const uint32_t f = first_lane;
  if (f == kTileLanes) {
    first = kNoPos;
    return true;
  }
  // lanes before it: no record starts there
  __shared__ uint32_t fs;
  if (k == f) fs = L.s;
  __syncthreads();
  if (k < f) {
    L.s = L.e = fs;
    L.c = 0;
    L.stuck = false;
  }
  first = fs;
  // repair: lane k restarts from lane k-1's end until nothing changes
  for (uint32_t it = 0; it <= kTileLanes; ++it) {
    E[k] = L.e;
    __syncthreads();
    int changed = 0;
    if (k > f) {
      const uint32_t x = E[k - 1];
      if (x != kNoPos && (x != L.s || L.e == kNoPos)) {
        if (x >= sub_hi) {
          L.s = L.e = x;
          L.c = 0;
          L.stuck = false;
        } else {
          tile_chain(a.prog, src, pc, x, sub_hi, avail, L, nullptr);
        }
        changed = 1;
      }
    }
    if (!__syncthreads_or(changed)) break;
  }
  *flag = 0;
  __syncthreads();
  if (L.stuck || L.e == kNoPos) *flag = 1;
  __syncthreads();
  return *flag == 0;
}

__global__ __launch_bounds__(kTileLanes) void index_tile_spec_kernel(IndexArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kTileLds];
  __shared__ uint32_t E[kTileLanes];
  __shared__ int flag;
  __shared__ unsigned long long csum;
  const uint64_t j = blockIdx.x;
  const uint32_t entry = (j == 0 && !a.speculative) ? 0u : kNoPos;  // + sh below
  TileLane L;
  uint32_t sh, first;
  // tile 0 of a non-speculative call starts at begin exactly (relative 0 + sh)
  uint32_t ent = entry;
  if (ent != kNoPos) ent = (uint32_t)((uintptr_t)(a.in + chunk_lo(a, j)) & 15);
  const bool ok = tile_resolve(a, j, lds, ent, L, sh, first, E, &flag);
  const uint64_t lo = chunk_lo(a, j);
  if (threadIdx.x == 0) csum = 0;
  __syncthreads();
  if (ok && first != kNoPos) atomicAdd(&csum, (unsigned long long)L.c);
  __syncthreads();
  // per-lane starts/counts for the emit pass (valid while the tile keeps this
  // start: pf[j] == kLanesValid)
  if (ok && first != kNoPos)
    a.lanes[j * kTileLanes + threadIdx.x] = (L.s & 0xffffu) | ((uint32_t)L.c << 16);
  if (threadIdx.x == kTileLanes - 1) {
    if (first == kNoPos) {
      a.s[j] = kNo;
      a.e[j] = kNo;
      a.cnt[j] = 0;
    } else if (!ok) {
      // the general reader walks the whole tile from its (speculated) start
      a.s[j] = lo - sh + first;
      a.e[j] = kPartial;
      a.pf[j] = lo - sh + first;
      a.cnt[j] = 0;
    } else {
      a.s[j] = lo - sh + first;
      a.e[j] = lo - sh + L.e;
      a.cnt[j] = csum;
      a.pf[j] = kLanesValid;
    }
  }
}

// Emit for a tile whose first start is verified (a.s[j]); records starting in
// the tile get their starts written at offs[base[j] ..]. A tile the program
// cannot finish goes to index_emit_cont_kernel whole.
__global__ __launch_bounds__(kTileLanes) void index_tile_emit_kernel(IndexArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kTileLds];
  __shared__ uint32_t E[kTileLanes];
  __shared__ int flag;
  __shared__ unsigned long long part[4];
  const uint64_t j = blockIdx.x;
  if (threadIdx.x == 0) a.ep[j] = kNo;
  if (j >= a.scal[1] || a.cnt[j] == 0) return;
  const uint64_t lo = chunk_lo(a, j);
  const uint32_t sh0 = (uint32_t)((uintptr_t)(a.in + lo) & 15);
  const uint64_t sj = a.s[j];
  const uint32_t ent = (uint32_t)(sj - lo) + sh0;
  TileLane L;
  uint32_t sh, first;
  bool ok;
  if (a.pf[j] == kLanesValid) {
    // the speculation pass's lane results still hold: stage the tile only
    const uint8_t* g = a.in + lo;
    sh = sh0;
    const uint8_t* gb = g - sh;
    const uint64_t av = a.in_len - lo + sh;
    const uint32_t avail = (uint32_t)(av < kPosCap ? av : kPosCap);
    const uint32_t staged = avail < kTile + kOver + 16 ? avail : kTile + kOver + 16;
    const uint32_t nvec = (staged + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nvec; i += kTileLanes)
      ((uint4*)lds)[i] = ((const uint4*)gb)[i];
    const uint32_t v = a.lanes[j * kTileLanes + threadIdx.x];
    L.s = v & 0xffffu;
    L.c = v >> 16;
    first = ent;
    ok = true;
    __syncthreads();
  } else {
    ok = tile_resolve(a, j, lds, ent, L, sh, first, E, &flag);
  }
  const uint64_t b = a.base[j];
  if (!ok) {
    if (threadIdx.x == 0) {
      a.ep[j] = sj;
      a.ec[j] = 0;
    }
    return;
  }
  // lane k's records go after the records of lanes < k
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long x = L.c;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) part[wid] = x;
  __syncthreads();
  unsigned long long pre = x - L.c;
  for (int w = 0; w < wid; ++w) pre += part[w];
  if (L.c == 0) return;
  // re-walk this lane's records, writing absolute starts
  const uint64_t gb = lo - sh;
  uint32_t p = L.s;
  const uint8_t* g = a.in + gb;
  const uint64_t avail64 = a.in_len - gb;
  const uint32_t avail = (uint32_t)(avail64 < kPosCap ? avail64 : kPosCap);
  const uint32_t staged = avail < kTile + kOver + 16 ? avail : kTile + kOver + 16;
  const TileSrc src{(const uint32_t*)lds, staged & ~3u, prog::HbmSrc{g, avail}};
  const prog::Ctx pc{0, nullptr, 0, a.string_limit, a.container_limit};
  for (uint32_t i = 0; i < L.c; ++i) {
    const uint64_t idx = b + pre + i;
    if (idx <= a.max_records) a.offs[idx] = gb + p;
    uint32_t q = p;
    prog::run_program<false>(a.prog, src, pc, q, avail, nullptr);
    p = q;
  }
}

__device__ __forceinline__ bool link_broken(const IndexArgs& a, uint64_t j) {
  const uint64_t e = a.e[j];
  if (e == kNo || e == kErr || e == kPartial) return true;
  if (j == 0) return a.s[0] == kNo;
  return a.s[j] != a.e[j - 1];
}

__global__ __launch_bounds__(256) void index_flag_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < a.n_chunks) a.base[j] = link_broken(a, j) ? 1 : 0;
}

__global__ __launch_bounds__(256) void index_list_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < a.n_chunks && link_broken(a, j)) a.bad[a.base[j]] = j;
}

// One lane: repair the chain (see header). scal[1] = chunks in effect.
template <int P>
__global__ void index_fix_kernel(IndexArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t C = a.n_chunks;
  a.scal[2] = kNo;
  a.scal[1] = C;
  uint64_t T0 = a.begin, j0 = 0;
  if (a.speculative) {
    // the first chunk with a speculated start opens the range (a record may
    // cover the first chunks entirely); none at all: no record starts here
    while (j0 < C && a.s[j0] == kNo) ++j0;
    if (j0 == C) {
      a.scal[1] = 0;
      return;
    }
    T0 = a.s[j0];
    for (uint64_t i = 0; i < j0; ++i) {
      a.s[i] = T0;
      a.e[i] = T0;
      a.cnt[i] = 0;
    }
  }
  const uint64_t m = a.scal[0];
  uint64_t next = 0;  // chunks below are final
  uint8_t* scratch = a.scratch;
  for (uint64_t k = 0; k < m; ++k) {
    uint64_t j = a.bad[k];
    if (j < next || j < j0) continue;
    uint64_t T = j == 0 ? T0 : a.e[j - 1];
    for (;;) {
      const uint64_t hi = chunk_hi(a, j);
      if (T >= hi) {  // no record starts inside this chunk
        a.s[j] = T;
        a.e[j] = T;
        a.cnt[j] = 0;
        a.pf[j] = 0;
      } else {
        Chain c;
        chain<P>(a, T, hi, false, scratch, c, nullptr, 0, kNo);
        a.s[j] = T;
        a.cnt[j] = c.count;
        a.pf[j] = 0;
        if (c.code) {
          a.e[j] = c.end;
          a.scal[1] = j + 1;
          a.scal[2] = j;
          a.scal[3] = c.count;
          a.scal[4] = c.end;
          a.res->code = c.code;
          a.res->fail_offset = c.err_off;
          return;
        }
        a.e[j] = c.end;
      }
      T = a.e[j];
      if (j + 1 < C && (a.s[j + 1] != T || a.e[j + 1] == kNo || a.e[j + 1] == kErr)) {
        ++j;
        continue;
      }
      break;
    }
    next = j + 1;
  }
}

__global__ __launch_bounds__(256) void index_prep_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < a.n_chunks) a.base[j] = j < a.scal[1] ? a.cnt[j] : 0;
}

// Emit, program-only; a chain the program cannot finish is handed to
// index_emit_cont_kernel (ep = where it stopped, ec = starts written).
__global__ __launch_bounds__(256) void index_emit_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n_chunks) return;
  a.ep[j] = kNo;
  if (j >= a.scal[1]) return;
  const uint64_t b = a.base[j];
  const uint64_t n = a.cnt[j];
  if (n == 0 || b > a.max_records) return;
  const uint64_t cap = a.max_records + 1 - b;
  uint64_t p = a.s[j];
  bool stuck = true;
  uint64_t c = 0;
  if (a.prog) c = prog_chain(a, p, kNo, n, a.offs + b, cap, stuck);
  if (c < n) {
    a.ep[j] = p;
    a.ec[j] = c;
  }
}

template <int P>
__global__ __launch_bounds__(256) void index_emit_cont_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n_chunks || a.ep[j] == kNo) return;
  const uint64_t b = a.base[j] + a.ec[j];
  const uint64_t n = a.cnt[j] - a.ec[j];
  if (b > a.max_records) return;
  Chain c;
  chain<P>(a, a.ep[j], kNo, false, a.scratch + j * a.rec_size, c, a.offs + b,
           a.max_records + 1 - b, n);
}

// total records; end of the last one; status; decode padding of the index.
__global__ void index_finish_kernel(IndexArgs a, unsigned long long* total_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t ce = a.scal[1];
  uint64_t total = 0, end = a.begin;
  if (ce) {
    total = a.base[ce - 1] + a.cnt[ce - 1];
    end = a.e[ce - 1];
  }
  DevResult* res = a.res;
  res->first_start = ce ? a.s[0] : kNo;
  if (a.scal[2] != kNo && ce) {  // reader error: total = records before it
    res->first_fail = total;
    end = a.scal[4];
  } else if (!ce) {
    end = a.speculative ? kNo : a.begin;  // no record starts in the range
  }
  res->n_records = total;
  res->total_bytes = end;
  if (total <= a.max_records) a.offs[total] = end;
  *total_out = total;
}

// offs[total+1 .. fill_to] = offs[total]: records past the stream's end (or
// its first bad record) re-read that position, so the decoder reports them
// exactly (underflow / the same error) without a host round trip.
__global__ __launch_bounds__(256) void index_pad_kernel(IndexArgs a,
                                                        const unsigned long long* total_p) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t total = *total_p;
  if (i > total && i <= a.fill_to && total <= a.max_records) a.offs[i] = a.offs[total];
}

__global__ __launch_bounds__(256) void index_empty_kernel(DevResult* res, uint64_t* offs,
                                                          uint64_t pos, uint64_t fill_to) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i <= fill_to) offs[i] = pos;
  if (i == 0) {
    res->n_records = 0;
    res->total_bytes = pos;
    res->first_start = kNo;
  }
}

}  // namespace

hipError_t launch_index_empty(DevResult* res, uint64_t* offs, uint64_t pos, uint64_t fill_to,
                              hipStream_t stream) {
  hipLaunchKernelGGL(index_empty_kernel, dim3((uint32_t)((fill_to + 256) / 256)), dim3(256), 0,
                     stream, res, offs, pos, fill_to);
  return hipGetLastError();
}

uint64_t index_tile_bytes() { return kTile; }
uint64_t index_tile_lanes() { return kTileLanes; }

uint64_t index_chunk_bytes(uint64_t span, bool tiles) {
  // schemas with a program: LDS tiles once there are enough of them
  if (tiles && span >= 64ull * kTile) return kTile;
  // lane chunks: ~1k+ chunks keep the chip busy; chunks stay >= 1 KiB so a
  // chunk holds several records and speculation has a long chain to confirm
  uint64_t c = 4096;
  while (c > 1024 && span / c < 4096) c >>= 1;
  return c;
}

hipError_t launch_index_stream(const IndexArgs& a, hipStream_t stream) {
  const uint64_t C = a.n_chunks;
  const dim3 g((uint32_t)((C + 255) / 256)), b(256);
  const bool bin = a.protocol == TGPU_PROTOCOL_BINARY;
  if (a.prog && a.chunk == kTile) {
    hipLaunchKernelGGL(index_tile_spec_kernel, dim3((uint32_t)C), dim3(kTileLanes), 0, stream, a);
    if (bin)
      hipLaunchKernelGGL(index_cont_kernel<TGPU_PROTOCOL_BINARY>, g, b, 0, stream, a);
    else
      hipLaunchKernelGGL(index_cont_kernel<TGPU_PROTOCOL_COMPACT>, g, b, 0, stream, a);
  } else if (a.prog) {
    hipLaunchKernelGGL(index_spec_kernel, g, b, 0, stream, a);
    if (bin)
      hipLaunchKernelGGL(index_cont_kernel<TGPU_PROTOCOL_BINARY>, g, b, 0, stream, a);
    else
      hipLaunchKernelGGL(index_cont_kernel<TGPU_PROTOCOL_COMPACT>, g, b, 0, stream, a);
  } else if (bin) {
    hipLaunchKernelGGL(index_spec_general_kernel<TGPU_PROTOCOL_BINARY>, g, b, 0, stream, a);
  } else {
    hipLaunchKernelGGL(index_spec_general_kernel<TGPU_PROTOCOL_COMPACT>, g, b, 0, stream, a);
  }
  hipLaunchKernelGGL(index_flag_kernel, g, b, 0, stream, a);
  hipError_t e = launch_scan_tiles(a.base, C, a.part, a.scal, nullptr, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(index_list_kernel, g, b, 0, stream, a);
  if (bin)
    hipLaunchKernelGGL(index_fix_kernel<TGPU_PROTOCOL_BINARY>, dim3(1), dim3(64), 0, stream, a);
  else
    hipLaunchKernelGGL(index_fix_kernel<TGPU_PROTOCOL_COMPACT>, dim3(1), dim3(64), 0, stream, a);
  hipLaunchKernelGGL(index_prep_kernel, g, b, 0, stream, a);
  e = launch_scan_tiles(a.base, C, a.part, nullptr, nullptr, stream);
  if (e != hipSuccess) return e;
  if (a.prog && a.chunk == kTile)
    hipLaunchKernelGGL(index_tile_emit_kernel, dim3((uint32_t)C), dim3(kTileLanes), 0, stream, a);
  else
    hipLaunchKernelGGL(index_emit_kernel, g, b, 0, stream, a);
  if (bin)
    hipLaunchKernelGGL(index_emit_cont_kernel<TGPU_PROTOCOL_BINARY>, g, b, 0, stream, a);
  else
    hipLaunchKernelGGL(index_emit_cont_kernel<TGPU_PROTOCOL_COMPACT>, g, b, 0, stream, a);
  hipLaunchKernelGGL(index_finish_kernel, dim3(1), dim3(64), 0, stream, a, a.scal + 5);
  if (a.fill_to > 0)
    hipLaunchKernelGGL(index_pad_kernel, dim3((uint32_t)((a.fill_to + 256) / 256)), b, 0, stream,
                       a, a.scal + 5);
  return hipGetLastError();
}

}  // namespace tgpu
