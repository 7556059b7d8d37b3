// k_plan_binary.hip — word-gather kernels for fixed-layout Binary records
// (BASELINE config 1/2 {1..8: i64}: L = 89 wire bytes, S = 72 record bytes).
//
// Same semantics as k_fixed_binary.hip (canonical template match, first
// non-canonical record latched for the serial fallback), organised so that
// the HBM side of each kernel is a plain coalesced stream:
//   decode: wire tile HBM -> LDS (16-byte loads); each lane then produces
//           whole 8-byte words of the output records (word j of record r =
//           const isset/padding bits | the values whose members live in that
//           word, read from LDS with aligned dword reads + v_alignbyte +
//           byte swap) and stores them coalesced, 512 bytes per wave store.
//           No output tile, no LDS zero-fill, one barrier.
//   encode: each lane loads whole 8-byte record words coalesced into
//           registers, ORs the header + big-endian value bytes of the items
//           they own into the LDS wire tile (ds_or_b32; items of one record
//           are disjoint, the 2 dwords shared with a neighbour record are
//           merged by the OR), then the tile goes LDS -> HBM with 16-byte
//           stores.
// LDS per workgroup is one wire tile (~23 KB) + the 1.5 KB plan, so 6
// workgroups (24 waves) fit a CU; the HBM streams of the co-resident
// workgroups overlap each other's LDS phases.
#include <cstdio>
#include <cstdlib>

#include "tgpu_internal.h"
#include "tgpu_program.h"

#ifdef TGPU_PLAN_STALE_CHECK
// (diagnostics build) plan-decode value words whose staged copy differed from HBM
__device__ unsigned long long tgpu_plan_stale_words;
#endif

namespace tgpu {
namespace {

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// LDS bytes of a T-record wire tile: + 16-byte phase + over-read/-write slack,
// rounded to whole rounds of T x 16-byte staging chunks (LDS-DMA writes a
// full round).
__host__ __device__ __forceinline__ uint32_t wire_region(uint32_t T, uint32_t L) {
  return (T * L + 32 + 16 * T - 1) / (16 * T) * (16 * T);
}


// Output word j of the record whose wire bytes start at LDS byte `base`.
__device__ __forceinline__ unsigned long long decode_word(const FixedPlan* P,
                                                          const uint32_t* w32, uint32_t base,
                                                          uint32_t j, bool& ok) {
  const PlanWord w = P->words[j];
  unsigned long long v = w.const_bits;
  for (uint32_t k = 0; k < w.n_items; ++k) {
    const PlanItem it = P->items[w.first_item + k];
    const uint32_t a = base + it.wire_off;
    const uint32_t d = a >> 2, s = a & 3;
    const uint32_t W0 = w32[d], W1 = w32[d + 1], W2 = w32[d + 2], W3 = w32[d + 3];
    const uint32_t G0 = __builtin_amdgcn_alignbyte(W1, W0, s);
    const uint32_t G1 = __builtin_amdgcn_alignbyte(W2, W1, s);
    const uint32_t G2 = __builtin_amdgcn_alignbyte(W3, W2, s);
    const uint32_t h = it.hdr_len;
    if (h) {
      const uint32_t mask = h >= 4 ? 0xffffffffu : ((1u << (8 * h)) - 1);
      ok &= ((G0 ^ it.hdr) & mask) == 0;
    }
    if (it.width) {
      const uint32_t X0 = __builtin_amdgcn_alignbyte(G1, G0, h);
      const uint32_t X1 = __builtin_amdgcn_alignbyte(G2, G1, h);
      unsigned long long val;
      switch (it.width) {
        case 8: val = ((unsigned long long)bswap32(X0) << 32) | bswap32(X1); break;
        case 4: val = bswap32(X0); break;
        case 2: val = bswap32(X0) >> 16; break;
        default:
          val = X0 & 0xff;
          if (it.is_bool) ok &= val <= 1;  // readBool: byte >= 2 throws
          break;
      }
      v |= val << (8 * it.dst);
    }
  }
  return v;
}

// The exception records of a tile: a record with a word the plan cannot take
// is marked in the tile's LDS bitmap `seen` (once, however many of its words
// fail) and the tile lists them at its end — one atomicMin / atomicAdd per
// tile, so a stream off the stride from early on (every record fails) costs
// two global atomics per tile, not one per word (the same-address atomics of
// every lane of every wave were 28 ms on 64 Mi records, 15x the decode).
template <uint32_t T>
__device__ __forceinline__ void list_tile_exceptions(uint64_t tile0, const uint32_t* seen,
                                                     DevResult* res, uint64_t* exc, uint64_t cap) {
  static_assert(T / 32 <= 64, "one bitmap word per lane of wave 0");
  const uint32_t lane = threadIdx.x;
  const uint32_t w = lane < T / 32 ? seen[lane] : 0u;
  const uint64_t nz = __ballot(w != 0);
  if (!nz) return;
  const uint32_t c = (uint32_t)__builtin_popcount(w);
  uint32_t pre = c;  // inclusive prefix of the counts over the lanes
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(pre, o, 64);
    if (lane >= o) pre += x;
  }
  const uint32_t total = __shfl(pre, 63, 64);
  const uint32_t fl = (uint32_t)__builtin_ctzll(nz);
  unsigned long long k0 = ~0ull;
  if (lane == fl) {
    const uint64_t i = tile0 + 32 * lane + (uint32_t)__builtin_ctz(w);
    if (i < __hip_atomic_load(&res->first_irregular, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMin(&res->first_irregular, (unsigned long long)i);
    // (an overflowed list is left alone; the relaxed load may be stale, which
    // only costs the atomic)
    if (__hip_atomic_load(&res->n_irregular, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= cap)
      k0 = atomicAdd(&res->n_irregular, (unsigned long long)total);
  }
  k0 = __shfl(k0, (int)fl, 64);
  if (k0 == ~0ull) return;
  unsigned long long k = k0 + (pre - c);
  for (uint32_t m = w; m; m &= m - 1, ++k)
    if (k < cap) exc[k] = tile0 + 32 * lane + (uint32_t)__builtin_ctz(m);
}

// T records (= threads) per tile. kGlds: stage through LDS-DMA
// (global_load_lds_dwordx4) instead of registers. kPair: 16-byte stores of
// two consecutive words. kNT: non-temporal stores (output is never re-read).
template <uint32_t T, bool kGlds, bool kPair, bool kNT>
__global__ __launch_bounds__(T) void plan_binary_decode_kernel(
    const FixedPlan* __restrict__ pp, const uint8_t* __restrict__ in, uint64_t n,
    unsigned long long* __restrict__ out, DevResult* __restrict__ res, uint64_t* __restrict__ exc,
    uint64_t exc_cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t L = pp->wire_len, Q = pp->n_words;
  const uint64_t tile0 = (uint64_t)blockIdx.x * T;
  const uint32_t nrec = (uint32_t)min((uint64_t)T, n - tile0);
  FixedPlan* P = (FixedPlan*)(smem + wire_region(T, L));

  // stage the wire tile (16-byte phase of the stream preserved)
  const uint8_t* g = in + tile0 * L;
  const uint32_t sh = (uint32_t)((uintptr_t)g & 15);
  {
    const uint4* src = (const uint4*)(g - sh);
    const uint32_t nvec = (nrec * L + sh + 15) >> 4;
    if (kGlds) {
      const uint32_t wave = threadIdx.x >> 6;
      for (uint32_t k = 0; k * T < nvec; ++k) {
        const uint32_t i = k * T + threadIdx.x;
        const uint4* s = src + (i < nvec ? i : nvec - 1);  // clamp: never past the stream
        __builtin_amdgcn_global_load_lds(
            (const void*)s,
            (__attribute__((address_space(3))) void*)(smem + (size_t)(k * T + wave * 64) * 16), 16,
            0, 0);
      }
      // (lds_dma_settle, tgpu_program.h; TGPU_NO_DMA_SETTLE builds leave it out)
#ifndef TGPU_NO_DMA_SETTLE
      prog::lds_dma_settle(smem, threadIdx.x, T, (nvec + T - 1) / T);
#endif
    } else {
      for (uint32_t i = threadIdx.x; i < nvec; i += T) ((uint4*)smem)[i] = src[i];
    }
  }
  for (uint32_t i = threadIdx.x; i < (uint32_t)(sizeof(FixedPlan) / 16); i += T)
    ((uint4*)P)[i] = ((const uint4*)pp)[i];
  uint32_t* seen = (uint32_t*)(smem + wire_region(T, L) + sizeof(FixedPlan));
  if (threadIdx.x < T / 32) seen[threadIdx.x] = 0;
  // an overflowed exception list below this tile: every record from
  // first_irregular on is re-read by the tail (index, or the stream-ordered
  // strided decode), so the tile's work is moot (read with the staging in
  // flight; both values only move one way; seen[T / 32]: the tile's verdict)
  if (threadIdx.x == 0) {
    const unsigned long long irr0 =
        __hip_atomic_load(&res->first_irregular, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long nirr0 =
        __hip_atomic_load(&res->n_irregular, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    seen[T / 32] = nirr0 > exc_cap && irr0 < tile0;
  }
  __syncthreads();
  if (seen[T / 32]) return;

  const uint32_t* w32 = (const uint32_t*)smem;
  const uint32_t total = nrec * Q;
  unsigned long long* o = out + tile0 * Q;
  if (!kPair) {
    uint32_t r = threadIdx.x / Q, j = threadIdx.x - r * Q;
    const uint32_t sr = T / Q, sj = T - sr * Q;
    for (uint32_t q = threadIdx.x; q < total; q += T) {
      bool ok = true;
      const unsigned long long v = decode_word(P, w32, sh + r * L, j, ok);
      if (kNT) __builtin_nontemporal_store(v, o + q);
      else o[q] = v;
      // a record one of whose words the plan cannot take joins the exception
      // list (once)
      if (!ok) atomicOr(&seen[r >> 5], 1u << (r & 31));
      r += sr;
      j += sj;
      if (j >= Q) {
        j -= Q;
        ++r;
      }
    }
  } else {
    const uint32_t q0 = 2 * threadIdx.x;
    uint32_t r = q0 / Q, j = q0 - r * Q;
    const uint32_t sr = (2 * T) / Q, sj = 2 * T - sr * Q;
    for (uint32_t q = q0; q < total; q += 2 * T) {
      bool ok0 = true, ok1 = true;
      const unsigned long long v0 = decode_word(P, w32, sh + r * L, j, ok0);
      const uint32_t r1 = j + 1 == Q ? r + 1 : r, j1 = j + 1 == Q ? 0 : j + 1;
      if (q + 1 < total) {
        const unsigned long long v1 = decode_word(P, w32, sh + r1 * L, j1, ok1);
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        u64x2 pr = {v0, v1};
        if (kNT) __builtin_nontemporal_store(pr, (u64x2*)(o + q));
        else *(u64x2*)(o + q) = pr;
      } else {
        o[q] = v0;
      }
      if (!ok0) atomicOr(&seen[r >> 5], 1u << (r & 31));
      if (!ok1) atomicOr(&seen[r1 >> 5], 1u << (r1 & 31));
      r += sr;
      j += sj;
      if (j >= Q) {
        j -= Q;
        ++r;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) list_tile_exceptions<T>(tile0, seen, res, exc, exc_cap);
}


// ---- lane-stationary forms (round 5) ---------------------------------------
// The word-gather kernels above give lane t the output words t, t + T, …: with
// Q words per record and T not a multiple of Q, a lane's word index j moves
// every pass, so each pass re-reads its PlanWord / PlanItems from LDS and runs
// a divergent per-item loop with a switch on the width (round-4 SQ counters:
// 607 VALU + 596 SALU + 92 LDS instructions per wave for 9 words a lane).
// Here a tile is R·P records with R = ⌊T/Q⌋: lane t < R·Q owns word
// j = t mod Q of records t/Q, t/Q + R, … — the same j in every pass — so its
// word's items are read once (from the global plan, before the staging DMA)
// into registers, and every pass is straight-line: the window reads, the
// header compare and one 64-bit shift that takes a big-endian value of any
// width (val = be64 >> (64 − 8·width)). Lane-consecutive words are still
// record-consecutive words, so the stores stay one contiguous 8·64-byte run per
// wave. T mod Q lanes idle (8 of 512 for flat8).
// LDS bytes of a TR-record wire tile staged by T threads: whole rounds of
// T x 16-byte LDS-DMA chunks.
__host__ __device__ __forceinline__ uint32_t ls_wire_region(uint32_t T, uint32_t TR, uint32_t L) {
  return (TR * L + 32 + 16 * T - 1) / (16 * T) * (16 * T);
}

struct LsItem {
  uint32_t off_h_w;   // wire_off | hdr_len << 16 | width << 24
  uint32_t hdr;
  uint32_t hmask;     // header bytes compared
  uint32_t vsh_dst;   // 64 − 8·width | 8·dst << 8 | is_bool << 16 (width 0: vsh 0, no value)
};

__device__ __forceinline__ LsItem ls_item(const PlanItem& it) {
  LsItem x;
  x.off_h_w = (uint32_t)it.wire_off | ((uint32_t)it.hdr_len << 16) | ((uint32_t)it.width << 24);
  x.hdr = it.hdr;
  x.hmask = it.hdr_len >= 4 ? 0xffffffffu : ((1u << (8 * it.hdr_len)) - 1);
  x.vsh_dst = (it.width ? 64u - 8u * it.width : 0u) | ((uint32_t)it.dst * 8u << 8) |
              ((uint32_t)it.is_bool << 16);
  return x;
}

// Value bits one item contributes to its word (0 for a header-only item);
// ok cleared on a header mismatch or a bool byte >= 2.
__device__ __forceinline__ unsigned long long ls_decode_item(const LsItem& x, const uint32_t* w32,
                                                             uint32_t base, bool& ok) {
  const uint32_t a = base + (x.off_h_w & 0xffff);
  const uint32_t d = a >> 2, s = a & 3;
  const uint32_t W0 = w32[d], W1 = w32[d + 1], W2 = w32[d + 2], W3 = w32[d + 3];
  const uint32_t G0 = __builtin_amdgcn_alignbyte(W1, W0, s);
  const uint32_t G1 = __builtin_amdgcn_alignbyte(W2, W1, s);
  const uint32_t G2 = __builtin_amdgcn_alignbyte(W3, W2, s);
  const uint32_t h = (x.off_h_w >> 16) & 0xff;
  ok &= ((G0 ^ x.hdr) & x.hmask) == 0;
  const uint32_t X0 = __builtin_amdgcn_alignbyte(G1, G0, h);
  const uint32_t X1 = __builtin_amdgcn_alignbyte(G2, G1, h);
  const unsigned long long be = ((unsigned long long)bswap32(X0) << 32) | bswap32(X1);
  // (a header-only item, width 0, contributes nothing; selects, not branches)
  const unsigned long long val = (x.off_h_w >> 24) ? be >> (x.vsh_dst & 0xff) : 0ull;
  ok &= !(((x.vsh_dst >> 16) & 1) && val > 1);  // readBool: byte >= 2 throws
  return val << ((x.vsh_dst >> 8) & 0xff);
}

// KI: the most items any word holds (1, 2, 4 or 8). kChk: the tile verdict of
// an overflowed exception list below the tile (round 4's prologue), kept for
// the A/B the round-4 verdict asked for.
template <uint32_t T, uint32_t KI, bool kNT, bool kChk>
__global__ __launch_bounds__(T) void plan_binary_decode_ls_kernel(
    const FixedPlan* __restrict__ pp, const uint8_t* __restrict__ in, uint64_t n, uint32_t R,
    uint32_t passes, unsigned long long* __restrict__ out, DevResult* __restrict__ res,
    uint64_t* __restrict__ exc, uint64_t exc_cap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t L = pp->wire_len, Q = pp->n_words;
  const uint32_t TR = R * passes;  // records per tile
  const uint64_t tile0 = (uint64_t)blockIdx.x * TR;
  const uint32_t nrec = (uint32_t)min((uint64_t)TR, n - tile0);
  const uint32_t tid = threadIdx.x;
  const bool act = tid < R * Q;
  const uint32_t r0 = tid / Q, j = act ? tid - r0 * Q : 0;

  // this lane's word: its items into registers (plain loads of the small
  // plan, L2-resident; issued before the staging DMA so that the settle's
  // vmcnt(0) covers them at no extra wait)
  const PlanWord pw = pp->words[j];
  const uint32_t nit = pw.n_items;
  LsItem it[KI];
#pragma unroll
  for (uint32_t m = 0; m < KI; ++m) {
    const PlanItem pi = pp->items[pw.first_item + (m < nit ? m : 0)];
    it[m] = ls_item(pi);
  }

  const uint32_t wreg = ls_wire_region(T, TR, L);
  uint32_t* seen = (uint32_t*)(smem + wreg);
  const uint8_t* g = in + tile0 * L;
  const uint32_t sh = (uint32_t)((uintptr_t)g & 15);
  {
    const uint4* src = (const uint4*)(g - sh);
    const uint32_t nvec = (nrec * L + sh + 15) >> 4;
    const uint32_t wave = tid >> 6;
    for (uint32_t k = 0; k * T < nvec; ++k) {
      const uint32_t i = k * T + tid;
      const uint4* s = src + (i < nvec ? i : nvec - 1);
      __builtin_amdgcn_global_load_lds(
          (const void*)s,
          (__attribute__((address_space(3))) void*)(smem + (size_t)(k * T + wave * 64) * 16), 16, 0,
          0);
    }
    if (tid < (TR + 31) / 32) seen[tid] = 0;
    if (kChk && tid == 0) {
      const unsigned long long irr0 =
          __hip_atomic_load(&res->first_irregular, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long nirr0 =
          __hip_atomic_load(&res->n_irregular, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      seen[(TR + 31) / 32] = nirr0 > exc_cap && irr0 < tile0;
    }
#ifndef TGPU_NO_DMA_SETTLE
    prog::lds_dma_settle(smem, tid, T, (nvec + T - 1) / T);
#endif
  }
  __syncthreads();
  if (kChk && seen[(TR + 31) / 32]) return;

  const uint32_t* w32 = (const uint32_t*)smem;
  unsigned long long* o = out + tile0 * Q;
  if (act) {
    uint32_t r = r0;
    for (uint32_t k = 0; k < passes && r < nrec; ++k, r += R) {
      const uint32_t base = sh + r * L;
      unsigned long long v = pw.const_bits;
      bool ok = true;
#pragma unroll
      for (uint32_t m = 0; m < KI; ++m)
        if (m < nit) v |= ls_decode_item(it[m], w32, base, ok);
      if (kNT) __builtin_nontemporal_store(v, o + (size_t)r * Q + j);
      else o[(size_t)r * Q + j] = v;
      if (!ok) atomicOr(&seen[r >> 5], 1u << (r & 31));
#ifdef TGPU_PLAN_STALE_CHECK
      if (r + 1 < nrec) {  // diagnostics: the same
         // word decoded from HBM (its 16-byte window stays inside the tile);
         // a stale staged word that keeps its header bytes differs here
        unsigned long long vg = pw.const_bits;
        bool okg = true;
#pragma unroll
        for (uint32_t m = 0; m < KI; ++m)
          if (m < nit) vg |= ls_decode_item(it[m], (const uint32_t*)(g - sh), base, okg);
        if (vg != v || okg != ok) atomicAdd(&tgpu_plan_stale_words, 1ull);
      }
#endif
    }
  }
  __syncthreads();
  if (tid < 64) {
    // (list_tile_exceptions for a tile of TR <= 2048 records: up to 64
    // bitmap words, one per lane of wave 0)
    const uint32_t nw = (TR + 31) / 32;
    const uint32_t w = tid < nw ? seen[tid] : 0u;
    const uint64_t nz = __ballot(w != 0);
    if (!nz) return;
    const uint32_t c = (uint32_t)__builtin_popcount(w);
    uint32_t pre = c;
    for (uint32_t s2 = 1; s2 < 64; s2 <<= 1) {
      const uint32_t x = __shfl_up(pre, s2, 64);
      if (tid >= s2) pre += x;
    }
    const uint32_t total = __shfl(pre, 63, 64);
    const uint32_t fl = (uint32_t)__builtin_ctzll(nz);
    unsigned long long k0 = ~0ull;
    if (tid == fl) {
      const uint64_t i = tile0 + 32 * tid + (uint32_t)__builtin_ctz(w);
      if (i < __hip_atomic_load(&res->first_irregular, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMin(&res->first_irregular, (unsigned long long)i);
      if (__hip_atomic_load(&res->n_irregular, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= exc_cap)
        k0 = atomicAdd(&res->n_irregular, (unsigned long long)total);
    }
    k0 = __shfl(k0, (int)fl, 64);
    if (k0 == ~0ull) return;
    unsigned long long kk = k0 + (pre - c);
    for (uint32_t m = w; m; m &= m - 1, ++kk)
      if (kk < exc_cap) exc[kk] = tile0 + 32 * tid + (uint32_t)__builtin_ctz(m);
  }
}

// Encode, lane-stationary: lane t < R·Q loads word j of its records
// (coalesced), ORs its word's items' header + big-endian value bytes into the
// zero-filled LDS wire tile (items in registers, no plan in LDS), then the
// tile leaves with 16-byte stores.
template <uint32_t T, uint32_t KI, uint32_t PMAX, bool kNT>
__global__ __launch_bounds__(T) void plan_binary_encode_ls_kernel(
    const FixedPlan* __restrict__ pp, const unsigned long long* __restrict__ recs, uint64_t n,
    uint32_t R, uint32_t passes, uint8_t* __restrict__ out, uint64_t* __restrict__ offsets,
    DevResult* __restrict__ res) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t L = pp->wire_len, Q = pp->n_words;
  const uint32_t TR = R * passes;
  const uint64_t tile0 = (uint64_t)blockIdx.x * TR;
  const uint32_t nrec = (uint32_t)min((uint64_t)TR, n - tile0);
  const uint32_t tid = threadIdx.x;
  const bool act = tid < R * Q;
  const uint32_t r0 = tid / Q, j = act ? tid - r0 * Q : 0;
  const uint32_t wreg = ls_wire_region(T, TR, L);

  const PlanWord pw = pp->words[j];
  const uint32_t nit = pw.n_items;
  const bool load = act && pw.has_value;
  // 1. record words -> registers (coalesced, issued first)
  // (PMAX >= passes: the register array is sized by the launch)
  unsigned long long vals[PMAX];
#pragma unroll
  for (uint32_t k = 0; k < PMAX; ++k) {
    const uint32_t r = r0 + k * R;
    vals[k] = 0;
    if (k < passes && load && r < nrec) {
      const unsigned long long* p = recs + (tile0 + r) * Q + j;
      vals[k] = kNT ? __builtin_nontemporal_load(p) : *p;
    }
  }
  PlanItem pit[KI];
#pragma unroll
  for (uint32_t m = 0; m < KI; ++m) pit[m] = pp->items[pw.first_item + (m < nit ? m : 0)];
  // 2. zero the wire tile
  uint8_t* gout = out + tile0 * L;
  const uint32_t osh = (uint32_t)((uintptr_t)gout & 15);
  {
    const uint4 z = {0u, 0u, 0u, 0u};
    for (uint32_t i = tid; i < (wreg >> 4); i += T) ((uint4*)smem)[i] = z;
  }
  __syncthreads();

  // 3. OR each owned item's wire bytes into the tile
  uint32_t* w32 = (uint32_t*)smem;
  bool bad_bool = false;
  uint32_t bad_rec = 0;
  if (act) {
#pragma unroll
    for (uint32_t k = 0; k < PMAX; ++k) {
      const uint32_t r = r0 + k * R;
      if (k < passes && r < nrec) {
        const unsigned long long v = vals[k];
        const uint32_t base = osh + r * L;
#pragma unroll
        for (uint32_t m = 0; m < KI; ++m) {
          if (m < nit) {
            const PlanItem it = pit[m];
            const uint32_t h = it.hdr_len, w = it.width;
            const unsigned long long raw = v >> (8 * it.dst);
            // the low `w` bytes of raw, big-endian, first byte lowest
            const unsigned long long top = w ? raw << (64 - 8 * w) : 0;
            const unsigned long long vbe =
                ((unsigned long long)bswap32((uint32_t)(top >> 32))) |
                ((unsigned long long)bswap32((uint32_t)top) << 32);
            if (it.is_bool && (raw & 0xff) > 1) {  // validate_bool
              bad_bool = true;
              bad_rec = r;
            }
            const unsigned long long Flo = (unsigned long long)it.hdr | (vbe << (8 * h));
            const unsigned long long Fhi = h ? (vbe >> (64 - 8 * h)) : 0;
            const uint32_t a = base + it.wire_off;
            const uint32_t d = a >> 2, s = a & 3;
            const unsigned long long Hlo = Flo << (8 * s);
            const unsigned long long Hhi = (Fhi << (8 * s)) | (s ? (Flo >> (64 - 8 * s)) : 0);
            const uint32_t nb = s + h + w;
            atomicOr(&w32[d], (uint32_t)Hlo);
            if (nb > 4) atomicOr(&w32[d + 1], (uint32_t)(Hlo >> 32));
            if (nb > 8) atomicOr(&w32[d + 2], (uint32_t)Hhi);
            if (nb > 12) atomicOr(&w32[d + 3], (uint32_t)(Hhi >> 32));
          }
        }
      }
    }
  }
  if (bad_bool) atomicMin(&res->first_fail, (unsigned long long)(tile0 + bad_rec));
  if (offsets) {
    for (uint32_t i = tid; i < nrec; i += T) offsets[tile0 + i] = (tile0 + i) * L;
    if (tile0 + nrec == n && tid == 0) offsets[n] = n * L;
  }
  __syncthreads();

  // 4. wire tile -> HBM
  {
    uint8_t* base = gout - osh;
    const uint32_t end = osh + nrec * L;
    const uint32_t nvec = (end + 15) >> 4;
    for (uint32_t i = tid; i < nvec; i += T) {
      const uint32_t lo = i << 4, hi = lo + 16;
      if (lo >= osh && hi <= end) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        if (kNT) __builtin_nontemporal_store(((const u32x4*)smem)[i], (u32x4*)base + i);
        else ((uint4*)base)[i] = ((const uint4*)smem)[i];
      } else {
        for (uint32_t b = (lo < osh ? osh : lo); b < (hi < end ? hi : end); ++b) base[b] = smem[b];
      }
    }
  }
}

// Encode, direct (round 6 A/B, TGPU_PLAN_ENCODE ls=2): the lane-stationary
// layout without the LDS wire tile — each lane stores its items' bytes
// straight to HBM with unaligned 8/4/2/1-byte stores (items never share a
// byte, so no lane's store overlaps another's; the 128-byte lines fill in
// L2 before they leave). No LDS: occupancy is bounded by registers only.
typedef unsigned long long u64_u __attribute__((aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));
typedef uint16_t u16_u __attribute__((aligned(1)));

template <uint32_t T, uint32_t KI, uint32_t PMAX>
__global__ __launch_bounds__(T) void plan_binary_encode_direct_kernel(
    const FixedPlan* __restrict__ pp, const unsigned long long* __restrict__ recs, uint64_t n,
    uint32_t R, uint32_t passes, uint8_t* __restrict__ out, uint64_t* __restrict__ offsets,
    DevResult* __restrict__ res) {
  const uint32_t L = pp->wire_len, Q = pp->n_words;
  const uint32_t TR = R * passes;
  const uint64_t tile0 = (uint64_t)blockIdx.x * TR;
  const uint32_t nrec = (uint32_t)min((uint64_t)TR, n - tile0);
  const uint32_t tid = threadIdx.x;
  const bool act = tid < R * Q;
  const uint32_t r0 = tid / Q, j = act ? tid - r0 * Q : 0;
  const PlanWord pw = pp->words[j];
  const uint32_t nit = pw.n_items;
  const bool load = act && pw.has_value;
  unsigned long long vals[PMAX];
#pragma unroll
  for (uint32_t k = 0; k < PMAX; ++k) {
    const uint32_t r = r0 + k * R;
    vals[k] = 0;
    if (k < passes && load && r < nrec)
      vals[k] = __builtin_nontemporal_load(recs + (tile0 + r) * Q + j);
  }
  PlanItem pit[KI];
#pragma unroll
  for (uint32_t m = 0; m < KI; ++m) pit[m] = pp->items[pw.first_item + (m < nit ? m : 0)];
  uint8_t* gout = out + tile0 * L;
  bool bad_bool = false;
  uint32_t bad_rec = 0;
  if (act) {
#pragma unroll
    for (uint32_t k = 0; k < PMAX; ++k) {
      const uint32_t r = r0 + k * R;
      if (k < passes && r < nrec) {
        const unsigned long long v = vals[k];
#pragma unroll
        for (uint32_t m = 0; m < KI; ++m) {
          if (m < nit) {
            const PlanItem it = pit[m];
            const uint32_t h = it.hdr_len, w = it.width;
            const unsigned long long raw = v >> (8 * it.dst);
            const unsigned long long top = w ? raw << (64 - 8 * w) : 0;
            const unsigned long long vbe =
                ((unsigned long long)bswap32((uint32_t)(top >> 32))) |
                ((unsigned long long)bswap32((uint32_t)top) << 32);
            if (it.is_bool && (raw & 0xff) > 1) {  // validate_bool
              bad_bool = true;
              bad_rec = r;
            }
            const unsigned long long Flo = (unsigned long long)it.hdr | (vbe << (8 * h));
            const unsigned long long Fhi = h ? (vbe >> (64 - 8 * h)) : 0;
            uint8_t* p = gout + (size_t)r * L + it.wire_off;
            const uint32_t nb = h + w;
            unsigned long long x = Flo;
            uint32_t off = 0;
            if (nb >= 8) {
              *(u64_u*)p = Flo;
              x = Fhi;
              off = 8;
            }
            const uint32_t m2 = nb - off;
            if (m2 & 4) {
              *(u32_u*)(p + off) = (uint32_t)x;
              x >>= 32;
              off += 4;
            }
            if (m2 & 2) {
              *(u16_u*)(p + off) = (uint16_t)x;
              x >>= 16;
              off += 2;
            }
            if (m2 & 1) p[off] = (uint8_t)x;
          }
        }
      }
    }
  }
  if (bad_bool) atomicMin(&res->first_fail, (unsigned long long)(tile0 + bad_rec));
  if (offsets) {
    for (uint32_t i = tid; i < nrec; i += T) offsets[tile0 + i] = (tile0 + i) * L;
    if (tile0 + nrec == n && tid == 0) offsets[n] = n * L;
  }
}

template <uint32_t T, bool kNT>
__global__ __launch_bounds__(T) void plan_binary_encode_kernel(
    const FixedPlan* __restrict__ pp, const unsigned long long* __restrict__ recs, uint64_t n,
    uint32_t value_words, uint8_t* __restrict__ out, uint64_t* __restrict__ offsets,
    DevResult* __restrict__ res) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t L = pp->wire_len, Q = pp->n_words;
  const uint64_t tile0 = (uint64_t)blockIdx.x * T;
  const uint32_t nrec = (uint32_t)min((uint64_t)T, n - tile0);
  const uint32_t wreg = wire_region(T, L);
  FixedPlan* P = (FixedPlan*)(smem + wreg);
  const uint32_t total = nrec * Q;

  // 1. record words -> registers (coalesced 8-byte loads, issued first)
  unsigned long long vals[kMaxPlanWords];
  {
    uint32_t j = threadIdx.x % Q;
    const uint32_t sj = T % Q;
#pragma unroll
    for (int m = 0; m < kMaxPlanWords; ++m) {
      const uint32_t q = threadIdx.x + T * m;
      vals[m] = 0;
      if ((uint32_t)m < Q && q < total && ((value_words >> j) & 1))
        vals[m] = kNT ? __builtin_nontemporal_load(recs + tile0 * Q + q) : recs[tile0 * Q + q];
      j += sj;
      if (j >= Q) j -= Q;
    }
  }
  // 2. zero the wire tile, plan -> LDS
  uint8_t* gout = out + tile0 * L;
  const uint32_t osh = (uint32_t)((uintptr_t)gout & 15);
  {
    const uint4 z = {0u, 0u, 0u, 0u};
    for (uint32_t i = threadIdx.x; i < (wreg >> 4); i += T) ((uint4*)smem)[i] = z;
  }
  for (uint32_t i = threadIdx.x; i < (uint32_t)(sizeof(FixedPlan) / 16); i += T)
    ((uint4*)P)[i] = ((const uint4*)pp)[i];
  __syncthreads();

  // 3. OR each owned item's wire bytes into the tile
  uint32_t* w32 = (uint32_t*)smem;
  bool bad_bool = false;
  uint32_t bad_rec = 0;
  {
    uint32_t r = threadIdx.x / Q, j = threadIdx.x - r * Q;
    const uint32_t sr = T / Q, sj = T - sr * Q;
#pragma unroll
    for (int m = 0; m < kMaxPlanWords; ++m) {
      const uint32_t q = threadIdx.x + T * m;
      if ((uint32_t)m < Q && q < total) {
        const PlanWord w = P->words[j];
        const unsigned long long v = vals[m];
        const uint32_t base = osh + r * L;
        for (uint32_t k = 0; k < w.n_items; ++k) {
          const PlanItem it = P->items[w.first_item + k];
          const uint32_t h = it.hdr_len;
          const unsigned long long raw = v >> (8 * it.dst);
          unsigned long long vbe;  // big-endian value bytes, first byte lowest
          switch (it.width) {
            case 8:
              vbe = ((unsigned long long)bswap32((uint32_t)raw) << 32) |
                    bswap32((uint32_t)(raw >> 32));
              break;
            case 4: vbe = bswap32((uint32_t)raw); break;
            case 2: vbe = bswap32((uint32_t)(raw & 0xffff)) >> 16; break;
            case 1:
              vbe = raw & 0xff;
              if (it.is_bool && vbe > 1) {  // validate_bool
                bad_bool = true;
                bad_rec = r;
              }
              break;
            default: vbe = 0; break;
          }
          const unsigned long long Flo = (unsigned long long)it.hdr | (vbe << (8 * h));
          const unsigned long long Fhi = h ? (vbe >> (64 - 8 * h)) : 0;
          const uint32_t a = base + it.wire_off;
          const uint32_t d = a >> 2, s = a & 3;
          const unsigned long long Hlo = Flo << (8 * s);
          const unsigned long long Hhi = (Fhi << (8 * s)) | (s ? (Flo >> (64 - 8 * s)) : 0);
          const uint32_t nb = s + h + it.width;
          atomicOr(&w32[d], (uint32_t)Hlo);
          if (nb > 4) atomicOr(&w32[d + 1], (uint32_t)(Hlo >> 32));
          if (nb > 8) atomicOr(&w32[d + 2], (uint32_t)Hhi);
          if (nb > 12) atomicOr(&w32[d + 3], (uint32_t)(Hhi >> 32));
        }
      }
      r += sr;
      j += sj;
      if (j >= Q) {
        j -= Q;
        ++r;
      }
    }
  }
  if (bad_bool) atomicMin(&res->first_fail, (unsigned long long)(tile0 + bad_rec));
  if (offsets) {
    for (uint32_t i = threadIdx.x; i < nrec; i += T) offsets[tile0 + i] = (tile0 + i) * L;
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) offsets[n] = n * L;
  }
  __syncthreads();

  // 4. wire tile -> HBM (full 16-byte chunks; byte stores at the tile edges)
  {
    uint8_t* base = gout - osh;
    const uint32_t end = osh + nrec * L;
    const uint32_t nvec = (end + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nvec; i += T) {
      const uint32_t lo = i << 4, hi = lo + 16;
      if (lo >= osh && hi <= end) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        if (kNT) __builtin_nontemporal_store(((const u32x4*)smem)[i], (u32x4*)base + i);
        else ((uint4*)base)[i] = ((const uint4*)smem)[i];
      } else {
        for (uint32_t b = (lo < osh ? osh : lo); b < (hi < end ? hi : end); ++b) base[b] = smem[b];
      }
    }
  }
}

// ---- variant selection -----------------------------------------------------
// Defaults are the tuned configuration ("fixed-layout kernels");
// TGPU_PLAN_DECODE="T,glds,pair,nt[,ls,chk,tr]" / TGPU_PLAN_ENCODE="T,nt[,ls,tr]"
// override them for tuning runs (tools/kbench.py): ls = the lane-stationary
// forms, chk = their overflowed-list tile verdict, tr = target records per
// tile (R·passes <= tr).
struct DecVariant { uint32_t T; int glds, pair, nt, ls, chk; uint32_t tr; };
struct EncVariant { uint32_t T; int nt, ls; uint32_t tr; };

DecVariant dec_variant() {
  DecVariant v{512, 1, 0, 1, 1, 1, 512};
  if (const char* s = getenv("TGPU_PLAN_DECODE")) {
    unsigned t = 256, tr = 512;
    int g = 0, p = 0, nt = 0, ls = 0, chk = 1;
    const int k = sscanf(s, "%u,%d,%d,%d,%d,%d,%u", &t, &g, &p, &nt, &ls, &chk, &tr);
    if (k >= 4) v = DecVariant{t, g, p, nt, k >= 5 ? ls : 0, chk, tr};
  }
  return v;
}
EncVariant enc_variant() {
  // (256-thread blocks, 512 records per block: 1.953 ms against 1.982 for
  // 512 threads, tools/kbench.py six interleaved rounds on one box,
  // profiles/r05/ab/plan_tile_ab.log)
  EncVariant v{256, 1, 1, 512};
  if (const char* s = getenv("TGPU_PLAN_ENCODE")) {
    unsigned t = 256, tr = 512;
    int nt = 0, ls = 0;
    const int k = sscanf(s, "%u,%d,%d,%u", &t, &nt, &ls, &tr);
    if (k >= 2) v = EncVariant{t, nt, k >= 3 ? ls : 0, tr};
  }
  return v;
}

// KI for the lane-stationary forms: the most items one word holds, rounded up
// to 1 / 2 / 4 / 8 (0 = more than 8: the word-gather form).
uint32_t ls_items(const FixedPlan* p) {
  uint32_t m = 0;
  for (uint32_t j = 0; j < p->n_words; ++j) m = m > p->words[j].n_items ? m : p->words[j].n_items;
  return m <= 1 ? 1 : m <= 2 ? 2 : m <= 4 ? 4 : m <= 8 ? 8 : 0;
}

// Records per pass R = T / Q and passes, so that R·passes <= tr (>= one pass).
void ls_shape(uint32_t T, uint32_t Q, uint32_t tr, uint32_t& R, uint32_t& passes) {
  R = T / Q;
  passes = tr / R;
  if (passes < 1) passes = 1;
  if (passes > (uint32_t)kMaxPlanWords) passes = kMaxPlanWords;
}

template <uint32_t T>
hipError_t launch_dec_T(const DecVariant& v, uint32_t lds, uint64_t blocks, hipStream_t stream,
                        const FixedPlan* d_p, const uint8_t* in, uint64_t n,
                        unsigned long long* out, DevResult* res, uint64_t* exc, uint64_t cap) {
#define TGPU_DEC(G, P_, N)                                                                   \
  if (v.glds == G && v.pair == P_ && v.nt == N) {                                            \
    hipLaunchKernelGGL((plan_binary_decode_kernel<T, G, P_, N>), dim3((uint32_t)blocks),     \
                       dim3(T), lds, stream, d_p, in, n, out, res, exc, cap);                \
    return hipGetLastError();                                                                \
  }
  TGPU_DEC(0, 0, 0) TGPU_DEC(1, 0, 0) TGPU_DEC(0, 1, 0) TGPU_DEC(1, 1, 0)
  TGPU_DEC(0, 0, 1) TGPU_DEC(1, 0, 1) TGPU_DEC(0, 1, 1) TGPU_DEC(1, 1, 1)
#undef TGPU_DEC
  return hipErrorInvalidValue;
}

template <uint32_t T>
hipError_t launch_dec_ls_T(uint32_t KI, int chk, uint32_t R, uint32_t passes, uint32_t lds,
                           uint64_t blocks, hipStream_t stream, const FixedPlan* d_p,
                           const uint8_t* in, uint64_t n, unsigned long long* out, DevResult* res,
                           uint64_t* exc, uint64_t cap) {
#define TGPU_DECLS(K, C)                                                                      \
  if (KI == K && chk == C) {                                                                  \
    hipLaunchKernelGGL((plan_binary_decode_ls_kernel<T, K, true, C>), dim3((uint32_t)blocks), \
                       dim3(T), lds, stream, d_p, in, n, R, passes, out, res, exc, cap);      \
    return hipGetLastError();                                                                 \
  }
  TGPU_DECLS(1, 1) TGPU_DECLS(2, 1) TGPU_DECLS(4, 1) TGPU_DECLS(8, 1)
  TGPU_DECLS(1, 0) TGPU_DECLS(2, 0) TGPU_DECLS(4, 0) TGPU_DECLS(8, 0)
#undef TGPU_DECLS
  return hipErrorInvalidValue;
}

template <uint32_t T>
hipError_t launch_enc_direct_T(uint32_t KI, uint32_t R, uint32_t passes, uint64_t blocks,
                               hipStream_t stream, const FixedPlan* d_p,
                               const unsigned long long* recs, uint64_t n, uint8_t* out,
                               uint64_t* offsets, DevResult* res) {
#define TGPU_ENCD(K, PM)                                                                       \
  if (KI == K && passes <= PM) {                                                               \
    hipLaunchKernelGGL((plan_binary_encode_direct_kernel<T, K, PM>), dim3((uint32_t)blocks),   \
                       dim3(T), 0, stream, d_p, recs, n, R, passes, out, offsets, res);        \
    return hipGetLastError();                                                                  \
  }
  TGPU_ENCD(1, 2) TGPU_ENCD(1, 4) TGPU_ENCD(1, 8) TGPU_ENCD(2, 2) TGPU_ENCD(2, 4) TGPU_ENCD(2, 8)
  TGPU_ENCD(4, 2) TGPU_ENCD(4, 4) TGPU_ENCD(4, 8) TGPU_ENCD(8, 2) TGPU_ENCD(8, 4) TGPU_ENCD(8, 8)
#undef TGPU_ENCD
  return hipErrorInvalidValue;
}

template <uint32_t T>
hipError_t launch_enc_ls_T(uint32_t KI, uint32_t R, uint32_t passes, uint32_t lds,
                           uint64_t blocks, hipStream_t stream, const FixedPlan* d_p,
                           const unsigned long long* recs, uint64_t n, uint8_t* out,
                           uint64_t* offsets, DevResult* res) {
#define TGPU_ENCLS(K, PM)                                                                     \
  if (KI == K && passes <= PM) {  /* the smallest PM that holds the passes */              \
    hipLaunchKernelGGL((plan_binary_encode_ls_kernel<T, K, PM, true>), dim3((uint32_t)blocks), \
                       dim3(T), lds, stream, d_p, recs, n, R, passes, out, offsets, res);     \
    return hipGetLastError();                                                                 \
  }
  TGPU_ENCLS(1, 4) TGPU_ENCLS(1, 10) TGPU_ENCLS(1, 20) TGPU_ENCLS(2, 4) TGPU_ENCLS(2, 10)
  TGPU_ENCLS(2, 20) TGPU_ENCLS(4, 4) TGPU_ENCLS(4, 10) TGPU_ENCLS(4, 20) TGPU_ENCLS(8, 4)
  TGPU_ENCLS(8, 10) TGPU_ENCLS(8, 20)
#undef TGPU_ENCLS
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_plan_binary_decode(const FixedPlan* p, const FixedPlan* d_p, const uint8_t* in,
                                     uint64_t n, uint8_t* out, DevResult* res, uint64_t* exc,
                                     uint64_t exc_cap, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const DecVariant v = dec_variant();
  auto* o = (unsigned long long*)out;
  const uint32_t KI = ls_items(p);
  if (v.ls && KI && (v.T == 256 || v.T == 512) && p->n_words <= v.T) {
    uint32_t R, passes;
    ls_shape(v.T, p->n_words, v.tr, R, passes);
    const uint32_t TR = R * passes;
    if (TR <= 2048) {
      const uint64_t blocks = (n + TR - 1) / TR;
      const uint32_t lds = ls_wire_region(v.T, TR, p->wire_len) + ((TR + 31) / 32 + 1) * 4;
      if (v.T == 256)
        return launch_dec_ls_T<256>(KI, v.chk, R, passes, lds, blocks, stream, d_p, in, n, o, res,
                                    exc, exc_cap);
      return launch_dec_ls_T<512>(KI, v.chk, R, passes, lds, blocks, stream, d_p, in, n, o, res,
                                  exc, exc_cap);
    }
  }
  DecVariant use = v;
  if (((uintptr_t)out & 15) != 0) use.pair = 0;  // 16-byte stores need 16-byte records base
  const uint64_t blocks = (n + use.T - 1) / use.T;
  // + the tile's bitmap of exception records (one bit per record) + its verdict
  const uint32_t lds =
      wire_region(use.T, p->wire_len) + (uint32_t)sizeof(FixedPlan) + use.T / 8 + 16;
  switch (use.T) {
    case 128: return launch_dec_T<128>(use, lds, blocks, stream, d_p, in, n, o, res, exc, exc_cap);
    case 512: return launch_dec_T<512>(use, lds, blocks, stream, d_p, in, n, o, res, exc, exc_cap);
    default: return launch_dec_T<256>(use, lds, blocks, stream, d_p, in, n, o, res, exc, exc_cap);
  }
}

hipError_t launch_plan_binary_encode(const FixedPlan* p, const FixedPlan* d_p,
                                     const uint8_t* recs, uint64_t n, uint8_t* out,
                                     uint64_t* offsets, DevResult* res, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const EncVariant v = enc_variant();
  const uint32_t KI = ls_items(p);
  if (v.ls && KI && (v.T == 256 || v.T == 512) && p->n_words <= v.T) {
    uint32_t R, passes;
    ls_shape(v.T, p->n_words, v.tr, R, passes);
    const uint32_t TR = R * passes;
    const uint64_t blocks = (n + TR - 1) / TR;
    const uint32_t lds = ls_wire_region(v.T, TR, p->wire_len);
    const auto* r = (const unsigned long long*)recs;
    if (v.ls == 2 && passes <= 8) {  // (the direct form: no LDS tile)
      if (v.T == 256)
        return launch_enc_direct_T<256>(KI, R, passes, blocks, stream, d_p, r, n, out, offsets,
                                        res);
      return launch_enc_direct_T<512>(KI, R, passes, blocks, stream, d_p, r, n, out, offsets, res);
    }
    if (v.T == 256)
      return launch_enc_ls_T<256>(KI, R, passes, lds, blocks, stream, d_p, r, n, out, offsets, res);
    return launch_enc_ls_T<512>(KI, R, passes, lds, blocks, stream, d_p, r, n, out, offsets, res);
  }
  uint32_t value_words = 0;
  for (uint32_t j = 0; j < p->n_words; ++j)
    if (p->words[j].has_value) value_words |= 1u << j;
  const uint64_t blocks = (n + v.T - 1) / v.T;
  const uint32_t lds = wire_region(v.T, p->wire_len) + (uint32_t)sizeof(FixedPlan);
  const auto* r = (const unsigned long long*)recs;
#define TGPU_ENC(TT, N)                                                                        \
  if (v.T == TT && v.nt == N) {                                                                \
    hipLaunchKernelGGL((plan_binary_encode_kernel<TT, N>), dim3((uint32_t)blocks), dim3(TT), lds, \
                       stream, d_p, r, n, value_words, out, offsets, res);                     \
    return hipGetLastError();                                                                  \
  }
  TGPU_ENC(128, 0) TGPU_ENC(128, 1) TGPU_ENC(256, 0) TGPU_ENC(256, 1) TGPU_ENC(512, 0)
  TGPU_ENC(512, 1)
#undef TGPU_ENC
  return hipErrorInvalidValue;
}

}  // namespace tgpu

#ifdef TGPU_PLAN_STALE_CHECK
// (diagnostics build only: not in thrift_gpu.h) the stale-word counter
extern "C" unsigned long long tgpu_debug_plan_stale(int reset) {
  unsigned long long v = 0;
  (void)hipDeviceSynchronize();
  (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(tgpu_plan_stale_words), sizeof(v));
  if (reset) {
    const unsigned long long z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(tgpu_plan_stale_words), &z, sizeof(z));
  }
  (void)hipGetLastError();
  return v;
}
#endif
