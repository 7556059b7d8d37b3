// tgpu_prog_kernels.h — bodies of the compiled-program kernels, templated on
// the program accessor (tgpu_program.h). The AOT library instantiates them
// with DynProg (k_program.hip, k_program_enc.hip, k_index.hip); the schema
// kernels generated at run time instantiate them with the schema's ops as
// compile-time constants (tgpu_jit.cpp). Not part of the public ABI.
//
//   decode_tile  indexed decode of one 256-record tile (configs 3, 4)
//   size_tile    encode pass 1: per-record wire size + tile sum
//   write_tile   encode pass 3: records -> LDS output tile -> HBM
//   index_spec_tile / index_emit_tile  stream index over one LDS tile
#pragma once

#include "tgpu_program.h"

namespace tgpu {
namespace prog {

constexpr uint32_t kPT = 256;            // decode: records per tile = threads per workgroup
constexpr uint32_t kET = 256;            // encode: records per tile = threads per workgroup
constexpr uint32_t kOutCap = 24 * 1024;  // encode: LDS bytes for one tile's wire output

// ---- block helpers (256 threads) --------------------------------------------
// Workgroup barrier ordering LDS only: unlike __syncthreads it does not wait
// for the wave's outstanding global loads/stores (s_waitcnt vmcnt(0)), so a
// prefetch issued before it stays in flight across it.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long x) {
  const int lane = threadIdx.x & 63;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// exclusive scan across the block; *total = block sum (all threads)
__device__ __forceinline__ unsigned long long block_exscan256(unsigned long long v,
                                                              unsigned long long* part,
                                                              unsigned long long* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long x = wave_incl_scan(v);
  if (lane == 63) part[wid] = x;
  __syncthreads();
  unsigned long long pre = 0;
  for (int w = 0; w < wid; ++w) pre += part[w];
  *total = part[0] + part[1] + part[2] + part[3];
  return pre + x - v;
}

// ================================================================ decode ======
// One lane runs the program over one record of the tile:
//   * the tile's bytes [offs[r0], offs[r0+256]) go HBM -> LDS with coalesced
//     16-byte loads (a tile larger than wire_cap falls back);
//   * each lane reads its record from LDS through 8-byte windows, decodes
//     varints branch-free, and writes the record into an LDS record tile
//     (strings become zero-copy views; list elements go to the arena);
//   * the record tile goes LDS -> HBM with coalesced 16-byte stores.
// (A persistent, register-prefetching form — each workgroup looping over
// tiles with the next tile's bytes in flight — measured slower: 2.7 vs
// 1.85 ms on config 3, the prefetch buffer spilled to scratch.)
// A record that deviates from the canonical form in any way is NOT decided
// here: its index is appended to `irr` and the general decoder (full
// readNoXfer semantics, tgpu_device.h) decodes it.
// smem: decode_wire_region(wire_cap) bytes of wire tile, then kPT * S + 16
// record tile.
__host__ __device__ __forceinline__ uint32_t decode_wire_region(uint32_t wire_cap) {
  return (wire_cap + 32 + 16 * kPT - 1) / (16 * kPT) * (16 * kPT);  // whole staging rounds
}
// Bytes of the LDS record tile (decode_tile without kRS).
__host__ __device__ __forceinline__ uint32_t decode_rtile_bytes(uint32_t S) {
  return (kPT * S + 16 + 15) & ~15u;
}
template <uint32_t kRS>
__device__ __forceinline__ void store_reg_record(uint8_t* go, const uint8_t* rbuf,
                                                 const uint8_t* recs) {
  // (16-byte stores of a lane's record, TGPU_RR_STORE16: the same time but
  // +27 B fetched and +40 B written per config-4 record in the PMC counters
  // — 64 lanes' 16-byte pieces at a 64-byte stride; round 6)
#ifdef TGPU_RR_STORE16
  if constexpr (kRS % 16 == 0) {
    if (((uintptr_t)recs & 15) == 0) {  // whole 16-byte words (S 64: a record = 4 stores)
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (uint32_t b = 0; b < kRS; b += 16) *(u32x4*)(go + b) = *(const u32x4*)(rbuf + b);
      return;
    }
  }
#endif
  if (((uintptr_t)recs & 7) == 0) {  // (the batch's records: 8- or 4-byte aligned)
#pragma unroll
    for (uint32_t b = 0; b < kRS; b += 8) *(uint64_t*)(go + b) = *(const uint64_t*)(rbuf + b);
  } else {
#pragma unroll
    for (uint32_t b = 0; b < kRS; b += 4) *(uint32_t*)(go + b) = *(const uint32_t*)(rbuf + b);
  }
}

// The block rule in a compiled Binary decode tile (kArenaBlock = 64: a
// block is one wave's records). The wave's records took the program (else it
// returns false and the wave keeps the position rule): their list elements
// sit converted in the LDS wire tile, inside the wave's own wire bytes. Each
// lane takes its arrays' bytes into registers (8-byte words, at most
// kPackWords per record, else false), the wave's exclusive scan gives each
// record its packed offset, the lanes write their words back into the
// wave's wire range at the packed image's position (an array never moves
// up, and every read of the wave precedes its writes: no other wave reads
// these bytes), and the wave stores the image with 16-byte vectors, whole
// lines of the arena — the element bytes only, 32 B / record on config 4
// against 89 for the position rule's converted wire tile. Spans rewritten.
// (Measured and dropped, round 6: a block of 256 records with a block scan,
// the lanes storing their own arrays with 8-byte stores — 1.92 ms against
// 1.69 for the position rule on config 4, the scattered stores cost 0.39
// ms; the same with whole vectors gathered through a binary search of an
// LDS array table — 1.82 ms.)
constexpr uint32_t kPackWords = 8;  // 64 bytes of arrays per record (config 4: 16 x i32)
template <class PP, uint32_t kK>
// (`rec` is always a valid record buffer, `active` says whether the lane
// has a record: a pointer that may be null kept the register record of the
// `_rr` tile out of registers — 32 bytes of scratch per lane, round 6)
__device__ __forceinline__ bool pack_wave(const DecodeArgs& a, const PP& P, uint8_t* rec,
                                          bool active, bool lane_ok, uint64_t rstart,
                                          uint64_t t0, uint32_t sh, uint8_t* wire) {
  if (__ballot(active && !lane_ok)) return false;  // (wave-uniform)
  const uint64_t act = __ballot(active);
  if (!act) return true;
  uint32_t o[kK > 0 ? kK : 1], by[kK > 0 ? kK : 1], ps[kK > 0 ? kK : 1];
  uint32_t size = 0;
  {
    uint32_t k = 0;
    all_ops(P, [&](const VOp op) {
      if (op.kind == VOP_LIST) {
        const tgpu_span sp = active ? *(const tgpu_span*)(rec + op.member) : tgpu_span{0, 0, 0};
        by[k] = sp.length * op.width;
        ps[k] = by[k] ? (uint32_t)(sp.offset - (t0 - sh)) : 0u;  // LDS position
        o[k] = size;
        size += (by[k] + 7) & ~7u;
        ++k;
      }
      return true;
    });
  }
  if (__ballot(size > 8 * kPackWords)) return false;
  const uint64_t incl = wave_incl_scan(size);
  const uint32_t pre = (uint32_t)(incl - size);
  const uint32_t wsize = (uint32_t)__shfl(incl, 63, 64);
  const uint64_t base = (__shfl(rstart, 0, 64) + 7) & ~7ull;  // align8(scale x start), scale 1
  if (base + wsize > a.arena_cap) return false;
  // the lane's packed words: word j is array k's bytes from 8j - o[k]
  const LdsSrc src{(const uint32_t*)wire};
  uint64_t w[kPackWords];
#pragma unroll
  for (uint32_t j = 0; j < kPackWords; ++j) {
    uint32_t from = 0;
    bool have = false;
#pragma unroll
    for (uint32_t k = 0; k < kK; ++k)
      if (8 * j >= o[k] && 8 * j < o[k] + by[k]) from = ps[k] + 8 * j - o[k], have = true;
    w[j] = have ? src.win8(from) : 0ull;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  // the image: LDS position q <-> arena offset (t0 - sh) + q (the staging's
  // congruence: both 16-byte aligned at q = 0), so 8-byte aligned
  const uint32_t q0 = (uint32_t)(base - (t0 - sh));
#pragma unroll
  for (uint32_t j = 0; j < kPackWords; ++j)
    if (8 * j < size) *(uint64_t*)(wire + q0 + pre + 8 * j) = w[j];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  // LDS [q0, q0 + wsize) -> arena [base, base + wsize): 16-byte vectors, the
  // edge halves as 8-byte stores
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t v0 = q0 >> 4, v1 = (q0 + wsize + 15) >> 4;
  uint8_t* gb = a.arena + (t0 - sh);  // LDS position 0's arena address (16-byte aligned)
  for (uint32_t v = v0 + lane; v < v1; v += 64) {
    const uint32_t lo = v << 4, hi = lo + 16;
    if (lo >= q0 && hi <= q0 + wsize) {
#ifdef TGPU_PACK_PLAIN_STORE  // (A/B)
      *((u32x4*)gb + v) = ((const u32x4*)wire)[v];
#else
      __builtin_nontemporal_store(((const u32x4*)wire)[v], (u32x4*)gb + v);
#endif
    } else {
      if (lo >= q0) ((uint64_t*)gb)[2 * v] = ((const uint64_t*)wire)[2 * v];
      if (hi <= q0 + wsize) ((uint64_t*)gb)[2 * v + 1] = ((const uint64_t*)wire)[2 * v + 1];
    }
  }
  if (active) {
    uint32_t k = 0;
    all_ops(P, [&](const VOp op) {
      if (op.kind == VOP_LIST) {
        tgpu_span* sp = (tgpu_span*)(rec + op.member);
        sp->offset = by[k] ? base + pre + o[k] : 0;
        ++k;
      }
      return true;
    });
  }
  return true;
}

// kTail: the stream-ordered fixed-layout tail (DevResult tail_*): records
// r0.. of the tile at pos + (i - first) * stride; their offsets are written,
// a record not taken is listed (wave-aggregated atomics: a wrong stride
// fails every record) and moves tail_min instead of first_irregular.
struct TailStride {
  uint64_t first, pos, stride, r0;
};
// kRS > 0 (= S, a multiple of 8, <= 128): each lane builds its record in
// registers and stores it with 8-byte stores (no LDS record tile: the
// workgroup's LDS is the wire tile alone, so more workgroups share a CU).
template <class PP, bool kTail = false, uint32_t kRS = 0>
__device__ __forceinline__ void decode_tile(const DecodeArgs& a, const PP& P, uint32_t S,
                                            uint32_t wire_cap, uint64_t* __restrict__ irr,
                                            unsigned long long* __restrict__ nirr,
                                            uint8_t* smem, const TailStride& ts = {}) {
  static_assert(kRS % 8 == 0 && kRS <= 128, "register record: whole 8-byte words");
  uint8_t* wire = smem;
  uint8_t* rtile = smem + decode_wire_region(wire_cap);
  const uint64_t r0 = kTail ? ts.r0 : (uint64_t)blockIdx.x * kPT;
  const uint64_t n_all = !kTail && a.n_dev ? min(a.n, (uint64_t)*a.n_dev) : a.n;
  if (r0 >= n_all) return;  // (whole workgroup)
  const uint32_t nrec = (uint32_t)min((uint64_t)kPT, n_all - r0);
  const uint64_t L = kTail ? ts.stride : a.fixed_len;
  const uint64_t b0 = kTail ? ts.pos - ts.first * L : 0;  // record i at b0 + i * L
  const uint64_t t0 = L ? b0 + r0 * L : a.offs[r0];
  const uint64_t t1 = L ? b0 + (r0 + nrec) * L : a.offs[r0 + nrec];
  const bool tile_ok = t1 >= t0 && t1 <= a.in_len && (t1 - t0) + 16 <= wire_cap;
  uint32_t sh = 0;
  if (tile_ok) {
    const uint8_t* g = a.in + t0;
    sh = (uint32_t)((uintptr_t)g & 15);
    const uint4* src = (const uint4*)(g - sh);
    const uint32_t nvec = (uint32_t)((t1 - t0) + sh + 15) >> 4;
    // LDS DMA (global_load_lds_dwordx4): the bytes go HBM -> LDS without
    // registers; lanes past the tile re-read its last vector into the slack
    // (measured faster than masking them off)
    const uint32_t wave = threadIdx.x >> 6;
    for (uint32_t k = 0; k * kPT < nvec; ++k) {
      const uint32_t i = k * kPT + threadIdx.x;
      __builtin_amdgcn_global_load_lds(
          (const void*)(src + (i < nvec ? i : nvec - 1)),
          (__attribute__((address_space(3))) void*)(wire + (size_t)(k * kPT + wave * 64) * 16), 16,
          0, 0);
    }
#ifndef TGPU_NO_DMA_SETTLE
    lds_dma_settle(wire, threadIdx.x, kPT, (nvec + kPT - 1) / kPT);
#endif
  }
  uint8_t* gout = a.recs + r0 * S;
  const uint32_t osh = (uint32_t)((uintptr_t)gout & 15);
  if constexpr (kRS == 0) {
    const uint4 z = {0u, 0u, 0u, 0u};
    const uint32_t nz = (kPT * S + osh + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nz; i += kPT) ((uint4*)rtile)[i] = z;
  }
  __syncthreads();

  // Binary lists: elements converted in place in the wire tile (an element's
  // arena slot is its own wire bytes), then the whole tile goes to the arena
  // with coalesced 16-byte stores (arena and stream 16-byte congruent; arena
  // bytes outside spans are unspecified). Config 4 decode: per-element 4-byte
  // stores 2.27 ms, whole-tile copy 1.82 ms, each lane copying its own lists
  // with 16-byte stores 3.15 ms.
  const bool stage_lists = P.has_lists() && P.protocol() == TGPU_PROTOCOL_BINARY && tile_ok &&
                           a.arena && t1 <= a.arena_cap &&
                           (((uintptr_t)a.arena - (uintptr_t)a.in) & 15) == 0;
  // Block rule (round 6, ArenaPack): a compiled Binary program packs the
  // element arrays itself, each wave its block of kArenaBlock records
  // (pack_wave) when all of them took the program; otherwise the wave keeps
  // the position rule and arena_pack_kernel packs its block later.
  constexpr uint32_t kK = (PP::kStatic && !kTail) ? PP::kLists : 0;
  static_assert(kArenaBlock == 64 && kPT % kArenaBlock == 0, "an arena block is one wave's records");
  const bool pack_on = kK > 0 && kK <= kPackSlots && stage_lists && !L && a.pack_flags &&
                       a.pack_k == kK && ((uintptr_t)a.arena & 7) == 0;
  const uint32_t r = threadIdx.x;
  bool failed = false;
  bool lane_ok = true;
  alignas(16) uint8_t rbuf[kRS ? kRS : 8];
  if (r < nrec) {
    uint8_t* rec = kRS ? rbuf : rtile + osh + r * S;
    if constexpr (kRS != 0) {
#pragma unroll
      for (uint32_t b = 0; b < kRS; b += 8) *(uint64_t*)(rbuf + b) = 0;
    }
    bool ok = tile_ok;
    if (ok) {
      const uint64_t s = L ? t0 + r * L : a.offs[r0 + r], e = L ? s + L : a.offs[r0 + r + 1];
      ok = s >= t0 && e >= s && e <= t1;
      if (ok) {
        const Ctx c{t0 - sh, a.arena, a.arena_cap, a.string_limit, a.container_limit,
                    stage_lists ? wire : nullptr};
        const LdsSrc src{(const uint32_t*)wire};
        uint32_t p = (uint32_t)(s - t0) + sh;
        const uint32_t pe = (uint32_t)(e - t0) + sh;
        ok = run_program<true>(P, src, c, p, pe, rec) && p == pe;
      }
    }
    lane_ok = ok;
    // (pack mode stores the register record once its spans are final)
    if constexpr (kRS != 0) {
      if (!pack_on) store_reg_record<kRS>(gout + (uint64_t)r * kRS, rbuf, a.recs);
    }
    if constexpr (kTail) {
      failed = !ok;
      if (a.offs) {
        uint64_t* offs = const_cast<uint64_t*>(a.offs);
        offs[r0 + r] = t0 + r * L;
        if (r0 + r + 1 == a.n) offs[a.n] = t1;
      }
    } else if (!ok) {
      // general decoder list; a fixed-stride batch's exception list (irr ==
      // a.exc, read again at the stride position by fixed_exception_kernel)
      const unsigned long long k = atomicAdd(nirr, 1ull);
      if (!L || k < a.exc_cap) irr[k] = r0 + r;
      if (L) atomicMin(&a.res->first_irregular, (unsigned long long)(r0 + r));
    }
  }
  if constexpr (kTail) {
    const uint64_t bad = __ballot(failed);
    if (bad) {
      const uint32_t lane = threadIdx.x & 63, lead = (uint32_t)__builtin_ctzll(bad);
      unsigned long long k0 = 0;
      if (lane == lead) {
        k0 = atomicAdd(nirr, (unsigned long long)__builtin_popcountll(bad));
        atomicMin(&a.res->tail_min, (unsigned long long)(r0 + r));
      }
      k0 = __shfl(k0, (int)lead, 64);
      const unsigned long long k = k0 + __builtin_popcountll(bad & ((1ull << lane) - 1));
      if (failed && k < a.exc_cap) irr[k] = r0 + r;
    }
  }
  // (wave-local packing touches only its own records' wire bytes, but
  // dropping this barrier for it measured slower: config 4 decode 2.24 vs
  // 2.12 ms, pack_ab round 6 — the waves of a tile then store at once)
  __syncthreads();
  bool packed = false;  // (the tile's arena bytes are written: skip the tile copy)
  if constexpr (kK > 0) {
    if (pack_on) {
      // each wave its own block (kArenaBlock = 64 records): packed, or its
      // converted wire range as the position rule has it
      const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
      const uint64_t rs = r < nrec ? a.offs[r0 + r] : 0;
      uint8_t* rec = kRS ? rbuf : rtile + osh + r * S;  // (inside the tile for r >= nrec)
      const bool wpacked = pack_wave<PP, kK>(a, P, rec, r < nrec, lane_ok, rs, t0, sh, wire);
      // the register records leave through the dead wire tile when it holds
      // them (after every wave's packing): whole lines instead of each
      // lane's 64-byte record in 8-byte pieces (TGPU_RR_LANE_STORES: those)
#ifdef TGPU_RR_LANE_STORES
      constexpr bool kStageRecs = false;
#else
      constexpr bool kStageRecs = kRS != 0;
#endif
      const bool stage_recs = kStageRecs && ((uintptr_t)gout & 7) == 0 &&
                              osh + kPT * kRS <= decode_wire_region(wire_cap);
      if constexpr (kRS != 0) {
        if (r < nrec && !stage_recs) store_reg_record<kRS>(gout + (uint64_t)r * kRS, rbuf, a.recs);
      }
      const uint32_t wr0 = wv * 64;
      if (wr0 < nrec) {
        if (wpacked) {
          if (lane == 0) a.pack_flags[(r0 >> 6) + wv] = a.pack_epoch;
        } else {
          // the wave's records' bytes [offs[wr0], offs[wr1]) of the converted
          // tile -> arena, 16-byte vectors (byte stores on the edges shared
          // with the neighbouring waves)
          const uint32_t wr1 = min(nrec, wr0 + 64);
          const uint32_t lo_b = (uint32_t)(a.offs[r0 + wr0] - t0) + sh;
          const uint32_t hi_b = (uint32_t)(a.offs[r0 + wr1] - t0) + sh;
          uint8_t* ab = a.arena + t0 - sh;
          for (uint32_t i = (lo_b >> 4) + lane; i < ((hi_b + 15) >> 4); i += 64) {
            const uint32_t lo = i << 4, hi = lo + 16;
            if (lo >= lo_b && hi <= hi_b) {
              ((uint4*)ab)[i] = ((const uint4*)wire)[i];
            } else {
              for (uint32_t b = (lo < lo_b ? lo_b : lo); b < (hi < hi_b ? hi : hi_b); ++b)
                ab[b] = wire[b];
            }
          }
        }
      }
      packed = true;
      if constexpr (kRS != 0) {
        if (stage_recs) {
          __syncthreads();  // every wave's packing / range copy has read its wire bytes
          if (r < nrec) {
#pragma unroll
            for (uint32_t b = 0; b < kRS; b += 8)
              *(uint64_t*)(wire + osh + r * kRS + b) = *(const uint64_t*)(rbuf + b);
          }
          __syncthreads();
          const uint32_t end = osh + nrec * kRS;
          uint8_t* base = gout - osh;
          for (uint32_t i = threadIdx.x; i < ((end + 15) >> 4); i += kPT) {
            const uint32_t lo = i << 4, hi = lo + 16;
            if (lo >= osh && hi <= end) {
              ((uint4*)base)[i] = ((const uint4*)wire)[i];
            } else {  // (8-byte aligned records: the edge halves)
              if (lo >= osh) ((uint64_t*)base)[2 * i] = ((const uint64_t*)wire)[2 * i];
              if (hi <= end) ((uint64_t*)base)[2 * i + 1] = ((const uint64_t*)wire)[2 * i + 1];
            }
          }
        }
        return;
      }
      // (the record tile leaves below in 16-byte chunks that cross the waves'
      // records: every wave's span rewrite must be in LDS first)
      __syncthreads();
    }
  }
  if (stage_lists && !packed) {  // converted wire tile -> arena [t0, t1), coalesced
    const uint32_t wend = sh + (uint32_t)(t1 - t0);
    uint8_t* ab = a.arena + t0 - sh;
    for (uint32_t i = threadIdx.x; i < ((wend + 15) >> 4); i += kPT) {
      const uint32_t lo = i << 4, hi = lo + 16;
      if (lo >= sh && hi <= wend) {
        ((uint4*)ab)[i] = ((const uint4*)wire)[i];
      } else {
        for (uint32_t b = (lo < sh ? sh : lo); b < (hi < wend ? hi : wend); ++b) ab[b] = wire[b];
      }
    }
  }
  if constexpr (kRS != 0) return;
  // record tile -> HBM
  const uint32_t end = osh + nrec * S;
  const uint32_t nvec = (end + 15) >> 4;
  uint8_t* base = gout - osh;
  for (uint32_t i = threadIdx.x; i < nvec; i += kPT) {
    const uint32_t lo = i << 4, hi = lo + 16;
    if (lo >= osh && hi <= end) {
      ((uint4*)base)[i] = ((const uint4*)rtile)[i];
    } else {
      for (uint32_t b = (lo < osh ? osh : lo); b < (hi < end ? hi : end); ++b) base[b] = rtile[b];
    }
  }
}

// ================================================================ encode ======
__device__ __forceinline__ uint32_t varint_len(uint64_t v) {
  const uint32_t bits = 64 - (uint32_t)__builtin_clzll(v | 1);
  return (bits + 6) / 7;
}

__device__ __forceinline__ uint64_t load_member(const uint8_t* p, uint32_t width) {
  switch (width) {
    case 8: return *(const uint64_t*)p;
    case 4: return *(const uint32_t*)p;
    case 2: return *(const uint16_t*)p;
    default: return *p;
  }
}

// zigzag of a signed member of `width` bytes, as i32 (bits 32) or i64
__device__ __forceinline__ uint64_t zz_member(uint64_t raw, uint32_t width, uint32_t bits) {
  int64_t v;
  switch (width) {
    case 2: v = (int16_t)(uint16_t)raw; break;
    case 4: v = (int32_t)(uint32_t)raw; break;
    default: v = (int64_t)raw; break;
  }
  if (bits == 32) return i32_to_zz((int32_t)v);
  return i64_to_zz(v);
}

// A record's members as the encoder reads them: PtrRec through a pointer
// (HBM or the LDS record tile), RegRec from registers — the record loaded
// once at the start of the write pass (8-byte loads), every member access a
// constant register select in the compiled programs (their offsets fold).
struct PtrRec {
  const uint8_t* p;
  __device__ __forceinline__ uint32_t u8(uint32_t off) const { return p[off]; }
  __device__ __forceinline__ uint64_t member(uint32_t off, uint32_t width) const {
    return load_member(p + off, width);
  }
  __device__ __forceinline__ tgpu_span span(uint32_t off) const {
    return *(const tgpu_span*)(p + off);
  }
};
template <uint32_t S>
struct RegRec {
  static constexpr uint32_t kW = (S + 7) / 8 * 2;
  uint32_t w[kW];
  __device__ __forceinline__ void load(const uint8_t* p) {
    // records are at least 8-byte aligned when S % 8 == 0 (i64/double/span
    // members); otherwise 4-byte loads
    if constexpr (S % 8 == 0) {
#pragma unroll
      for (uint32_t i = 0; i < S / 8; ++i) {
        const uint2 v = ((const uint2*)p)[i];
        w[2 * i] = v.x;
        w[2 * i + 1] = v.y;
      }
    } else {
#pragma unroll
      for (uint32_t i = 0; i < kW; ++i) w[i] = i * 4 < S ? ((const uint32_t*)p)[i] : 0u;
    }
  }
  __device__ __forceinline__ uint32_t u8(uint32_t off) const {
    return (w[off >> 2] >> (8 * (off & 3))) & 0xffu;
  }
  __device__ __forceinline__ uint64_t member(uint32_t off, uint32_t width) const {
    // members at natural alignment
    switch (width) {
      case 8: return ((uint64_t)w[(off >> 2) + 1] << 32) | w[off >> 2];
      case 4: return w[off >> 2];
      case 2: return (w[off >> 2] >> (8 * (off & 3))) & 0xffffu;
      default: return u8(off);
    }
  }
  __device__ __forceinline__ tgpu_span span(uint32_t off) const {
    tgpu_span sp;
    sp.offset = ((uint64_t)w[(off >> 2) + 1] << 32) | w[off >> 2];
    sp.length = w[(off >> 2) + 2];
    sp.reserved = 0;
    return sp;
  }
};

// list elements of `width` bytes from HBM, kElemBatch loads in flight
#ifndef TGPU_ELEM_BATCH
#define TGPU_ELEM_BATCH 8
#endif
// 4- and 8-byte elements as 16-byte vectors of the aligned blocks they
// occupy (str_load32 / str_shift below): each batch takes the whole elements
// of the 32 bytes from the batch's first element on. TGPU_ELEM_X4=0: one
// load per element (A/B).
#ifndef TGPU_ELEM_X4
#define TGPU_ELEM_X4 1
#endif
__device__ __forceinline__ void str_load32(uint32_t (&v)[8], const uint8_t* __restrict__ blk,
                                           uint32_t nvec);
__device__ __forceinline__ void str_shift(uint32_t (&v)[8], uint32_t off);
template <class F>
__device__ __forceinline__ void for_elems(const uint8_t* __restrict__ e, uint32_t len,
                                          uint32_t width, F&& f) {
  constexpr uint32_t B = TGPU_ELEM_BATCH;
#if TGPU_ELEM_X4
  if (width == 4 || width == 8) {
    uint32_t left = len;
    while (left) {
      const uint32_t off = (uint32_t)((uintptr_t)e & 15);
      const uint32_t fit = (32 - off) / width;  // whole elements in this batch's window
      const uint32_t m = left < fit ? left : fit;
      const uint32_t nv = (off + m * width + 15) >> 4;
      uint32_t v[8];
      str_load32(v, e - off, nv < 2 ? nv : 2);
      str_shift(v, off);
      if (width == 4) {
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k)
          if (k < m) f((uint64_t)v[k]);
      } else {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
          if (k < m) f(((uint64_t)v[2 * k + 1] << 32) | v[2 * k]);
      }
      e += m * width;
      left -= m;
    }
    return;
  }
#endif
  if constexpr (B == 1) {
    for (uint32_t i = 0; i < len; ++i) f(load_member(e + (uint64_t)i * width, width));
  } else {
    for (uint32_t i0 = 0; i0 < len; i0 += B) {
      uint64_t v[B];
#pragma unroll
      for (uint32_t k = 0; k < B; ++k)
#ifndef TGPU_NO_ELEM_LOAD  // A/B only (tools/kbench_jit.py --no-check): cost of the loads
        v[k] = i0 + k < len ? load_member(e + (uint64_t)(i0 + k) * width, width) : 0;
#else
        v[k] = i0 + k;
#endif
#pragma unroll
      for (uint32_t k = 0; k < B; ++k)
        if (i0 + k < len) f(v[k]);
    }
  }
}

// Bytes T::write emits for the record at `rec`; ok = false where the writer
// would throw or abort (the finish kernel re-derives the exact code).
// Size of a record whose string or list length fails the writer's size check
// (> INT32_MAX): larger than any output buffer, so the write pass never
// emits it (emission would copy `length` bytes) and reports the record.
constexpr uint64_t kNeverFits = 1ull << 44;

template <class PP, class R>
__device__ __forceinline__ uint64_t program_size(const PP& P, const R& rec,
                                                 const uint8_t* __restrict__ lbase, bool& ok) {
  const bool compact = P.protocol() == TGPU_PROTOCOL_COMPACT;
  uint64_t n = 0;
  all_ops(P, [&](const VOp op) {
    switch (op.kind) {
      case VOP_CONST:
        n += op.hdr_len;
        break;
      case VOP_CBOOL:
        if (rec.u8(op.member) > 1) ok = false;
        n += op.hdr_len;
        break;
      case VOP_FIXED:
        if (op.is_bool && rec.u8(op.member) > 1) ok = false;
        n += op.width;
        break;
      case VOP_VARINT:
        n += varint_len(zz_member(rec.member(op.member, op.width), op.width, op.bits));
        break;
      case VOP_STRING: {
        const uint32_t len = rec.span(op.member).length;
        if (len > 0x7fffffffu) {  // checkBinarySize: never emitted (see kNeverFits)
          ok = false;
          n += kNeverFits;
          break;
        }
        n += (compact ? varint_len(len) : 4) + (uint64_t)len;
        break;
      }
      case VOP_LIST: {
        const tgpu_span sp = rec.span(op.member);
        const uint32_t len = sp.length;
        if (len > 0x7fffffffu) {
          ok = false;
          n += kNeverFits;
          break;
        }
        n += compact ? (len <= 14 ? 1 : 1 + varint_len(len)) : 5;
        const uint8_t* e = lbase + sp.offset;
        if (op.elem_kind == VEL_VARINT) {
          for_elems(e, len, op.width, [&](uint64_t x) {
            n += varint_len(zz_member(x, op.width, op.bits));
          });
        } else if (op.elem_kind == VEL_BOOL) {
          for_elems(e, len, 1, [&](uint64_t x) {
            if (x > 1) ok = false;
          });
          n += len;
        } else {
          n += (uint64_t)len * op.width;
        }
        break;
      }
      default:
        break;
    }
    return true;
  });
  return n;
}

// ---- record emission ----------------------------------------------------------
// A sink appends little-endian packed bytes: put(v, n <= 4), put64(v, n <= 8)
// (bytes of v past n are ignored).
//   OrSink   — the zero-filled LDS output tile: every put ORs its bytes into
//              the (up to three) dwords they cover with ds_or_b32 — no
//              branches, no per-lane state beyond the position; bytes a
//              record shares a dword with its neighbour merge by the OR.
//   ByteSink — HBM directly, a byte at a time (records past the LDS tile).
// (A dword-assembling sink that flushed full dwords measured ~25 % slower:
// its per-put flush branch left the unrolled emitter with thousands of
// divergent basic blocks and SGPR spills.)
struct OrSink {
  uint32_t* w32;
  uint32_t q;
  __device__ __forceinline__ OrSink(uint32_t* tile, uint32_t pos) : w32(tile), q(pos) {}
  __device__ __forceinline__ void put64(uint64_t v, uint32_t n) {
    if (n < 8) v &= (1ull << (8 * n)) - 1;
    const uint32_t d = q >> 2, sh = 8 * (q & 3);
    const uint64_t lo = v << sh;
    const uint32_t hi = sh ? (uint32_t)(v >> (64 - sh)) : 0u;
    atomicOr(&w32[d], (uint32_t)lo);
    atomicOr(&w32[d + 1], (uint32_t)(lo >> 32));
    atomicOr(&w32[d + 2], hi);
    q += n;
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
    if (n < 4) v &= (1u << (8 * n)) - 1;
    const uint32_t d = q >> 2, sh = 8 * (q & 3);
    const uint64_t x = (uint64_t)v << sh;
    atomicOr(&w32[d], (uint32_t)x);
    atomicOr(&w32[d + 1], (uint32_t)(x >> 32));
    q += n;
  }
  __device__ __forceinline__ void finish() {}
};
// (Round 5, measured on configs 3 / 4 and dropped: an 8-byte accumulating
// sink — whole aligned words stored with ds_write_b64, only the record's two
// edge words OR-ed — 2.61 -> 2.70 ms / neutral; skipping the ORs of dwords a
// value does not reach, and 64-bit ORs on 8-byte words: neutral, 2.59 ->
// 2.60 / 2.58 ms. The write pass is not bound by its LDS atomics.)
struct ByteSink {
  uint8_t* base;
  uint32_t q;
  __device__ __forceinline__ ByteSink(uint8_t* b) : base(b), q(0) {}
  __device__ __forceinline__ void put64(uint64_t v, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) base[q + i] = (uint8_t)(v >> (8 * i));
    q += n;
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) { put64(v, n); }
  __device__ __forceinline__ void finish() {}
};

template <class Sink>
__device__ __forceinline__ void put8(Sink& s, uint64_t v, uint32_t n) {
  s.put64(v, n);
}
// big-endian n-byte value (BinaryProtocol-inl.h:120-161 writeBE)
template <class Sink>
__device__ __forceinline__ void put_be(Sink& s, uint64_t v, uint32_t n) {
  s.put64(__builtin_bswap64(v) >> (64 - 8 * n), n);
}
// LEB128 (VarintUtils-inl.h:545-620): the first 8 bytes of the encoding are
// the 7-bit groups spread into bytes plus continuation bits, no loop
template <class Sink>
__device__ __forceinline__ void put_varint(Sink& s, uint64_t v) {
  const uint32_t len = varint_len(v);
  uint64_t x = v & 0x00ffffffffffffffull;
  x = (x & 0x000000000fffffffull) | ((x & 0x00fffffff0000000ull) << 4);
  x = (x & 0x00003fff00003fffull) | ((x & 0x0fffc0000fffc000ull) << 2);
  x = (x & 0x007f007f007f007full) | ((x & 0x3f803f803f803f80ull) << 1);
  if (len <= 8) {
    x |= 0x8080808080808080ull & ((1ull << (8 * (len - 1))) - 1);
    s.put64(x, len);
  } else {
    s.put64(x | 0x8080808080808080ull, 8);
    const uint32_t b8 = (uint32_t)((v >> 56) & 0x7f), b9 = (uint32_t)(v >> 63);
    s.put(len == 10 ? (b8 | 0x80u | (b9 << 8)) : b8, len - 8);
  }
}
// len bytes from HBM (any alignment): aligned dword loads, issued 8 at a
// time before any is used (one memory round trip per 32 bytes, not per dword)
// The first batch of a string's dwords, loaded ahead (compiled programs
// issue every string's first batch before emitting anything, so the lanes'
// string loads overlap instead of each waiting behind the previous ops).
struct StrPrefetch {
  uint32_t v[8];
};
// String payloads as 16-byte vectors of the 16-byte-aligned blocks the string
// touches (a whole aligned block never reaches a page the string does not),
// two per batch, shifted into place in registers: 2 loads per 32 bytes where
// the dword form issues 8. Round 5, config 3 encode 2.61 -> 2.49 ms (the
// payload loads cost 0.49 ms of it, A/B TGPU_NO_STR_LOAD;
// profiles/r05/ab/str_x4_ab.log). TGPU_STR_X4=0 keeps the dword form (A/B).
// for_elems reads 4- and 8-byte list elements the same way (TGPU_ELEM_X4).
#ifndef TGPU_STR_X4
#define TGPU_STR_X4 1
#endif
typedef uint32_t StrVec __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void str_load32(uint32_t (&v)[8], const uint8_t* __restrict__ blk,
                                           uint32_t nvec) {
  StrVec a = {0u, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
  if (nvec > 0) a = ((const StrVec*)blk)[0];
  if (nvec > 1) b = ((const StrVec*)blk)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
// v (a block's 8 dwords) -> the dwords of the bytes from `off` (0..15) on
__device__ __forceinline__ void str_shift(uint32_t (&v)[8], uint32_t off) {
  const bool d2 = (off & 8) != 0, d1 = (off & 4) != 0;
  const uint32_t by = off & 3;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) v[i] = d2 ? (i + 2 < 8 ? v[i + 2] : 0u) : v[i];
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) v[i] = d1 ? (i + 1 < 8 ? v[i + 1] : 0u) : v[i];
#pragma unroll
  for (uint32_t i = 0; i < 7; ++i) v[i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], by);
  v[7] = v[7] >> (8 * by);
}

__device__ __forceinline__ void str_prefetch(StrPrefetch& f, const uint8_t* __restrict__ src,
                                             uint32_t len) {
#if TGPU_STR_X4
  {
    const uint32_t off = (uint32_t)((uintptr_t)src & 15);
    const uint32_t nv = (off + len + 15) >> 4;
    str_load32(f.v, src - off, len ? (nv < 2 ? nv : 2) : 0);
    return;
  }
#endif
  const uint32_t sh = (uint32_t)((uintptr_t)src & 3);
  const uint32_t* w = (const uint32_t*)(src - sh);
  const uint32_t need = (sh + len + 3) >> 2;
#pragma unroll
#ifndef TGPU_NO_STR_LOAD  // (A/B only, as in put_bytes)
  for (uint32_t i = 0; i < 8; ++i) f.v[i] = i < need ? w[i] : 0u;
#else
  for (uint32_t i = 0; i < 8; ++i) f.v[i] = i < need ? i : 0u;
#endif
}

template <class Sink>
__device__ __forceinline__ void put_bytes(Sink& s, const uint8_t* __restrict__ src, uint32_t len,
                                          const StrPrefetch* pf = nullptr) {
  if (!len) return;
#if TGPU_STR_X4
  {
    uint32_t off = (uint32_t)((uintptr_t)src & 15);
    const uint8_t* blk = src - off;
    uint32_t left = len;
    bool first = true;
    while (left) {
      const uint32_t nv = (off + left + 15) >> 4;
      uint32_t v[8];
      if (pf && first) {
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) v[i] = pf->v[i];
      } else {
        str_load32(v, blk, nv < 2 ? nv : 2);
      }
      first = false;
      str_shift(v, off);
      const uint32_t room = 32 - off;
      const uint32_t take = left < room ? left : room;
#pragma unroll
      for (uint32_t i = 0; i < 8; ++i)
        if (4 * i < take) s.put(v[i], take - 4 * i < 4 ? take - 4 * i : 4);
      left -= take;
      blk += 32;
      off = 0;
    }
    return;
  }
#endif
  // (the aligned base by pointer arithmetic on src, not an integer cast: the
  // loads keep src's address space — global_load, not flat_load)
  uint32_t sh = (uint32_t)((uintptr_t)src & 3);
  const uint32_t* w = (const uint32_t*)(src - sh);
  uint32_t left = len;
  bool first = true;
  while (left) {
    const uint32_t need = (sh + left + 3) >> 2;  // dwords still to read
    uint32_t v[8];
    if (pf && first) {
#pragma unroll
      for (uint32_t i = 0; i < 8; ++i) v[i] = pf->v[i];
    } else {
#pragma unroll
#ifndef TGPU_NO_STR_LOAD  // A/B only (tools/kbench_jit.py --no-check): cost of the loads
      for (uint32_t i = 0; i < 8; ++i) v[i] = i < need ? w[i] : 0u;
#else
      for (uint32_t i = 0; i < 8; ++i) v[i] = i;
#endif
    }
    first = false;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
      if (i < need) {
        const uint32_t take = 4 - sh < left ? 4 - sh : left;
        s.put(v[i] >> (8 * sh), take);
        left -= take;
        sh = 0;
      }
    }
    w += 8;
  }
}

// String ops whose first batch is loaded before any emission (A/B knob, off:
// measured slower on config 3 — 5.62 ms with 4, 4.84 ms with 1, vs 3.81 ms —
// the held batches cost registers/occupancy; strings' loads themselves cost
// 0.86 ms of the encode, A/B TGPU_NO_STR_LOAD).
#ifndef TGPU_STR_PREFETCH
#define TGPU_STR_PREFETCH 0
#endif
// The first batch (8 dwords) of every string op's payload, up to kN strings,
// loaded ahead of the emission (the compiled write pass issues them before
// its block scan, so their latency overlaps the scan).
template <uint32_t kN>
struct StrAhead {
  StrPrefetch f[kN > 0 ? kN : 1];
  uint32_t n = 0;
};
template <uint32_t kN, class PP, class R>
__device__ __forceinline__ void str_ahead(const PP& P, const R& rec,
                                          const uint8_t* __restrict__ sbase, StrAhead<kN>& ah) {
  if constexpr (kN > 0) {
    all_ops(P, [&](const VOp op) {
      if (op.kind == VOP_STRING && ah.n < kN) {
        const tgpu_span sp = rec.span(op.member);
        str_prefetch(ah.f[ah.n], sbase + sp.offset, sp.length);
        ++ah.n;
      }
      return true;
    });
  }
}

template <class PP, class Sink, class R, uint32_t kA = 0>
__device__ __forceinline__ void program_emit(const PP& P, const R& rec,
                                             const uint8_t* __restrict__ sbase,
                                             const uint8_t* __restrict__ lbase, Sink& s,
                                             const StrAhead<kA>* ahead = nullptr) {
  const bool compact = P.protocol() == TGPU_PROTOCOL_COMPACT;
  constexpr uint32_t kPf = PP::kStatic && kA == 0 ? TGPU_STR_PREFETCH : 0;
  StrAhead<kPf> own;
  str_ahead(P, rec, sbase, own);
  uint32_t ipf = 0;
  all_ops(P, [&](const VOp op) {
    switch (op.kind) {
      case VOP_CONST:
        put8(s, op.hdr, op.hdr_len);
        break;
      case VOP_CBOOL:
        // the bool's value rides in the header's type nibble (CT_BOOLEAN_TRUE/FALSE)
        put8(s, op.hdr | (rec.u8(op.member) ? 1u : 2u), op.hdr_len);
        break;
      case VOP_FIXED:
        if (op.bits == kFixedLE) put8(s, rec.member(op.member, op.width), op.width);
        else put_be(s, rec.member(op.member, op.width), op.width);
        break;
      case VOP_VARINT:
        put_varint(s, zz_member(rec.member(op.member, op.width), op.width, op.bits));
        break;
      case VOP_STRING: {
        const tgpu_span sp = rec.span(op.member);
        if (compact) put_varint(s, sp.length);
        else put_be(s, sp.length, 4);
        // (no pointer chosen at run time between a prefetched batch and
        // none: that kept the batches in scratch)
        const uint32_t k = ipf++;
        if constexpr (kA > 0) {
          if (k < kA) {
            put_bytes(s, sbase + sp.offset, sp.length, &ahead->f[k < kA ? k : 0]);
            break;
          }
        } else if constexpr (kPf > 0) {
          if (k < kPf) {
            put_bytes(s, sbase + sp.offset, sp.length, &own.f[k < kPf ? k : 0]);
            break;
          }
        }
        put_bytes(s, sbase + sp.offset, sp.length);
        break;
      }
      case VOP_LIST: {
        const tgpu_span sp = rec.span(op.member);
        const uint32_t len = sp.length;
        if (compact) {
          if (len <= 14) {
            s.put((len << 4) | op.elem_ct, 1);
          } else {
            s.put(0xf0 | op.elem_ct, 1);
            put_varint(s, len);
          }
        } else {
          s.put(op.elem_ttype, 1);
          put_be(s, len, 4);
        }
        const uint8_t* e = lbase + sp.offset;
        if (op.elem_kind == VEL_VARINT) {
          for_elems(e, len, op.width, [&](uint64_t x) {
            put_varint(s, zz_member(x, op.width, op.bits));
          });
        } else if (op.elem_kind == VEL_BOOL) {
          for_elems(e, len, 1, [&](uint64_t x) { s.put(compact ? (x ? 1u : 2u) : (uint32_t)x, 1); });
        } else {
          if (op.bits == kFixedLE)
            for_elems(e, len, op.width, [&](uint64_t x) { put8(s, x, op.width); });
          else
            for_elems(e, len, op.width, [&](uint64_t x) { put_be(s, x, op.width); });
        }
        break;
      }
      default:
        break;
    }
    return true;
  });
  s.finish();
}

// A record past the tile's LDS output cap goes straight to HBM, a byte at a
// time (rare; out of line so the common path stays small).
#ifdef TGPU_INLINE_HBM_EMIT
#define TGPU_HBM_EMIT_ATTR __forceinline__
#else
#define TGPU_HBM_EMIT_ATTR __attribute__((noinline))
#endif
template <class PP>
__device__ TGPU_HBM_EMIT_ATTR void emit_to_hbm(const PP P, const uint8_t* rec,
                                                      const uint8_t* __restrict__ sbase,
                                                      const uint8_t* __restrict__ lbase,
                                                      uint8_t* dst) {
  ByteSink b(dst);
  program_emit(P, PtrRec{rec}, sbase, lbase, b);
}

// Records [r0, r0+nrec) of stride S into LDS; returns the 16-byte phase.
// The LDS region is enc_record_region(S) bytes (kept tight: 4 workgroups of
// record + output tiles must fit a CU's 160 KiB).
__host__ __device__ __forceinline__ uint32_t enc_record_region(uint32_t S) {
  return (kET * S + 16 + 15) & ~15u;
}
__device__ __forceinline__ uint32_t stage_records(const uint8_t* recs, uint64_t r0, uint32_t nrec,
                                                  uint32_t S, uint8_t* rtile) {
  const uint8_t* g = recs + r0 * S;
  const uint32_t sh = (uint32_t)((uintptr_t)g & 15);
  const uint4* src = (const uint4*)(g - sh);
  const uint32_t nvec = (nrec * S + sh + 15) >> 4;
  for (uint32_t i = threadIdx.x; i < nvec; i += kET) ((uint4*)rtile)[i] = src[i];
  return sh;
}

// Pass 1: record tile HBM -> LDS; each lane sizes its record; sizes ->
// a.offs[i]; tile sum -> block_sums[t]; validation failures -> first_fail.
template <class PP>
__device__ __forceinline__ void size_tile(const EncodeArgs& a, const PP& P, uint32_t S,
                                          uint8_t* smem, unsigned long long* part) {
  const uint64_t r0 = (uint64_t)blockIdx.x * kET;
  const uint32_t nrec = (uint32_t)min((uint64_t)kET, a.n - r0);
  const uint8_t* recs = smem;
  const uint32_t sh = stage_records(a.recs, r0, nrec, S, smem);
  __syncthreads();
  unsigned long long sz = 0;
  if (threadIdx.x < nrec) {
    bool ok = true;
    sz = program_size(P, PtrRec{recs + sh + threadIdx.x * S}, a.lbase, ok);
    if (!ok) atomicMin(&a.res->first_fail, (unsigned long long)(r0 + threadIdx.x));
    // (a.recompute: the write pass sizes its records itself; tile sums only)
    if (!a.recompute) a.offs[r0 + threadIdx.x] = sz;
  }
  unsigned long long total;
  (void)block_exscan256(sz, part, &total);
  if (threadIdx.x == 0) a.block_sums[blockIdx.x] = total;
}

// Pass 3 of the encode: the record tile goes HBM -> LDS again, the sizes of
// pass 1 (a.offs) are scanned inside the block and offset by the tile's
// stream offset (a.block_sums after the tile scan); every lane emits its
// record into the zero-filled LDS output tile a dword at a time (records past
// the LDS cap go to HBM directly); the tile leaves with coalesced 16-byte
// stores (byte stores only on the two edge chunks shared with the
// neighbouring tiles). a.offs receives every record's start.
// (A single-pass variant with decoupled look-back was measured slower here:
// its ticket counter alone — one atomic per tile on one address — cost
// 1.5 ms on 256 Ki tiles, and the look-back wait another 1.4 ms.)
struct EncodeShared {
  unsigned long long part[4];
  unsigned int lds_end;
  unsigned long long elo, ehi;  // the tile's list elements in list_base
  unsigned long long base;      // single-pass transcoder: the tile's output start
};

// Encode, compiled programs: the tile's list elements are staged in LDS with
// coalesced 16-byte loads when their extent in list_base fits kElemStage
// bytes (each lane's own 4-byte element loads cost 1.0 of config 4's 2.5 ms).
#ifndef TGPU_ELEM_STAGE
#define TGPU_ELEM_STAGE 0
#endif
constexpr uint32_t kElemStage = TGPU_ELEM_STAGE;

// Strings whose first 32 bytes the compiled write pass loads before its block
// scan (A/B: TGPU_ENC_AHEAD=0 loads them during the emission)
#ifndef TGPU_ENC_AHEAD
#define TGPU_ENC_AHEAD 2
#endif

// SR (compiled programs: the record size as a constant): with a.recompute the
// size pass left tile sums only, and this pass loads its record into
// registers (RegRec), sizes it for the block scan and emits from the same
// registers — the record is read once, and the string loads (issued right
// after it, before the scan) overlap the scan's barriers, where the size
// pass's per-record sizes cost a dependent HBM round trip first.
template <class PP, uint32_t SR = 0>
__device__ __forceinline__ void write_tile(const EncodeArgs& a, const PP& P, uint32_t S,
                                           uint8_t* smem, EncodeShared& sm) {
  const uint64_t r0 = (uint64_t)blockIdx.x * kET;
  const uint32_t nrec = (uint32_t)min((uint64_t)kET, a.n - r0);
  const uint32_t ocap = a.out_cap ? a.out_cap : kOutCap;  // LDS output tile bytes
  // compiled programs read their record's members straight from HBM (the
  // unrolled loads issue together; no LDS record tile, so 6 instead of 4
  // workgroups fit a CU: config 3 encode -9 %, config 4 -21 %); the
  // interpreter's op-by-op loads need the LDS-staged tile
  uint8_t* rtile;
  uint8_t* otile;
  uint32_t rsh;
  if constexpr (PP::kStatic) {
    rtile = (uint8_t*)a.recs + r0 * S;
    otile = smem;
    rsh = 0;
  } else {
    rtile = smem;
    otile = smem + enc_record_region(S);
    rsh = stage_records(a.recs, r0, nrec, S, rtile);
  }
  const uint32_t r = threadIdx.x;
  // (one emission path per kernel: two instantiations of the unrolled
  // emitter left the compiler's unroller short, and the register record then
  // went to scratch)
  constexpr bool kReg = PP::kStatic && SR > 0;
  constexpr uint32_t kAhead = kReg ? TGPU_ENC_AHEAD : 0;
  RegRec<kReg ? SR : 8> R;
  StrAhead<kAhead> ah;
  if constexpr (kReg) {
    if (r < nrec) R.load(a.recs + (r0 + r) * S);
  }
  if (kElemStage > 0 && r == 0) {
    sm.elo = ~0ull;
    sm.ehi = 0;
  }
  unsigned long long sz, tile_total, rel, tile_base;
  if (a.fixed_len) {
    // fixed layout: every record is fixed_len bytes; the size pass only
    // validates (validate_bool -> first_fail)
    sz = r < nrec ? a.fixed_len : 0;
    tile_total = (unsigned long long)nrec * a.fixed_len;
    rel = (unsigned long long)r * a.fixed_len;
    tile_base = r0 * a.fixed_len;
    if (a.offs && r == 0 && r0 + nrec == a.n) a.offs[a.n] = a.n * a.fixed_len;
  } else if (kReg) {
    // (a.recompute, set for every compiled write: the size pass wrote tile
    // sums only)
    tile_base = a.block_sums[blockIdx.x];
    sz = 0;
    if (r < nrec) {
      bool ok = true;  // (the size pass reported validation failures)
      sz = program_size(P, R, a.lbase, ok);
      str_ahead(P, R, a.sbase, ah);
    }
    rel = block_exscan256(sz, sm.part, &tile_total);
  } else {
    sz = r < nrec ? a.offs[r0 + r] : 0;
    rel = block_exscan256(sz, sm.part, &tile_total);
    tile_base = a.block_sums[blockIdx.x];
  }
  uint8_t* gtile = a.out + tile_base;
  const uint32_t osh = (uint32_t)((uintptr_t)gtile & 15);
  const uint8_t* lbase = a.lbase;
  if constexpr (PP::kStatic && kElemStage > 0) {
    if (P.has_lists()) {
      // extent of the tile's elements (block barrier in the exscan above
      // orders thread 0's init before the atomics)
      unsigned long long lo = ~0ull, hi = 0;
      if (r < nrec) {
        const uint8_t* rec = rtile + r * S;
        all_ops(P, [&](const VOp op) {
          if (op.kind == VOP_LIST) {
            const tgpu_span sp = *(const tgpu_span*)(rec + op.member);
            if (sp.length) {
              lo = min(lo, (unsigned long long)sp.offset);
              hi = max(hi, (unsigned long long)sp.offset + (unsigned long long)sp.length * op.width);
            }
          }
          return true;
        });
      }
      if (lo != ~0ull) {
        atomicMin(&sm.elo, lo);
        atomicMax(&sm.ehi, hi);
      }
      __syncthreads();
      const unsigned long long elo = sm.elo, ehi = sm.ehi;
      if (elo < ehi) {
        const uintptr_t g0 = ((uintptr_t)a.lbase + elo) & ~(uintptr_t)15;
        const uint32_t nvec = (uint32_t)(((uintptr_t)a.lbase + ehi - g0 + 15) >> 4);
        if (nvec * 16 <= kElemStage) {
          uint8_t* stage = smem + ocap + 32;
          for (uint32_t i = threadIdx.x; i < nvec; i += kET)
            ((uint4*)stage)[i] = ((const uint4*)g0)[i];
          // a flat (generic) address into the LDS aperture, computed in 64-bit
          // integers so element offsets added later stay inside it
          const uintptr_t sg = (uintptr_t)(void*)stage;
          lbase = (const uint8_t*)(sg - (g0 - (uintptr_t)a.lbase));
        }
      }
    }
  }
  {  // zero the part of the output tile the records will OR into
    const uint4 z = {0u, 0u, 0u, 0u};
    const uint32_t nz =
        (osh + (uint32_t)min(tile_total, (unsigned long long)ocap) + 4 + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nz; i += kET) ((uint4*)otile)[i] = z;
  }
  if (r == 0) sm.lds_end = (unsigned int)min(tile_total, (unsigned long long)ocap);
  __syncthreads();  // record tile staged, output tile zeroed, lds_end initialised
  bool fits = false;
  if (r < nrec) {
    const unsigned long long start = tile_base + rel;
    if (a.offs) a.offs[r0 + r] = start;
    if (start + sz > a.cap) {
      atomicMin(&a.res->first_fail, (unsigned long long)(r0 + r));
      atomicMin(&sm.lds_end, (unsigned int)min(rel, (unsigned long long)ocap));
    } else {
      fits = rel + sz <= ocap;
      if (!fits) atomicMin(&sm.lds_end, (unsigned int)rel);
    }
  }
  __syncthreads();
  if (r < nrec) {
    const uint8_t* rec = rtile + rsh + r * S;
    if (a.fixed_len) {  // the validation the size pass does otherwise (validate_bool)
      bool ok = true;
      if constexpr (kReg) (void)program_size(P, R, a.lbase, ok);
      else (void)program_size(P, PtrRec{rec}, a.lbase, ok);
      if (!ok) atomicMin(&a.res->first_fail, (unsigned long long)(r0 + r));
    }
    if (fits && rel + sz <= sm.lds_end) {
      using Sink = OrSink;
      Sink w((uint32_t*)otile, osh + (uint32_t)rel);
      if constexpr (kReg)
        program_emit<PP, Sink, RegRec<kReg ? SR : 8>, kAhead>(P, R, a.sbase, lbase, w, &ah);
      else
        program_emit(P, PtrRec{rec}, a.sbase, lbase, w);
    } else if (tile_base + rel + sz <= a.cap) {
      emit_to_hbm(P, rec, a.sbase, a.lbase, gtile + rel);
    }
  }
  __syncthreads();
  // LDS tile [osh, osh + lds_end) -> HBM [gtile, gtile + lds_end)
  const uint32_t end = osh + sm.lds_end;
  const uint32_t nvec = (end + 15) >> 4;
  uint8_t* gb = gtile - osh;
  for (uint32_t i = threadIdx.x; i < nvec; i += kET) {
    const uint32_t lo = i << 4, hi = lo + 16;
    if (lo >= osh && hi <= end) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(((const u32x4*)otile)[i], (u32x4*)gb + i);
    } else {
      for (uint32_t b = (lo < osh ? osh : lo); b < (hi < end ? hi : end); ++b) gb[b] = otile[b];
    }
  }
}

// ================================================================= index ======
// A chunk is a tile of kTile bytes handled by one workgroup: the tile (plus
// kOver bytes for the records that straddle its end) is staged in LDS with
// coalesced 16-byte loads; lane k speculates the first record start in its
// kSub-byte slice and chains to the slice's end; the lanes' links are then
// repaired inside the workgroup (lane k restarts from lane k-1's end until
// no lane changes), so the tile behaves like one chunk of the lane path:
// (first start, end, count). A tile any lane could not finish with the
// program is handed to the general-reader kernels whole (kPartial).
constexpr uint64_t kNo = ~0ull;             // no start found / unset
constexpr uint64_t kErr = ~0ull - 1;        // chain ended in a reader error
constexpr uint64_t kPartial = ~0ull - 2;    // program stopped: general reader continues
constexpr uint64_t kLanesValid = ~0ull - 3; // pf: the tile's per-lane results are current
constexpr uint64_t kStartsValid = ~0ull - 4; // pf: ... and its record starts are in st16
constexpr uint32_t kPosCap = 0x7fffff00u;
constexpr uint32_t kTileLanes = 256;
// bytes per lane slice: the tile is kTileLanes * kSub bytes (A/B builds:
// -DTGPU_KSUB with the same TGPU_JIT_DEFINES for the schema kernels)
#ifndef TGPU_KSUB
#define TGPU_KSUB 64
#endif
constexpr uint32_t kSub = TGPU_KSUB;
constexpr uint32_t kTile = kTileLanes * kSub;
#ifndef TGPU_KOVER
#define TGPU_KOVER 512
#endif
constexpr uint32_t kOver = TGPU_KOVER;
constexpr uint32_t kTileLds = kTile + kOver + 32;
constexpr uint32_t kNoPos = 0xffffffffu;

__device__ __forceinline__ uint64_t chunk_lo(const IndexArgs& a, uint64_t j) {
  return a.begin + j * a.chunk;
}
__device__ __forceinline__ uint64_t chunk_hi(const IndexArgs& a, uint64_t j) {
  const uint64_t h = a.begin + (j + 1) * a.chunk;
  return h < a.end ? h : a.end;
}

// LDS window with HBM fallback past the staged bytes (positions relative to
// the 16-byte aligned tile base)
// (the HBM path is rare — records straddling the staged bytes — and kept out
// of line: inlined at every window of an unrolled program it multiplies the
// schema compiler's code size and compile time)
// (out-of-line helpers take plain scalars: a struct passed by value to a
// call goes through scratch, stored by every lane of every tile)
__device__ __attribute__((noinline)) uint64_t hbm_win8(const uint8_t* base, uint32_t avail,
                                                       uint32_t p) {
  return HbmSrc{base, avail}.win8(p);
}
struct TileSrc {
  const uint32_t* w32;
  uint32_t lds_len;
  HbmSrc g;
  __device__ __forceinline__ uint64_t win8(uint32_t p) const {
    if (p + 12 <= lds_len) return LdsSrc{w32}.win8(p);
    return hbm_win8(g.base, g.avail, p);
  }
};

constexpr uint32_t kLaneStarts = 8;  // record starts a lane keeps (u16 pairs in st[])
struct TileLane {
  uint32_t s, e, c;  // first start, end, count (tile-relative); s == kNoPos: none
  bool stuck;
  uint32_t st[kLaneStarts / 2];  // the chain's record starts, u16 each (first kLaneStarts)
};

// start k of the lane's chain := p (register selects: no dynamic indexing)
__device__ __forceinline__ void put_start(TileLane& L, uint32_t k, uint32_t p) {
  const uint32_t sh = (k & 1) * 16, m = 0xffffu << sh, x = (p & 0xffffu) << sh;
#pragma unroll
  for (uint32_t w = 0; w < kLaneStarts / 2; ++w) L.st[w] = (k >> 1) == w ? (L.st[w] & ~m) | x : L.st[w];
}
__device__ __forceinline__ uint32_t get_start(const TileLane& L, uint32_t k) {
  uint32_t v = 0;
#pragma unroll
  for (uint32_t w = 0; w < kLaneStarts / 2; ++w) v = (k >> 1) == w ? L.st[w] : v;
  return (v >> ((k & 1) * 16)) & 0xffffu;
}

// Cheap rejection of a candidate start before running the program: the byte
// after the first header's value must be the second header (first ops
// CONST, VARINT|FIXED, CONST — every schema whose first two fields are
// unqualified scalars). Never rejects a canonical record start.
template <class PP>
__device__ __forceinline__ bool quick_reject(const PP& P, const TileSrc& src, uint32_t cand) {
  if (P.n_ops() < 3) return false;
  const VOp o0 = P.op(0), v = P.op(1), o2 = P.op(2);
  if (o0.kind != VOP_CONST || o2.kind != VOP_CONST) return false;
  const uint64_t w = src.win8(cand + o0.hdr_len);
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
  return ((w >> (8 * len)) & 0xff) != (o2.hdr & 0xff);
}

// run_program<false> over the tile source, out of line: the rare records the
// branch-free walk leaves undecided (see measure_lds)
// (returns ok << 32 | the end: a position passed by address would live in
// scratch, stored on every walk of the hot path)
template <class PP>
__device__ __attribute__((noinline)) uint64_t tile_walk_slow(const PP P, const uint32_t* w32,
                                                             uint32_t lds_len, const uint8_t* gb,
                                                             uint32_t avail, int32_t string_limit,
                                                             int32_t container_limit, uint32_t pos,
                                                             uint32_t end) {
  const TileSrc src{w32, lds_len, HbmSrc{gb, avail}};
  const Ctx pc{0, nullptr, 0, string_limit, container_limit};
  uint32_t q = pos;
  const bool ok = run_program<false>(P, src, pc, q, end, nullptr);
  return ((uint64_t)ok << 32) | q;
}

// One record's measuring walk at q (tile-relative): branch-free over the
// staged bytes, run_program for what that leaves undecided.
template <class PP>
__device__ __forceinline__ bool tile_walk(const PP& P, const TileSrc& src, const Ctx& pc,
                                          uint32_t& q, uint32_t end) {
#ifdef TGPU_BRANCHY_WALK  // A/B: the early-return program walk
  return run_program<false>(P, src, pc, q, end, nullptr);
#else
  bool slow = src.lds_len < 12;
  bool ok = false;
  if (!slow) ok = measure_lds(P, src.w32, src.lds_len - 12, pc, q, end, slow);
  if (slow) {
    const uint64_t r = tile_walk_slow(P, src.w32, src.lds_len, src.g.base, src.g.avail,
                                      pc.string_limit, pc.container_limit, q, end);
    q = (uint32_t)r;
    ok = (r >> 32) != 0;
  }
  return ok;
#endif
}

// The tile's nvec 16-byte vectors HBM -> LDS. Whole waves of vectors go by
// LDS DMA (global_load_lds_dwordx4: no register round trip); the last
// partial wave's vectors through registers. A DMA issued by a partially
// masked wave corrupted the tile now and then (speculated chains broke at
// random tiles, 200-600 of 217k per config-5 call, none under the profiler;
// decode_tile's DMA covers whole waves too). The caller's __syncthreads
// waits for the loads.
#ifdef TGPU_STAGE_BARRIER
#define TGPU_STAGE_SYNC() ((void)0)
#else
#define TGPU_STAGE_SYNC() __syncthreads()
#endif
__device__ __forceinline__ void stage_tile(uint8_t* lds, const uint8_t* gb, uint32_t nvec) {
#ifdef TGPU_SPEC_REGSTAGE  // A/B: staging through registers
  for (uint32_t i = threadIdx.x; i < nvec; i += kTileLanes)
    ((uint4*)lds)[i] = ((const uint4*)gb)[i];
#else
  const uint32_t whole = nvec & ~63u;  // vectors in whole waves
  const uint32_t wave = threadIdx.x >> 6;
  for (uint32_t k = 0; k * kTileLanes < whole; ++k) {
    const uint32_t w0 = k * kTileLanes + wave * 64;  // this wave's first vector (uniform)
    if (w0 < whole)
      __builtin_amdgcn_global_load_lds(
          (const void*)((const uint4*)gb + w0 + (threadIdx.x & 63)),
          (__attribute__((address_space(3))) void*)(lds + (size_t)w0 * 16), 16, 0, 0);
  }
  const uint32_t i = whole + threadIdx.x;
  if (i < nvec) ((uint4*)lds)[i] = ((const uint4*)gb)[i];
#if defined(TGPU_STAGE_BARRIER)  // diagnostics: the staging's wait and
  // barrier exactly as given, in place of the settle and the caller's barrier
  asm volatile(TGPU_STAGE_BARRIER ::: "memory");
#elif !defined(TGPU_NO_DMA_SETTLE)  // A/B: (see lds_dma_settle)
  {
    const uint32_t w0 = wave * 64 + (threadIdx.x & 63);  // this lane's first DMA'd vector
    lds_dma_settle(lds, w0, kTileLanes, w0 < whole ? (whole - 1 - w0) / kTileLanes + 1 : 0);
  }
#endif
#endif
}

// Candidate starts of the tile, one bit per byte (cmask; tile-relative
// positions, 8 per byte), computed cooperatively: thread t owns 8-byte groups
// t, t + 256, ... (consecutive threads read consecutive LDS words: no bank
// conflicts, where one slice per lane read words 16 apart — 32-way
// conflicts). A candidate is a byte equal to the program's first header byte
// (h0) preceded by its STOP byte: every record ends with STOP, so every record
// start but the range's first is preceded by it (a necessary condition: it
// only prunes; for the mixed schema, whose four int headers all equal h0, it
// removes ~3 of 4). The caller's barrier publishes cmask.
template <class PP>
__device__ __forceinline__ void cand_mask(const PP& P, const TileSrc& src, const uint8_t* lds,
                                          uint64_t j, uint32_t sh, uint32_t thi, uint8_t* cmask) {
  const VOp o0 = P.op(0);
  const uint32_t h0 = o0.kind == VOP_CONST ? (o0.hdr & 0xff) : 0x100;
  const VOp ol = P.op(P.n_ops() - 1);
  const uint32_t stop =
      (ol.kind == VOP_CONST && ol.hdr_len) ? ((ol.hdr >> (8 * (ol.hdr_len - 1))) & 0xff) : 0x100;
  const uint32_t ngroups = (thi + 7) >> 3;
  for (uint32_t g = threadIdx.x; g < ngroups; g += kTileLanes) {
    const uint32_t base = g << 3;
    uint64_t m = 0x8080808080808080ull;
    // the group's 8 bytes (8-byte aligned: one LDS read) and the byte
    // before them (one more), where staged; HBM windows past that
    const bool in_lds = base + 8 <= src.lds_len;
    const uint64_t w = in_lds ? *(const uint64_t*)(lds + base) : src.win8(base);
    if (h0 < 0x100) {
      const uint64_t x = w ^ (h0 * 0x0101010101010101ull);
      m = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
    }
    if (stop < 0x100) {
      // byte i of y = the byte before position base + i
      const uint64_t prev = !base ? (w << 8)
                            : in_lds ? (w << 8) | lds[base - 1]
                                     : src.win8(base - 1);
      const uint64_t y = prev ^ (stop * 0x0101010101010101ull);
      uint64_t z = (y - 0x0101010101010101ull) & ~y & 0x8080808080808080ull;
      if (!base) z |= 0x80ull;  // position 0: predecessor not staged
      // the range's first byte has no predecessor inside the range
      if (j == 0 && sh >= base && sh < base + 8) z |= 0x80ull << (8 * (sh - base));
      m &= z;
    }
    cmask[g] = (uint8_t)((((m >> 7) & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
  }
  for (uint32_t g = ngroups + threadIdx.x; g < ngroups + 9; g += kTileLanes) cmask[g] = 0;
}

// chain of canonical records from x while position < hi (tile-relative)
template <class PP>
__device__ __forceinline__ void tile_chain(const PP& P, const TileSrc& src, const Ctx& pc,
                                           uint32_t x, uint32_t hi, uint32_t end, TileLane& L) {
  L.s = x;
  L.c = 0;
  L.stuck = false;
  uint32_t p = x;
  while (p < hi) {
    uint32_t q = p;
    if (!tile_walk(P, src, pc, q, end)) {
      L.stuck = true;
      break;
    }
    put_start(L, L.c, p);
    ++L.c;
    p = q;
  }
  L.e = p;
}

// Stages the tile, speculates and repairs the lanes' chains. entry: the
// tile's known first start (tile-relative; kNoPos: speculate lane 0 too).
// Returns false when the tile needs the general reader. *first: the tile's
// first record start (kNoPos: none).
template <class PP>
__device__ __forceinline__ bool tile_resolve(const IndexArgs& a, const PP& P, uint64_t j,
                                             uint8_t* lds, uint32_t entry, TileLane& L,
                                             uint32_t& sh, uint32_t& first, uint32_t* E, int* flag,
                                             uint32_t* first_lane, uint32_t* fs_p, uint8_t* cmask) {
  const uint64_t lo = chunk_lo(a, j);
  const uint64_t hi_abs = chunk_hi(a, j);
  const uint8_t* g = a.in + lo;
  sh = (uint32_t)((uintptr_t)g & 15);
  const uint8_t* gb = g - sh;
  const uint64_t avail64 = a.in_len - lo + sh;
  const uint32_t avail = (uint32_t)(avail64 < kPosCap ? avail64 : kPosCap);
  const uint32_t staged = avail < kTile + kOver + 16 ? avail : kTile + kOver + 16;
  const uint32_t nvec = (staged + 15) >> 4;
  stage_tile(lds, gb, nvec);
  TGPU_STAGE_SYNC();
#ifdef TGPU_SPEC_LATE
  uint32_t late0 = 0;
  for (uint32_t d = threadIdx.x; d < ((staged & ~3u) >> 2); d += kTileLanes)
    late0 ^= ((const volatile uint32_t*)lds)[d] * (d | 1);
#endif
  const TileSrc src{(const uint32_t*)lds, staged & ~3u, HbmSrc{gb, avail}};
  const Ctx pc{0, nullptr, 0, a.string_limit, a.container_limit};
  const uint32_t thi = sh + (uint32_t)(hi_abs - lo);  // tile end (relative)
  const uint32_t k = threadIdx.x;
  const uint32_t sub_lo = sh + k * kSub;
  const uint32_t sub_hi = sub_lo + kSub < thi ? sub_lo + kSub : thi;
  // candidate starts of the whole tile (see cand_mask)
  cand_mask(P, src, lds, j, sh, thi, cmask);
  if (threadIdx.x == 0) *first_lane = ~0u;  // (the first-start minimum below)
  __syncthreads();
  L.s = kNoPos;
  L.e = kNoPos;
  L.c = 0;
  L.stuck = false;
  if (k == 0 && entry != kNoPos) {
    tile_chain(P, src, pc, entry, sub_hi > entry ? sub_hi : entry, avail, L);
    if (entry >= sub_hi) {  // the entry lies past lane 0's slice
      L.s = entry;
      L.e = entry;
    }
  } else if (sub_lo < thi) {
    // this lane's slice [sub_lo, sub_hi) as 64 candidate bits (cmask);
    // candidates that survive quick_reject are chained in order (divergent
    // but cheap); the chain runs outside the search so all lanes of the
    // wave run it together
    // (the slice's 64 bits from the 8-byte aligned words around them)
    // (64 positions at a time: a slice of kSub > 64 bytes takes several)
    const uint64_t* cw = (const uint64_t*)cmask;
    bool need = true;
    for (uint32_t b0 = sub_lo; b0 < sub_hi && need; b0 += 64) {
      const uint32_t g0 = b0 >> 3, off = b0 & 7;
      const uint32_t d = g0 >> 3, bo = (g0 & 7) * 8 + off;  // bit offset in word d
      const uint64_t c0 = cw[d], c1 = cw[d + 1];
      uint64_t cm = bo ? (c0 >> bo) | (c1 << (64 - bo)) : c0;
      if (sub_hi - b0 < 64) cm &= (1ull << (sub_hi - b0)) - 1;
      while (need) {
        uint32_t cand = kNoPos;
        while (cm) {
          const uint32_t c = b0 + (uint32_t)__builtin_ctzll(cm);
          cm &= cm - 1;
#ifndef TGPU_NO_QUICK_REJECT  // A/B: the measuring walk alone rejects false candidates
          if (quick_reject(P, src, c)) continue;
#endif
          cand = c;
          break;
        }
        if (cand == kNoPos) break;  // no record start in these 64 positions
        TileLane t;
        tile_chain(P, src, pc, cand, sub_hi, avail, t);
        if (t.c) {
          L = t;
          need = false;
        }
      }
    }
  }
  // the tile's first start: the first lane that found one, and its start,
  // in one packed minimum (lane << 16 | start: starts are below 64 Ki;
  // *first_lane was reset before the candidate-mask barrier)
  if (L.s != kNoPos) atomicMin(first_lane, (k << 16) | (L.s < 0xffffu ? L.s : 0xffffu));
  __syncthreads();
  const uint32_t fv = *first_lane;
  if (fv == ~0u) {
    first = kNoPos;
    return true;
  }
  const uint32_t f = fv >> 16;
  uint32_t fs = fv & 0xffffu;
  if (fs == 0xffffu) {  // (a start 64 Ki or more into the tile: an entry past a long record)
    if (k == f) *fs_p = L.s;
    __syncthreads();
    fs = *fs_p;
  }
  // lanes before it: no record starts there
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
          tile_chain(P, src, pc, x, sub_hi, avail, L);
        }
        changed = 1;
      }
    }
    if (!__syncthreads_or(changed)) break;
  }
  (void)flag;
#ifdef TGPU_SPEC_LATE
  {
    uint32_t late1 = 0;
    for (uint32_t d = threadIdx.x; d < ((staged & ~3u) >> 2); d += kTileLanes)
      late1 ^= ((const volatile uint32_t*)lds)[d] * (d | 1);
    if (late1 != late0) atomicAdd(&a.scal[12], 1ull);
  }
#endif
  return !__syncthreads_or(L.stuck || L.e == kNoPos);
}

// The candidate-list speculation (spec_tile_cands): at most kCandCap
// candidates per tile (more, and the tile takes the slice speculation).
#ifndef TGPU_CAND_CAP
#define TGPU_CAND_CAP 768
#endif
constexpr uint32_t kCandCap = TGPU_CAND_CAP;
constexpr uint32_t kCandWords = kTile / 64 + 2;  // 64-position words of cmask
// (thread t counts word t; the last thread the words past 256, whose counts
// are packed 8 bits each into one 64-bit word: at most 8 of them)
static_assert(kCandWords <= kTileLanes + 8, "TGPU_KSUB > 64 needs a wider word-count packing");
struct CandLists {
  uint16_t cand[kCandCap + 2];  // candidate positions in order (+ a sentinel)
  uint16_t len[kCandCap];       // record length walked from each (0: not a record)
  uint16_t wbase[kCandWords];   // index of the first candidate of each cmask word
};

struct IndexTileShared {
  alignas(8) uint8_t cmask[kTile / 8 + 16];  // candidate bits of the tile (one per byte)
  union {
    uint32_t E[kTileLanes];  // slice speculation: the lanes' chain ends
    CandLists cl;            // candidate-list speculation
  };
  int flag;
  uint32_t first_lane, fs;
  unsigned long long csum;
  unsigned long long part[4];
};

// Tile speculation over the list of candidate starts (the common case; the
// slice speculation of tile_resolve is the fallback for tiles with more than
// kCandCap candidates). Every candidate is walked once, by its own lane
// (record i of the list on lane i mod 256: balanced, where a lane owning a
// 64-byte slice walked all its records in turn and the wave waited for the
// lane with the most); the walk gives each candidate's record length. The
// tile's first start is the first candidate that is a canonical record (as
// in the slice speculation), and its chain follows the lengths: a record
// whose end is the next candidate links to it, which wave 0 checks 64
// candidates per step (one ballot), hopping over the rare false candidates
// (a STOP byte followed by h0 inside a record) by the rank of the end in
// the candidate bits. The chain's starts are stored (u16, st16) as it goes.
// Writes the tile's (s, e, cnt, pf) like index_spec_tile; returns false,
// with nothing written, when the tile has too many candidates.
// kOnePass (index_onepass_rr_tile): the chain's starts go to `sdst` (LDS)
// and its result to *res; every wave stays (the caller's barrier follows).
struct CandResult {
  uint32_t first, e, count, stuck;  // tile-relative; first kNoPos: none
  uint32_t sh, staged, avail, thi;
};
template <class PP, bool kOnePass = false>
__device__ __forceinline__ bool spec_tile_cands(const IndexArgs& a, const PP& P, uint64_t j,
                                                uint8_t* lds, uint32_t ent,
                                                IndexTileShared& sm, uint16_t* sdst = nullptr,
                                                CandResult* res = nullptr) {
  const uint64_t lo = chunk_lo(a, j);
  const uint64_t hi_abs = chunk_hi(a, j);
  const uint8_t* g = a.in + lo;
  const uint32_t sh = (uint32_t)((uintptr_t)g & 15);
  const uint8_t* gb = g - sh;
  const uint64_t avail64 = a.in_len - lo + sh;
  const uint32_t avail = (uint32_t)(avail64 < kPosCap ? avail64 : kPosCap);
  const uint32_t staged = avail < kTile + kOver + 16 ? avail : kTile + kOver + 16;
  stage_tile(lds, gb, (staged + 15) >> 4);
  TGPU_STAGE_SYNC();
#ifdef TGPU_SPEC_EARLY  // diagnostics: the staged bytes right after the staging barrier
  {
    uint32_t bad = 0;
    for (uint32_t d = threadIdx.x; d < ((staged & ~3u) >> 2); d += kTileLanes)
      bad += ((const uint32_t*)lds)[d] != __builtin_nontemporal_load((const uint32_t*)gb + d);
    if (bad) atomicAdd(&a.scal[12], (unsigned long long)bad);
  }
#endif
#ifdef TGPU_SPEC_LATE  // diagnostics: does the staged tile change after the staging barrier?
  uint32_t late0 = 0;
  for (uint32_t d = threadIdx.x; d < ((staged & ~3u) >> 2); d += kTileLanes)
    late0 ^= ((const volatile uint32_t*)lds)[d] * (d | 1);
#endif
  const TileSrc src{(const uint32_t*)lds, staged & ~3u, HbmSrc{gb, avail}};
  const Ctx pc{0, nullptr, 0, a.string_limit, a.container_limit};
  const uint32_t thi = sh + (uint32_t)(hi_abs - lo);  // tile end (relative)
  cand_mask(P, src, lds, j, sh, thi, sm.cmask);
  if (threadIdx.x == 0) sm.first_lane = ~0u;
  __syncthreads();
  // candidates per cmask word (positions [64 w, 64 w + 64) inside [sh, thi)):
  // thread t owns word t and, for the last thread, the words past 256
  const uint64_t* cw = (const uint64_t*)sm.cmask;
  const uint32_t t = threadIdx.x;
  const uint32_t nw = (thi + 63) >> 6;
  auto word = [&](uint32_t w) -> uint64_t {
    if (w >= nw) return 0;
    uint64_t m = cw[w];
    const uint32_t b0 = w << 6;
    if (sh > b0) m &= sh - b0 >= 64 ? 0 : ~0ull << (sh - b0);      // before the tile
    if (thi < b0 + 64) m &= thi <= b0 ? 0 : (1ull << (thi - b0)) - 1;  // past its end
    return m;
  };
  const uint64_t m0 = word(t);
  uint64_t mx = 0;
  if (t == kTileLanes - 1)
    for (uint32_t w = kTileLanes; w < nw; ++w) mx |= (uint64_t)__builtin_popcountll(word(w)) << (8 * (w - kTileLanes));
  const uint32_t c0 = (uint32_t)__builtin_popcountll(m0);
  uint32_t cx = 0;
  for (uint32_t k = 0; kCandWords > kTileLanes && k < kCandWords - kTileLanes; ++k)
    cx += (uint32_t)((mx >> (8 * k)) & 0xff);
  unsigned long long total;
  const uint32_t pre = (uint32_t)block_exscan256(c0 + cx, sm.part, &total);
  const uint32_t N = (uint32_t)total;
  if (N > kCandCap || N > a.st_cap) return false;  // (uniform)
  if (t < kCandWords) sm.cl.wbase[t] = (uint16_t)pre;
  {
    uint32_t k = pre;
    for (uint64_t m = m0; m; m &= m - 1) sm.cl.cand[k++] = (uint16_t)((t << 6) + __builtin_ctzll(m));
    for (uint32_t w = kTileLanes; w < nw && t == kTileLanes - 1; ++w) {
      sm.cl.wbase[w] = (uint16_t)k;
      for (uint64_t m = word(w); m; m &= m - 1)
        sm.cl.cand[k++] = (uint16_t)((w << 6) + __builtin_ctzll(m));
    }
    if (t == 0) sm.cl.cand[N] = sm.cl.cand[N + 1] = 0xffffu;  // sentinel: no position
  }
  __syncthreads();
  // one walk per candidate
  for (uint32_t i = t; i < N; i += kTileLanes) {
    const uint32_t c = sm.cl.cand[i];
    uint32_t q = c;
#ifdef TGPU_ABL_NOWALK  // timing ablation only (wrong index): no walks
    const bool ok = false;
#else
    const bool ok = tile_walk(P, src, pc, q, avail);
#endif
    const uint32_t len = q - c;
    sm.cl.len[i] = ok ? (uint16_t)(len < 0xffffu ? len : 0xffffu) : 0;
    if (ok) atomicMin(&sm.first_lane, i);
  }
  __syncthreads();
#ifdef TGPU_SPEC_LATE
  {
    uint32_t late1 = 0;
    for (uint32_t d = threadIdx.x; d < ((staged & ~3u) >> 2); d += kTileLanes)
      late1 ^= ((const volatile uint32_t*)lds)[d] * (d | 1);
    if (late1 != late0) atomicAdd(&a.scal[12], 1ull);  // threads that saw their words change
  }
#endif
  if constexpr (!kOnePass) {
#ifdef TGPU_SPEC_NOEXIT  // A/B: waves 1-3 wait for wave 0 at a final barrier
    if (t >= 64) {
      __syncthreads();
      return true;
    }
#else
    if (t >= 64) return true;  // wave 0 follows the chain and writes the tile's result
#endif
  } else {
    if (threadIdx.x == 0) *res = CandResult{kNoPos, 0, 0, 1, sh, staged, avail, thi};
    if (t >= 64) return true;
  }
  const uint32_t lane = t;
  // the chain's first candidate: the range's first byte (tile 0 of a
  // non-speculative call), else the first canonical record
  uint32_t f;
  bool stuck = false;
  if (ent != kNoPos) {
    const uint64_t m = word(ent >> 6);  // (the counted bits: none before sh)
    const uint64_t bit = 1ull << (ent & 63);
    f = (m & bit) ? sm.cl.wbase[ent >> 6] + (uint32_t)__builtin_popcountll(m & (bit - 1)) : kNoPos;
    stuck = f == kNoPos || sm.cl.len[f] == 0;
  } else {
    f = sm.first_lane;
    if (f == ~0u) f = kNoPos;
  }
  const uint32_t first = f == kNoPos ? (ent != kNoPos ? ent : kNoPos) : sm.cl.cand[f];
  uint32_t count = 0, e = 0;
  uint16_t* dst = kOnePass ? sdst : a.st16 + j * a.st_cap;
  uint32_t i = f;
#ifdef TGPU_ABL_NOCHAIN  // timing ablation only (wrong index): no chain
  stuck = true;
#endif
  while (!stuck && f != kNoPos) {
    // candidates [i, i + 64): lane l's record links to candidate i + l + 1
    const uint32_t x = i + lane;
    const bool in = x < N;
    const uint32_t c = in ? sm.cl.cand[x] : 0xffffu;
    const uint32_t len = in ? sm.cl.len[x] : 0u;
    const uint32_t next = sm.cl.cand[in ? x + 1 : N];
    const uint32_t q = c + len;
    const bool link = in && len != 0 && len != 0xffffu && q < thi && q == next;
    const uint64_t brk = __ballot(!link);
    const uint32_t b = brk ? (uint32_t)__builtin_ctzll(brk) : 64u;
    // lanes [0, b) are records linked to their successor; lane b's record
    // ends the run (its successor is not the next candidate)
    if (lane < b) dst[count + lane] = (uint16_t)c;
    if (b == 64) {
      count += 64;
      i += 64;
      continue;
    }
    const uint32_t cb = __shfl(c, b, 64), lb = __shfl(len, b, 64);
    if (i + b >= N || lb == 0) {  // the run ends in a record the program cannot take
      stuck = true;
      break;
    }
    if (lane == b) dst[count + b] = (uint16_t)cb;
    count += b + 1;
    uint32_t qb = cb + lb;
    if (lb == 0xffffu) {  // a record of 64 KiB or more: measure it again
      qb = cb;
      tile_walk(P, src, pc, qb, avail);
    }
    if (qb >= thi) {  // the record straddling the tile's end: done
      e = qb;
      break;
    }
    // the next record starts at qb: a candidate (every canonical record
    // start after a STOP is one), whose index is its rank in the bits
    const uint64_t m = word(qb >> 6);  // (the counted bits: none before sh)
    const uint64_t bit = 1ull << (qb & 63);
    if (!(m & bit)) {
      stuck = true;
      break;
    }
    i = sm.cl.wbase[qb >> 6] + (uint32_t)__builtin_popcountll(m & (bit - 1));
  }
#ifdef TGPU_SPEC_CHECK  // diagnostics: a tile left partial, its staged bytes against HBM
  if (stuck) {
    uint32_t bad = 0, first_bad = ~0u;
    const uint32_t nw4 = (staged & ~3u) >> 2;
    for (uint32_t d = lane; d < nw4; d += 64) {
      const uint32_t x = ((const uint32_t*)lds)[d];
      const uint32_t y = __builtin_nontemporal_load((const uint32_t*)gb + d);
      if (x != y) {
        ++bad;
        first_bad = min(first_bad, d);
      }
    }
    for (int o = 32; o; o >>= 1) {
      bad += __shfl_xor(bad, o, 64);
      first_bad = min(first_bad, (uint32_t)__shfl_xor(first_bad, o, 64));
    }
    if (lane == 0) {
      atomicAdd(&a.scal[13], 1ull);             // stuck tiles
      if (bad) atomicAdd(&a.scal[14], 1ull);    // ... whose LDS copy differs from HBM
      atomicAdd(&a.scal[15], (unsigned long long)bad);
    }
  }
#endif
  if constexpr (kOnePass) {
    if (lane == 0) *res = CandResult{first, e, count, stuck ? 1u : 0u, sh, staged, avail, thi};
    return true;
  }
  if (lane == 0) {
    const bool none = first == kNoPos;
    const uint64_t st = lo - sh + first;
    a.s[j] = none ? kNo : st;
    // stuck: the general reader walks the whole tile from its (speculated) start
    a.e[j] = none ? kNo : (stuck ? kPartial : lo - sh + e);
    a.cnt[j] = none || stuck ? 0 : count;
    if (!none) a.pf[j] = stuck ? st : kStartsValid;
  }
#ifdef TGPU_SPEC_NOEXIT
  __syncthreads();
#endif
  return true;
}

template <class PP>
__device__ __forceinline__ void index_spec_tile(const IndexArgs& a, const PP& P, uint8_t* lds,
                                                IndexTileShared& sm) {
  const uint64_t j = blockIdx.x;
  const uint64_t lo = chunk_lo(a, j);
  // tile 0 of a non-speculative call starts at begin exactly (relative 0 + sh)
  const uint32_t ent = (j == 0 && !a.speculative) ? (uint32_t)((uintptr_t)(a.in + lo) & 15)
                                                  : kNoPos;
#ifndef TGPU_SLICE_SPEC  // A/B: the slice speculation for every tile
  if (a.st16) {
    if (spec_tile_cands(a, P, j, lds, ent, sm)) return;
    __syncthreads();  // (the slice speculation restages the tile)
  }
#endif
  TileLane L;
  uint32_t sh, first;
  const bool ok = tile_resolve(a, P, j, lds, ent, L, sh, first, sm.E, &sm.flag, &sm.first_lane,
                               &sm.fs, sm.cmask);
  // (ok and first are the same in every lane)
  const bool have = ok && first != kNoPos;
  unsigned long long tile_n = 0;
  const unsigned long long pre =
      block_exscan256(have ? (unsigned long long)L.c : 0ull, sm.part, &tile_n);
  // per-lane starts/counts for the emit pass (valid while the tile keeps this
  // start: pf[j] == kLanesValid)
  if (have) a.lanes[j * kTileLanes + threadIdx.x] = (L.s & 0xffffu) | ((uint32_t)L.c << 16);
  // the tile's record starts in order (pf[j] == kStartsValid): lane k's after
  // those of lanes < k
  bool stored = false;
  if (a.st16 && have) {
    stored = !__syncthreads_or(L.c > kLaneStarts) && tile_n <= a.st_cap;
    if (stored) {
      uint16_t* dst = a.st16 + j * a.st_cap + pre;
      for (uint32_t i = 0; i < L.c; ++i) dst[i] = (uint16_t)get_start(L, i);
    }
  }
  if (threadIdx.x == kTileLanes - 1) {
    // (values selected, then one store each: branches storing to different
    // fields made the compiler keep a table of the field pointers in
    // scratch, written by every lane of every tile)
    const bool none = first == kNoPos;
    const uint64_t st = lo - sh + first;
    a.s[j] = none ? kNo : st;
    // !ok: the general reader walks the whole tile from its (speculated) start
    a.e[j] = none ? kNo : (!ok ? kPartial : lo - sh + L.e);
    a.cnt[j] = none || !ok ? 0 : tile_n;
    if (!none) a.pf[j] = !ok ? st : (stored ? kStartsValid : kLanesValid);
  }
}

// Emit for a tile whose first start is verified (a.s[j]); records starting in
// the tile get their starts written at offs[base[j] ..]. A tile the program
// cannot finish goes to index_emit_cont_kernel whole.
// kDecode (fused index + decode, a.recs set): the walk that finds each start
// also decodes the record (the same program, storing) into an LDS record
// tile (zero-filled = default-initialized records) that leaves with
// coalesced 16-byte stores; records past the LDS tile go to HBM directly;
// a record the program cannot store (list arena overflow) is queued for the
// general decoder. This removes the decode pass's second read of the wire
// and of the index.
#ifndef TGPU_REC_TILE
#define TGPU_REC_TILE (16 * 1024)
#endif
constexpr uint32_t kRecTileBytes = TGPU_REC_TILE;  // keeps the fused tile kernel at 4 workgroups/CU

template <bool kDecode, class PP>
__device__ __forceinline__ void emit_lanes(const IndexArgs& a, const PP& P, const uint8_t* lds,
                                           IndexTileShared& sm, uint8_t* rtile, const TileLane& L,
                                           uint32_t sh, uint64_t lo, uint64_t b);

// Tile j's stored starts are current: the speculation pass stored them and
// the chain still begins where it did (the repair may move a tile's start
// forward onto its speculated chain, take_over).
__device__ __forceinline__ bool starts_current(const IndexArgs& a, uint64_t j) {
  if (a.pf[j] != kStartsValid) return false;
  const uint64_t lo = chunk_lo(a, j);
  const uint64_t gb = lo - ((uintptr_t)(a.in + lo) & 15);
  return gb + a.st16[j * a.st_cap] == a.s[j];
}

template <bool kDecode, class PP>
__device__ __forceinline__ void index_emit_tile(const IndexArgs& a, const PP& P, uint8_t* lds,
                                                IndexTileShared& sm, uint8_t* rtile,
                                                uint64_t j) {
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
    stage_tile(lds, gb, nvec);
    const uint32_t v = a.lanes[j * kTileLanes + threadIdx.x];
    L.s = v & 0xffffu;
    L.c = v >> 16;
    first = ent;
    ok = true;
    TGPU_STAGE_SYNC();
  } else {
    ok = tile_resolve(a, P, j, lds, ent, L, sh, first, sm.E, &sm.flag, &sm.first_lane, &sm.fs,
                      sm.cmask);
  }
  const uint64_t b = a.base[j];
  if (!ok) {
    if (threadIdx.x == 0) {
      a.ep[j] = sj;
      a.ec[j] = 0;
    }
    return;
  }
  emit_lanes<kDecode>(a, P, lds, sm, rtile, L, sh, lo, b);
}

// The emit kernel body: every tile (j = blockIdx.x), or, when the
// speculation pass stored starts (a.st16: index_starts_copy_kernel copied the
// current ones), the tiles it listed in bad[0 .. scal[6]), strided over the
// grid.
template <class PP>
__device__ __forceinline__ void index_emit_kernel_body(const IndexArgs& a, const PP& P,
                                                       uint8_t* lds, IndexTileShared& sm) {
  if (!a.st16) {
    index_emit_tile<false>(a, P, lds, sm, nullptr, blockIdx.x);
    return;
  }
  const uint64_t m = a.scal[6];
  for (uint64_t k = blockIdx.x; k < m; k += gridDim.x) {
    index_emit_tile<false>(a, P, lds, sm, nullptr, a.bad[k]);
    __syncthreads();  // the next tile's staging overwrites lds
  }
}

// The emission body of a tile whose lanes hold verified chains (L) and whose
// first record is record b of the range: starts to offs[b ..], and (kDecode)
// the records decoded through an LDS record tile.
template <bool kDecode, class PP>
__device__ __forceinline__ void emit_lanes(const IndexArgs& a, const PP& P, const uint8_t* lds,
                                           IndexTileShared& sm, uint8_t* rtile, const TileLane& L,
                                           uint32_t sh, uint64_t lo, uint64_t b) {
  // lane k's records go after the records of lanes < k
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long x = wave_incl_scan(L.c);
  if (lane == 63) sm.part[wid] = x;
  __syncthreads();
  unsigned long long pre = x - L.c;
  for (int w = 0; w < wid; ++w) pre += sm.part[w];
  const uint64_t gb = lo - sh;
  const uint8_t* g = a.in + gb;
  const uint64_t avail64 = a.in_len - gb;
  const uint32_t avail = (uint32_t)(avail64 < kPosCap ? avail64 : kPosCap);
  const uint32_t staged = avail < kTile + kOver + 16 ? avail : kTile + kOver + 16;
  const TileSrc src{(const uint32_t*)lds, staged & ~3u, HbmSrc{g, avail}};
  if constexpr (!kDecode) {
    if (L.c == 0) return;
    // re-walk this lane's records, writing absolute starts
    const Ctx pc{0, nullptr, 0, a.string_limit, a.container_limit};
    uint32_t p = L.s;
    for (uint32_t i = 0; i < L.c; ++i) {
      const uint64_t idx = b + pre + i;
      if (idx <= a.max_records) a.offs[idx] = gb + p;
      uint32_t q = p;
      tile_walk(P, src, pc, q, avail);
      p = q;
    }
  } else {
    const uint32_t S = a.rec_size;
    // the tile's records [b, b + m) that are decoded: below n_decode
    const uint64_t tile_n = sm.part[0] + sm.part[1] + sm.part[2] + sm.part[3];
    const uint64_t m = b >= a.n_decode ? 0 : min(tile_n, a.n_decode - b);
    const uint32_t cap_recs = kRecTileBytes / S;
    const uint32_t in_lds = (uint32_t)min(m, (uint64_t)cap_recs);
    uint8_t* gout = a.recs + b * S;
    const uint32_t osh = (uint32_t)((uintptr_t)gout & 15);
    {
      const uint4 z = {0u, 0u, 0u, 0u};
      const uint32_t nz = (osh + in_lds * S + 15) >> 4;
      for (uint32_t i = threadIdx.x; i < nz; i += kTileLanes) ((uint4*)rtile)[i] = z;
    }
    __syncthreads();
    const Ctx pc{gb, a.arena, a.arena_cap, a.string_limit, a.container_limit};
    uint32_t p = L.s;
    for (uint32_t i = 0; i < L.c; ++i) {
      const uint64_t t = pre + i, idx = b + t;
      if (idx <= a.max_records) a.offs[idx] = gb + p;
      uint32_t q = p;
      if (t < m) {
        uint8_t* rec;
        if (t < in_lds) {
          rec = rtile + osh + t * S;
        } else {
          rec = a.recs + idx * S;
          for (uint32_t k = 0; k < S; ++k) rec[k] = 0;
        }
        if (!run_program<true>(P, src, pc, q, avail, rec)) {
          // the program cannot store it (list arena): the general decoder
          // redoes the record from its start; the walk continues with the
          // measured length
          a.irr[atomicAdd(a.nirr, 1ull)] = idx;
          q = p;
          run_program<false>(P, src, pc, q, avail, nullptr);
        }
      } else {
        tile_walk(P, src, pc, q, avail);
      }
      p = q;
    }
    __syncthreads();
    // record tile -> HBM
    const uint32_t end = osh + in_lds * S;
    const uint32_t nvec = (end + 15) >> 4;
    uint8_t* base = gout - osh;
    for (uint32_t i = threadIdx.x; i < nvec; i += kTileLanes) {
      const uint32_t lo16 = i << 4, hi16 = lo16 + 16;
      if (lo16 >= osh && hi16 <= end) {
        ((uint4*)base)[i] = ((const uint4*)rtile)[i];
      } else {
        for (uint32_t k = (lo16 < osh ? osh : lo16); k < (hi16 < end ? hi16 : end); ++k)
          base[k] = rtile[k];
      }
    }
  }
}

// ---- single pass: speculate, look back, emit / decode ----------------------
// The two-pass index (spec, fix, scan, emit) reads every tile twice. Here tile
// j (workgroup j) speculates its chain (tile_resolve), publishes it (AGG: its
// first start s, end e and count) and looks back: predecessors are summed
// while each one's start is its predecessor's end, down to one whose chain is
// verified (INCL: its inclusive record prefix and end are known). Every link
// on the way matching means every chain on the way starts at the true end of
// a verified chain, so this tile's prefix is their sum and it is INCL. Its own
// link broken (the chain below verified): the tile re-chains from the true
// start (the bytes are still in LDS) — the repair the two-pass index does in
// index_fix_kernel. A broken link further down: that tile repairs itself;
// this one waits for it. Then the tile emits its starts and decodes its
// records exactly like the two-pass emit tile. Anything a tile cannot do
// alone (a record the program does not take, no record start in the tile, a
// record end past the packed fields' range, a wait past its bound) is FAIL,
// which every later tile inherits; the caller then runs the two-pass index.
//
// Each status is ONE 64-bit word written and read with relaxed agent-scope
// atomics (sc1 stores / loads): no release / acquire, whose L2 write-back and
// invalidate (buffer_wbl2 / buffer_inv, one per tile, with the L2 full of the
// decode's output) made the first version 6x slower than the two passes.
//   AGG  (a.pf[j]):  01 | cnt:15 | s - lo:15 (0x7fff: s = e) | e - lo:32
//   FAIL (a.pf[j]):  11 | 0
//   INCL (a.ep[j]):  1 | e - hi:23 | inclusive prefix:40
// Tiles go in workgroup order: workgroups are dispatched in index order (per
// XCD), so a lower tile is resident or done whenever this one runs (a ticket
// counter — one atomic per tile on one address — cost 1.5 ms over 256 Ki
// tiles in the encoder experiment). Every wait is bounded
// (kOpSpinCap): a missed bound fails the pass, never hangs it. a.scal[7]: the
// fail flag (TGPU_ONEPASS_STATS: counters in a.scal[8..11]).
constexpr uint32_t kOpSpinCap = 1u << 20;
constexpr uint64_t kAggTag = 1ull << 62, kFailTag = 3ull << 62, kInclTag = 1ull << 63;
constexpr uint64_t kSSame = 0x7fff;

template <class T>
__device__ __forceinline__ uint64_t op_ld(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void op_st(T* p, uint64_t v) {
  __hip_atomic_store(p, (T)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// AGG word for a chain [s, e) of c records in tile [lo, hi); 0 when the
// fields cannot hold it.
__device__ __forceinline__ uint64_t op_agg(uint64_t lo, uint64_t s, uint64_t e, uint64_t c) {
  if (e < lo || e - lo > 0xffffffffull || c > 0x7fff) return 0;
  const uint64_t sr = s == e ? kSSame : s - lo;
  if (sr > kSSame) return 0;
  return kAggTag | (c << 47) | (sr << 32) | (e - lo);
}
__device__ __forceinline__ uint64_t op_incl(uint64_t hi, uint64_t e, uint64_t incl) {
  if (e < hi || e - hi >= (1ull << 23) || incl >= (1ull << 40)) return 0;
  return kInclTag | ((e - hi) << 40) | incl;
}

// Waits until tile k is INCL or FAIL: its INCL word, or kFailTag, or 0 after
// the bound.
__device__ __forceinline__ uint64_t op_wait_final(const IndexArgs& a, uint64_t k) {
  for (uint32_t spin = 0; spin < kOpSpinCap; ++spin) {
    const uint64_t iw = op_ld(a.ep + k);
    if (iw) return iw;
    if (op_ld(a.pf + k) == kFailTag) return kFailTag;
    __builtin_amdgcn_s_sleep(2);
  }
  return 0;
}

struct OnePassShared {
  uint64_t e;       // the tile's chain end (absolute)
  uint64_t verdict; // 1 INCL, 3 FAIL, 0: repair from `start`
  uint64_t prefix, start;
};
constexpr uint64_t kOpIncl = 1, kOpFail = 3;

// Wave 0: the look-back of tile j whose speculated chain starts at s, 64
// predecessors per round trip (lane l reads tile top - l): the first lane
// whose tile is verified (INCL) or failed stops the window; every link above
// it (tile k's end == tile k + 1's start) must hold. Tile j's own link broken
// while the chain below verifies: re-chain from tile j - 1's end (verdict 0).
// A link broken further down: that tile repairs itself; wait for it and look
// again. No verified tile in the window: its counts are summed and the window
// moves down.
__device__ __forceinline__ void op_look_back(const IndexArgs& a, uint64_t j, uint64_t s,
                                             OnePassShared& op) {
  const uint32_t l = threadIdx.x;  // 0..63
  if (j == 0) {  // the range's first tile starts at begin (or opens a speculative range)
    if (l == 0) {
      op.verdict = kOpIncl;
      op.prefix = 0;
    }
    return;
  }
  int verdict = 2;  // 0 repair, 1 incl, 2 fail, 3 look again
  uint64_t prefix = 0, own = kNo;
  for (uint32_t restart = 0; restart < 64; ++restart) {
    uint64_t need = s, sum = 0;
    own = kNo;
    int64_t top = (int64_t)j - 1;
    verdict = -1;
    while (verdict < 0) {
      const int64_t k = top - (int64_t)l;
      const bool valid = k >= 0;
      uint64_t iw = 0, aw = 0;
      if (valid) {
        iw = op_ld(a.ep + k);
        aw = iw ? 0 : op_ld(a.pf + k);
      }
      for (uint32_t spin = 0; __any(valid && !iw && !aw); ++spin) {
        if (spin >= kOpSpinCap) {
          aw = kFailTag;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        if (valid && !iw && !aw) {
          iw = op_ld(a.ep + k);
          aw = iw ? 0 : op_ld(a.pf + k);
        }
      }
      const bool incl = iw != 0;
      const bool fail = !incl && aw == kFailTag;
      const uint64_t lo = valid ? chunk_lo(a, (uint64_t)k) : 0;
      const uint64_t hi = valid ? chunk_hi(a, (uint64_t)k) : 0;
      const uint64_t ek = incl ? hi + ((iw >> 40) & ((1ull << 23) - 1)) : lo + (aw & 0xffffffffull);
      const uint64_t sr = (aw >> 32) & kSSame;
      const uint64_t sk = sr == kSSame ? ek : lo + sr;
      const uint64_t ck = incl ? 0 : (aw >> 47) & 0x7fff;
      // the start of tile k + 1: lane l - 1's tile (lane 0: the chain above)
      uint64_t above = __shfl_up(sk, 1, 64);
      if (l == 0) above = need;
      const uint64_t stops = __ballot(valid && (incl || fail));
      const uint32_t stop = stops ? (uint32_t)__builtin_ctzll(stops) : 64u;
      bool broken = valid && l <= stop && !fail && ek != above;
      if (top == (int64_t)j - 1 && l == 0 && broken) {
        own = ek;  // tile j's own link: it re-chains from here if the rest holds
        broken = false;
      }
      own = __shfl(own, 0, 64);
      const uint64_t bm = __ballot(broken);
      if (bm) {  // tile (top - m) + 1 starts wrong: it repairs itself
        const uint32_t m = (uint32_t)__builtin_ctzll(bm);
        const uint64_t kb = (uint64_t)(top - (int64_t)m) + 1;
        uint64_t w = 0;
        if (l == 0) w = op_wait_final(a, kb);
        w = __shfl(w, 0, 64);
        verdict = (w == 0 || w == kFailTag) ? 2 : 3;
        break;
      }
      uint64_t c = l < stop && valid ? ck : 0;
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
      if (stop < 64) {
        const uint64_t ws = __shfl(iw, stop, 64);
        if (!ws) {  // the stop is a failed tile
          verdict = 2;
          break;
        }
        prefix = (ws & ((1ull << 40) - 1)) + c + sum;
        verdict = own == kNo ? 1 : 0;
        break;
      }
      if (top < 63) {  // down to tile 0, which is not verified yet: wait for it
        uint64_t w = 0;
        if (l == 0) w = op_wait_final(a, 0);
        w = __shfl(w, 0, 64);
        verdict = (w == 0 || w == kFailTag) ? 2 : 3;
        break;
      }
      sum += c;
      need = __shfl(sk, 63, 64);
      top -= 64;
#ifdef TGPU_ONEPASS_STATS
      if (l == 0) atomicAdd(&a.scal[8], 1ull);
#endif
    }
    if (verdict != 3) break;
#ifdef TGPU_ONEPASS_STATS
    if (l == 0) atomicAdd(&a.scal[9], 1ull);
#endif
  }
  if (l == 0) {
    op.verdict = verdict == 1 ? kOpIncl : verdict == 0 ? 0 : kOpFail;
    op.prefix = prefix;
    op.start = own;
  }
}

// Thread 0: tile j's final word (INCL, or FAIL when the fields cannot hold it)
// and the arrays the index epilogue reads.
__device__ __forceinline__ void op_publish_incl(const IndexArgs& a, uint64_t j, uint64_t s,
                                                uint64_t e, uint64_t c, uint64_t prefix,
                                                OnePassShared& op) {
  const uint64_t w = op_incl(chunk_hi(a, j), e, prefix + c);
  if (!w) {
    op.verdict = kOpFail;
    atomicExch(&a.scal[7], 1ull);
    op_st(a.pf + j, kFailTag);
    return;
  }
  a.s[j] = s;
  a.e[j] = e;
  a.cnt[j] = c;
  a.base[j] = prefix;
  op_st(a.ep + j, w);
}

template <bool kDecode, class PP>
__device__ __forceinline__ void index_onepass_tile(const IndexArgs& a, const PP& P, uint8_t* lds,
                                                   IndexTileShared& sm, uint8_t* rtile,
                                                   OnePassShared& op) {
  const uint64_t j = blockIdx.x;
  const uint64_t lo = chunk_lo(a, j), hi = chunk_hi(a, j);
  const uint32_t sh0 = (uint32_t)((uintptr_t)(a.in + lo) & 15);
  const uint32_t ent = (j == 0 && !a.speculative) ? sh0 : kNoPos;
  TileLane L;
  uint32_t sh, first;
  bool ok = tile_resolve(a, P, j, lds, ent, L, sh, first, sm.E, &sm.flag, &sm.first_lane, &sm.fs,
                         sm.cmask);
  bool good = ok && first != kNoPos;
  for (int pass = 0; pass < 2; ++pass) {
    if (threadIdx.x == 0) sm.csum = 0;
    __syncthreads();
    if (good) atomicAdd(&sm.csum, (unsigned long long)L.c);
    if (threadIdx.x == kTileLanes - 1) op.e = lo - sh + L.e;
    __syncthreads();
    const uint64_t sj = lo - sh + first, cj = sm.csum;
    uint64_t aw = 0;
    if (good && pass == 0) aw = op_agg(lo, sj, op.e, cj);
    if (threadIdx.x == 0) {
      if (!good || (pass == 0 && !aw)) {
        op.verdict = kOpFail;
        atomicExch(&a.scal[7], 1ull);
        op_st(a.pf + j, kFailTag);
      } else if (pass == 0) {
        op_st(a.pf + j, aw);
      }
    }
#ifdef TGPU_ONEPASS_NOLOOK  // A/B timing only: no look-back (wrong record positions)
    if (pass == 0 && aw && threadIdx.x == 0) {
      op.verdict = kOpIncl;
      op.prefix = 0;
    }
#else
    if (pass == 0 && aw && threadIdx.x < 64) op_look_back(a, j, sj, op);
#endif
    if (threadIdx.x == 0 && good && (pass == 1 || aw)) {
      if (pass == 1) op.verdict = kOpIncl;  // re-chained from the verified start
      if (op.verdict == kOpIncl) {
        op_publish_incl(a, j, sj, op.e, cj, op.prefix, op);
      } else if (op.verdict == kOpFail) {
        atomicExch(&a.scal[7], 1ull);
        op_st(a.pf + j, kFailTag);
#ifdef TGPU_ONEPASS_STATS
        atomicAdd(&a.scal[11], 1ull);
#endif
      }
    }
    __syncthreads();
    if (op.verdict != 0) break;
#ifdef TGPU_ONEPASS_STATS
    if (threadIdx.x == 0) atomicAdd(&a.scal[10], 1ull);
#endif
    if (op.start >= hi) {  // the true chain passes the whole tile: no record starts here
      L.s = L.e = L.c = 0;
      if (threadIdx.x == 0) {
        op.verdict = kOpIncl;
        op_publish_incl(a, j, op.start, op.start, 0, op.prefix, op);
      }
      __syncthreads();
      break;
    }
    // repair: the chain from the verified start, inside this tile
    ok = tile_resolve(a, P, j, lds, (uint32_t)(op.start - (lo - sh0)), L, sh, first, sm.E,
                      &sm.flag, &sm.first_lane, &sm.fs, sm.cmask);
    good = ok && first != kNoPos;
  }
  if (op.verdict != kOpIncl) return;
#ifndef TGPU_ONEPASS_NOEMIT  // A/B timing only: no emission
  emit_lanes<kDecode>(a, P, lds, sm, rtile, L, sh, lo, op.prefix);
#endif
}

// ---- one pass over the candidate-list speculation, records in registers ------
// (round 6, verdict item 2: config 5 parses each record once, where the two
// passes walked every record in the speculation and decoded it again from a
// second staging of the wire.) Per 16 KiB tile: the candidate-list
// speculation (spec_tile_cands) with the chain's record starts kept in LDS;
// the tile's (first, end, count) published as an AGG word and the record
// base found by the decoupled look-back (op_look_back: a window of 64
// predecessors per round trip, every link between neighbours checked; no
// single ticket counter — tiles publish at their own index); then every lane
// decodes records of the staged tile with the program into registers (kRS)
// and stores them at their global index, with their starts. Anything
// unusual — a tile the speculation or the program cannot take, a broken
// link, a record the program cannot store — publishes FAIL (scal[7]) and the
// host redoes the range with the two-pass index, which decides everything.
template <class PP, uint32_t kRS>
__device__ __forceinline__ void index_onepass_rr_tile(const IndexArgs& a, const PP& P,
                                                      uint8_t* lds, IndexTileShared& sm,
                                                      OnePassShared& op, uint16_t* sst,
                                                      CandResult& cr) {
  static_assert(kRS % 8 == 0 && kRS <= 128, "register record: whole 8-byte words");
  const uint64_t j = blockIdx.x;
  const uint64_t lo = chunk_lo(a, j);
  const uint32_t sh0 = (uint32_t)((uintptr_t)(a.in + lo) & 15);
  const uint32_t ent = (j == 0 && !a.speculative) ? sh0 : kNoPos;
  const bool listed = spec_tile_cands<PP, true>(a, P, j, lds, ent, sm, sst, &cr);
  __syncthreads();  // wave 0's chain (sst) and result (cr)
  const uint32_t first = cr.first, count = cr.count, sh = cr.sh;
  const bool good = listed && !cr.stuck && first != kNoPos && count > 0;
  const uint64_t sj = lo - sh + first, ej = lo - sh + cr.e;
  if (threadIdx.x == 0) {
    op.verdict = kOpFail;
    const uint64_t aw = good ? op_agg(lo, sj, ej, count) : 0;
    if (!aw) {
      atomicExch(&a.scal[7], 1ull);
      op_st(a.pf + j, kFailTag);
    } else {
      op_st(a.pf + j, aw);
    }
    op.e = aw;  // (here: the AGG word published, 0 when the tile failed)
  }
  __syncthreads();
  if (!op.e) return;
  const uint8_t* gb = a.in + lo - sh;
  const TileSrc src{(const uint32_t*)lds, cr.staged & ~3u, HbmSrc{gb, cr.avail}};
  const Ctx c{lo - sh, a.arena, a.arena_cap, a.string_limit, a.container_limit, nullptr};
  // Records of up to 64 bytes in a tile of at most 512: decoded into
  // registers while wave 0 looks back (waves 1-3 take records [0, 384), wave
  // 0 the rest after its look-back — the look-back's round trips, 0.67 ms
  // of the call when nothing overlapped them, hide behind the parse), then
  // they leave through an LDS image of 256 records in the (by then dead)
  // wire tile with 16-byte stores (per-lane stores of 56-byte records
  // measured dearer). Otherwise every lane decodes and stores its records
  // after the look-back.
  constexpr bool kStage = kRS <= 64 && kTileLanes * kRS + 16 <= kTileLds;
#ifdef TGPU_OP_LANE_STORES  // A/B: every record stored by its lane
  const bool staged = false;
#else
  const bool staged = kStage && count <= 2 * kTileLanes;
#endif
  const uint32_t t = threadIdx.x;
  bool bad = false;
  alignas(16) uint8_t rb[2][kRS];
  // record of slot q of lane t
  auto slot = [&](uint32_t q) -> uint32_t { return t < 64 ? 384 + t + 64 * q : (t - 64) + 192 * q; };
  auto parse = [&](uint32_t q) {
    const uint32_t i = slot(q);
#pragma unroll
    for (uint32_t b = 0; b < kRS; b += 8) *(uint64_t*)(rb[q] + b) = 0;
    if (i < count) {
      uint32_t p = sst[i];
      const uint32_t pe = i + 1 < count ? sst[i + 1] : cr.e;
      bad |= !(run_program<true>(P, src, c, p, pe, rb[q]) && p == pe);
    }
  };
  // (waves 1-3 skip the look-back block and parse at once; wave 0 after it:
  // one call site of the unrolled parse)
  if (t < 64) {
#ifdef TGPU_OP_ABL_NOLOOK  // timing ablation only (records at wrong positions): no look-back
    if (t == 0) {
      op.verdict = kOpIncl;
      op.prefix = 0;
    }
#else
    op_look_back(a, j, sj, op);
#endif
    if (t == 0) {
      if (op.verdict == kOpIncl) {
        op_publish_incl(a, j, sj, ej, count, op.prefix, op);  // (FAIL when the fields overflow)
      } else {  // a broken link (repair) or a failed predecessor: the two passes decide
        op.verdict = kOpFail;
        atomicExch(&a.scal[7], 1ull);
        op_st(a.pf + j, kFailTag);
      }
    }
  }
  if (staged) {
    parse(0);
    parse(1);
  }
  __syncthreads();  // look-back done, every staged record parsed (the wire tile is free)
  if (op.verdict != kOpIncl) return;
  const uint64_t base = op.prefix;
  const uint64_t lim = a.max_records < a.n_decode ? a.max_records : a.n_decode;
  for (uint32_t i = t; i < count; i += kTileLanes)  // record starts
    if (base + i < a.max_records) a.offs[base + i] = lo - sh + sst[i];
#ifdef TGPU_OP_ABL_NODECODE  // timing ablation only: the index without the records
  if (count) return;
#endif
  if (staged) {
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {  // image of records [256 h, 256 h + 256)
      const uint32_t r0 = h * kTileLanes;
      if (r0 >= count || base + r0 >= lim) break;  // (uniform)
      uint32_t nr = count - r0 < kTileLanes ? count - r0 : kTileLanes;
      if (base + r0 + nr > lim) nr = (uint32_t)(lim - base - r0);
      uint8_t* g = a.recs + (base + r0) * kRS;
      const uint32_t osh = (uint32_t)((uintptr_t)g & 15);
#pragma unroll
      for (uint32_t q = 0; q < 2; ++q) {
        const uint32_t i = slot(q);
        if (i >= r0 && i < r0 + nr) {
#pragma unroll
          for (uint32_t b = 0; b < kRS; b += 8)
            *(uint64_t*)(lds + osh + (i - r0) * kRS + b) = *(const uint64_t*)(rb[q] + b);
        }
      }
      __syncthreads();
      const uint32_t end = osh + nr * kRS;
      uint8_t* gbr = g - osh;
      for (uint32_t v = t; v < ((end + 15) >> 4); v += kTileLanes) {
        const uint32_t vlo = v << 4, vhi = vlo + 16;
        if (vlo >= osh && vhi <= end) {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(((const u32x4*)lds)[v], (u32x4*)gbr + v);
        } else {  // (records are 8-byte multiples: the edges are 8-byte halves)
          if (vlo >= osh && vlo + 8 <= end) ((uint64_t*)gbr)[2 * v] = ((const uint64_t*)lds)[2 * v];
          if (vlo + 8 >= osh && vhi <= end)
            ((uint64_t*)gbr)[2 * v + 1] = ((const uint64_t*)lds)[2 * v + 1];
        }
      }
      __syncthreads();
    }
  } else {
    for (uint32_t i = t; i < count; i += kTileLanes) {
      const uint64_t R = base + i;
      uint32_t p = sst[i];
      const uint32_t pe = i + 1 < count ? sst[i + 1] : cr.e;
      alignas(16) uint8_t rbuf[kRS];
#pragma unroll
      for (uint32_t b = 0; b < kRS; b += 8) *(uint64_t*)(rbuf + b) = 0;
      const bool ok = run_program<true>(P, src, c, p, pe, rbuf) && p == pe;
      bad |= !ok;
      if (R < lim) store_reg_record<kRS>(a.recs + R * kRS, rbuf, a.recs);
    }
  }
  if (__syncthreads_or(bad) && t == 0) atomicExch(&a.scal[7], 1ull);
}

// ================================================ single-pass encode ======
// Round 6 (verdict item 4): the compiled write pass without the size pass.
// Tile j sizes its records (register records, as the two-pass write does),
// publishes its byte total in a.block_sums[j] (AGG; tile 0 its INCL) and
// emits its records into the zero-filled LDS output tile at phase 0 — no base
// needed — and wave 0 looks back over the predecessors' words (AGG totals
// summed down to the first INCL) and publishes INCL. The tile then leaves
// through 16-byte stores assembled from the phase-0 tile with alignbyte (one
// more LDS dword per store). The base is only needed for the stores, the
// start offsets, the output cap check and the records past the LDS tile.
// Measured (config 3, kbench_env / kbench_jit A/Bs on one box each): the body
// without a look-back runs 2.07 ms against 2.51 ms for the two passes, but
// every look-back form found the base too late for 256-record tiles (~12 µs
// of workgroup life, ~1,500 resident; the predecessors' words cost a memory
// round trip each poll): look-back before wave 0's emission 3.11-3.18 ms; a
// two-level form over 64-tile groups (atomic group sums) 3.80 ms; a fifth
// wave that only looks back 3.27 ms (6.1 ms grouped); the 256 nearest words
// loaded ahead of wave 0's emission 3.03 ms (config 4: 1.76 vs 1.55 ms). So
// the two passes stay the default and this one is TGPU_ENCODE_ONEPASS=1.
// No failure state: every tile publishes AGG without waiting on anyone, and
// workgroups dispatch in index order, so every wait ends; past a bound
// (kEncSpinCap) the waiting wave sizes the silent predecessor's records
// itself from HBM (correct, only slower) rather than hang.
// a.block_sums: one status word per tile, zeroed before the launch.
constexpr uint32_t kEncSpinCap = 1u << 16;
constexpr uint64_t kEncAgg = 1ull << 62, kEncIncl = 2ull << 62, kEncVal = (1ull << 62) - 1;

template <class PP>
__device__ __forceinline__ unsigned long long enc_tile_total(const EncodeArgs& a, const PP P,
                                                         uint64_t k, uint32_t S) {
  // (wave 0: tile k's byte total, sized from HBM — the look-back's fallback)
  const uint64_t r0 = k * kET;
  const uint32_t nrec = (uint32_t)min((uint64_t)kET, a.n - r0);
  unsigned long long t = 0;
  for (uint32_t q = threadIdx.x; q < nrec; q += 64) {
    bool ok = true;
    t += program_size(P, PtrRec{a.recs + (r0 + q) * S}, a.lbase, ok);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  return t;
}

template <class PP>
__device__ __forceinline__ uint64_t enc_look_back(const EncodeArgs& a, const PP& P, uint64_t j,
                                                  uint32_t S) {
  const uint32_t l = threadIdx.x;
  unsigned long long* st = a.block_sums;
  uint64_t sum = 0;
  for (int64_t top = (int64_t)j - 1; top >= 0; top -= 64) {
    const int64_t k = top - (int64_t)l;
    uint64_t w = k >= 0 ? op_ld(st + k) : kEncIncl;  // (below tile 0: prefix 0)
    for (uint32_t spin = 0; __any(w == 0); ++spin) {
      if (spin >= kEncSpinCap) {
        for (uint64_t m = __ballot(w == 0); m; m &= m - 1) {
          const uint32_t q = (uint32_t)__builtin_ctzll(m);
          const unsigned long long t = enc_tile_total(a, P, (uint64_t)(top - q), S);
          if (l == q) w = kEncAgg | t;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      if (w == 0) w = op_ld(st + k);
    }
    const uint64_t fin = __ballot(w >= kEncIncl);
    const uint32_t stop = fin ? (uint32_t)__builtin_ctzll(fin) : 64u;
    uint64_t v = l <= stop ? (w & kEncVal) : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    sum += v;
    if (fin) break;
  }
  return sum;
}

// The tile is one workgroup of 256 lanes (one record each). Wave 0
// publishes the tile's AGG word and issues the loads of the 256 nearest
// predecessors' words before it emits its own records; it reads them after
// its emission, when they have arrived and are mostly final, and only
// re-polls the ones still empty (then continues 64 per round trip past the
// window if it held no INCL). Measured variants (config 3, kbench_jit):
// look-back before wave 0's emission +1.1 ms over no look-back; a fifth wave
// that only looks back: +0.27 ms for the extra wave alone.
#ifndef TGPU_ENC1_WIN
#define TGPU_ENC1_WIN 4  // predecessor words per lane of wave 0 loaded ahead
#endif

template <class PP, uint32_t SR>
__device__ __forceinline__ void write_tile_one(const EncodeArgs& a, const PP& P, uint8_t* smem,
                                               EncodeShared& sm) {
  static_assert(PP::kStatic && SR > 0, "compiled programs with register records");
  constexpr uint32_t kW = TGPU_ENC1_WIN;
  const uint64_t j = blockIdx.x;
  const uint64_t r0 = j * kET;
  const uint32_t nrec = (uint32_t)min((uint64_t)kET, a.n - r0);
  const uint32_t ocap = a.out_cap ? a.out_cap : kOutCap;
  uint8_t* otile = smem;
  const uint32_t r = threadIdx.x, lane = r & 63;
  const bool own = r < nrec;
  constexpr uint32_t kAhead = TGPU_ENC_AHEAD;
  RegRec<SR> R;
  StrAhead<kAhead> ah;
  if (own) R.load(a.recs + (r0 + r) * SR);
  unsigned long long sz = 0, tile_total;
  if (own) {
    bool ok = true;
    sz = program_size(P, R, a.lbase, ok);
    if (!ok) atomicMin(&a.res->first_fail, (unsigned long long)(r0 + r));
    str_ahead(P, R, a.sbase, ah);
  }
  const unsigned long long rel = block_exscan256(sz, sm.part, &tile_total);
  unsigned long long* ts = a.block_sums;
  uint64_t w[kW];
  if (r < 64) {
    if (r == 0) op_st(ts + j, (j == 0 ? kEncIncl : kEncAgg) | tile_total);
#pragma unroll
    for (uint32_t q = 0; q < kW; ++q) {  // (distance lane + 64 q + 1)
      const int64_t k = (int64_t)j - 1 - (int64_t)(lane + 64 * q);
      w[q] = k >= 0 ? op_ld(ts + k) : kEncIncl;  // (below tile 0: prefix 0)
    }
  }
  {  // zero the part of the (phase-0) output tile the records OR into
    const uint4 z = {0u, 0u, 0u, 0u};
    const uint32_t nz = ((uint32_t)min(tile_total, (unsigned long long)ocap) + 8 + 15) >> 4;
    for (uint32_t i = r; i < nz; i += kET) ((uint4*)otile)[i] = z;
  }
  if (r == 0) sm.lds_end = (unsigned int)min(tile_total, (unsigned long long)ocap);
  lds_barrier();
  // (rel is monotone: the records past the first one that misses the LDS
  // tile miss it too)
  const bool fits = own && rel + sz <= ocap;
  if (fits) {
    OrSink o((uint32_t*)otile, (uint32_t)rel);
    program_emit<PP, OrSink, RegRec<SR>, kAhead>(P, R, a.sbase, a.lbase, o, &ah);
  }
  if (own && !fits) atomicMin(&sm.lds_end, (unsigned int)min(rel, (unsigned long long)ocap));
  if (r < 64 && j > 0) {
#if defined(TGPU_ENC1_NOLB)  // (timing ablation only: wrong output)
    const uint64_t p = j * tile_total;
#else
    uint64_t p = 0;
    bool done = false;
#pragma unroll
    for (uint32_t q = 0; q < kW; ++q) {
      if (done) break;
      const int64_t k = (int64_t)j - 1 - (int64_t)(lane + 64 * q);
      for (uint32_t spin = 0; __any(w[q] == 0); ++spin) {
        if (spin >= kEncSpinCap) {  // (a silent predecessor: size it from HBM)
          for (uint64_t m = __ballot(w[q] == 0); m; m &= m - 1) {
            const uint32_t u = (uint32_t)__builtin_ctzll(m);
            const unsigned long long tt =
                enc_tile_total(a, P, j - 1 - (u + 64 * q), SR);
            if (lane == u) w[q] = kEncAgg | tt;
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if (w[q] == 0) w[q] = op_ld(ts + k);
      }
      const uint64_t fin = __ballot(w[q] >= kEncIncl);
      const uint32_t stop = fin ? (uint32_t)__builtin_ctzll(fin) : 64u;
      uint64_t v = lane <= stop ? (w[q] & kEncVal) : 0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      p += v;
      done = fin != 0;
    }
    if (!done)  // past the window (all AGG): the prefix below its farthest tile
      p += enc_look_back(a, P, j - 64 * kW, SR);
#endif
    if (r == 0) {
      op_st(ts + j, kEncIncl | (p + tile_total));
      sm.base = p;
    }
  }
  if (r == 0 && j == 0) sm.base = 0;
  lds_barrier();
  const unsigned long long tile_base = sm.base;
  uint8_t* gtile = a.out + tile_base;
  if (own) {
    const unsigned long long start = tile_base + rel;
    if (a.offs) a.offs[r0 + r] = start;
    if (start + sz > a.cap) {
      atomicMin(&a.res->first_fail, (unsigned long long)(r0 + r));
      atomicMin(&sm.lds_end, (unsigned int)min(rel, (unsigned long long)ocap));
    } else if (!fits) {  // (one unrolled emitter per kernel: this one from HBM)
      emit_to_hbm(P, a.recs + (r0 + r) * SR, a.sbase, a.lbase, gtile + rel);
    }
  }
  if (r == 0 && r0 + nrec == a.n) {  // (the scan's totals, two-pass form)
    if (a.offs) a.offs[a.n] = tile_base + tile_total;
    a.res->total_bytes = tile_base + tile_total;
  }
  lds_barrier();
  // LDS tile [0, lds_end) -> HBM [gtile, gtile + lds_end): 16-byte stores at
  // the stream's alignment, each from five LDS dwords (the phase is uniform)
  const uint32_t osh = (uint32_t)((uintptr_t)gtile & 15);
  const uint32_t end = osh + sm.lds_end;
  const uint32_t nvec = (end + 15) >> 4;
  uint8_t* gb = gtile - osh;
  const uint32_t* o32 = (const uint32_t*)otile;
  const uint32_t ph = (16 - osh) & 3;  // (16 i - osh) & 3
  for (uint32_t i = r; i < nvec; i += kET) {
    const uint32_t lo = i << 4, hi = lo + 16;
    if (lo >= osh && hi <= end) {
      const uint32_t d = (lo - osh) >> 2;
      const uint32_t w0 = o32[d], w1 = o32[d + 1], w2 = o32[d + 2], w3 = o32[d + 3];
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      u32x4 v;
      if (ph == 0) {
        v = u32x4{w0, w1, w2, w3};
      } else {
        const uint32_t w4 = o32[d + 4];
        v = u32x4{__builtin_amdgcn_alignbyte(w1, w0, ph), __builtin_amdgcn_alignbyte(w2, w1, ph),
                  __builtin_amdgcn_alignbyte(w3, w2, ph), __builtin_amdgcn_alignbyte(w4, w3, ph)};
      }
      __builtin_nontemporal_store(v, (u32x4*)gb + i);
    } else {
      for (uint32_t b = (lo < osh ? osh : lo); b < (hi < end ? hi : end); ++b)
        gb[b] = otile[b - osh];
    }
  }
}

}  // namespace prog
}  // namespace tgpu
