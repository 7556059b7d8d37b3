// tgpu_xcode.h — wire-to-wire transcoding of an indexed stream, one record
// per lane, without materializing records in HBM (tgpu_transcode_batch):
// the reference's transcoder is "single-pass without a DOM: wire-to-wire"
// (thrift/lib/cpp2/transcode/README.md:5,15); per record it equals
// serialize<To>(deserialize<From>(…)) with the generated codecs (unknown
// fields dropped, as readNoXfer drops them).
//
// Two tile passes over the source stream, each with the source program's
// decode and the target program's writer as compile-time constants (the
// schema compiler instantiates them on both programs, tgpu_jit.cpp
// JIT_XCODE; the AOT library on DynProg pairs, k_transcode.hip):
//   size   stage the tile's source bytes in LDS (LDS-DMA), decode each record
//          into registers (or an LDS record tile), size its target encoding
//          (program_size) -> the tile's sum; a record the source program
//          cannot take (off the canonical form, damaged, past a limit) is
//          listed for the general reader
//   scan   the tile sums (launch_scan_tiles)
//   write  stage and decode again, block scan of the sizes, emit each record
//          into the zero-filled LDS output tile (program_emit), 16-byte
//          stores out. String payloads are read from the staged source tile
//          (LDS), Binary list elements from the tile too (converted in place
//          by the decode, as decode_tile does); Compact list elements go
//          through a list workspace in HBM.
// The listed records are decoded by the general reader into a record
// workspace, sized and written by the general writer at the positions the
// write pass left them (k_transcode.hip) — only those records touch HBM as
// records. Nothing is read back to the host inside the call.
#pragma once

#include "tgpu_prog_kernels.h"

namespace tgpu {
namespace prog {

struct XcTile {
  uint64_t r0;
  uint32_t nrec;
  uint64_t t0, t1;
  uint32_t sh;
  bool ok;
};

// The tile's source bytes [offs[r0], offs[r0 + nrec]) -> LDS (LDS-DMA, the
// settle of decode_tile); ok = false when they do not fit wire_cap (every
// record of the tile then goes to the general reader).
__device__ __forceinline__ XcTile xc_stage(const DecodeArgs& a, uint32_t wire_cap, uint8_t* wire) {
  XcTile t;
  t.r0 = (uint64_t)blockIdx.x * kPT;
  t.nrec = (uint32_t)min((uint64_t)kPT, a.n - t.r0);
  t.t0 = a.offs[t.r0];
  t.t1 = a.offs[t.r0 + t.nrec];
  t.ok = t.t1 >= t.t0 && t.t1 <= a.in_len && (t.t1 - t.t0) + 16 <= wire_cap;
  t.sh = 0;
  if (t.ok) {
    const uint8_t* g = a.in + t.t0;
    t.sh = (uint32_t)((uintptr_t)g & 15);
    const uint4* src = (const uint4*)(g - t.sh);
    const uint32_t nvec = (uint32_t)((t.t1 - t.t0) + t.sh + 15) >> 4;
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
  return t;
}

// Record r0 + threadIdx.x decoded by the source program into rec (zeroed
// first); lists of a Binary source converted in place in the wire tile.
template <class PS, uint32_t kRS>
__device__ __forceinline__ bool xc_decode(const DecodeArgs& a, const PS& Ps, const XcTile& t,
                                          uint8_t* wire, bool stage_lists, uint8_t* rec,
                                          uint32_t S) {
  if constexpr (kRS != 0) {
#pragma unroll
    for (uint32_t b = 0; b < kRS; b += 8) *(uint64_t*)(rec + b) = 0;
  } else {
    for (uint32_t b = 0; b < S; ++b) rec[b] = 0;
  }
  if (!t.ok) return false;
  const uint32_t r = threadIdx.x;
  const uint64_t s = a.offs[t.r0 + r], e = a.offs[t.r0 + r + 1];
  if (!(s >= t.t0 && e >= s && e <= t.t1)) return false;
  // (a staged Binary list converts in the tile; the arena pointer is only
  // checked for capacity then, never written)
  const Ctx c{t.t0 - t.sh, stage_lists ? (uint8_t*)a.in : a.arena,
              stage_lists ? a.in_len : a.arena_cap, a.string_limit, a.container_limit,
              stage_lists ? wire : nullptr};
  uint32_t p = (uint32_t)(s - t.t0) + t.sh;
  const uint32_t pe = (uint32_t)(e - t.t0) + t.sh;
  return run_program<true>(Ps, LdsSrc{(const uint32_t*)wire}, c, p, pe, rec) && p == pe;
}

// Generic (flat) address of stream position 0 as seen through the LDS tile:
// base + offset for any offset inside [t0, t1) lands in the tile (computed
// in 64-bit integers, as the element stage of write_tile does).
__device__ __forceinline__ const uint8_t* xc_tile_base(const uint8_t* wire, const XcTile& t) {
  const uintptr_t g = (uintptr_t)(const void*)wire;
  return (const uint8_t*)(g - (uintptr_t)(t.t0 - t.sh));
}

__host__ __device__ __forceinline__ uint32_t xc_rec_region(uint32_t S, uint32_t kRS) {
  return kRS ? 0u : (kPT * S + 16 + 15) & ~15u;
}

template <class PS, class PD, uint32_t kRS>
__device__ __forceinline__ void xc_size_tile(const XcodeArgs& x, const PS& Ps, const PD& Pd,
                                             uint32_t S, uint32_t wire_cap, uint8_t* smem,
                                             unsigned long long* part) {
  const DecodeArgs& a = x.d;
  if ((uint64_t)blockIdx.x * kPT >= a.n) return;
  uint8_t* wire = smem;
  uint8_t* rtile = smem + decode_wire_region(wire_cap);
  const XcTile t = xc_stage(a, wire_cap, wire);
  __syncthreads();
  const bool stage_lists = Ps.has_lists() && Ps.protocol() == TGPU_PROTOCOL_BINARY && t.ok;
  const uint8_t* lb = stage_lists ? xc_tile_base(wire, t) : a.arena;
  const uint32_t r = threadIdx.x;
  unsigned long long sz = 0;
  alignas(8) uint8_t rbuf[kRS ? kRS : 8];
  if (r < t.nrec) {
    uint8_t* rec = kRS ? rbuf : rtile + r * S;
    if (xc_decode<PS, kRS>(a, Ps, t, wire, stage_lists, rec, S)) {
      bool ok = true;
      sz = program_size(Pd, PtrRec{rec}, lb, ok);
      if (!ok) atomicMin(&x.e.res->first_fail, (unsigned long long)(t.r0 + r));
    } else {
      const unsigned long long k = atomicAdd(x.nirr, 1ull);
      x.irr[k] = t.r0 + r;
    }
  }
  unsigned long long total;
  (void)block_exscan256(sz, part, &total);
  if (threadIdx.x == 0) x.e.block_sums[blockIdx.x] = total;
}

// Single pass (round 5): tile j publishes its output bytes (AGG) as soon as
// its records are sized, then wave 0 looks back over the predecessors' words
// — 64 per round trip, summing AGG totals down to the first INCL (a tile
// whose inclusive prefix is known) — and publishes its own INCL. The status
// words are single 64-bit relaxed agent-scope atomics (op_ld / op_st: no
// fences, the single-pass index's lesson, tgpu_prog_kernels.h); workgroups
// are dispatched in index order, so every predecessor is resident or done
// and each wait is bounded (kOpSpinCap) all the same: a tile past the bound
// publishes FAIL, which every later tile inherits.
//   xstat[j]: 0 not yet | 01 AGG total | 10 INCL prefix | 11 FAIL (bits 63:62)
constexpr uint64_t kXcAgg = 1ull << 62, kXcIncl = 2ull << 62, kXcFail = 3ull << 62;
constexpr uint64_t kXcVal = (1ull << 62) - 1;

// Wave 0 (all 64 lanes): tile j's exclusive output prefix; false when a
// predecessor failed or a wait passed its bound.
__device__ __forceinline__ bool xc_look_back(unsigned long long* stat, uint64_t j,
                                             uint64_t& prefix) {
  const uint32_t l = threadIdx.x;
  uint64_t sum = 0;
  for (int64_t top = (int64_t)j - 1; top >= 0; top -= 64) {
    const int64_t k = top - (int64_t)l;
    uint64_t w = k >= 0 ? op_ld(stat + k) : kXcIncl;  // (below tile 0: prefix 0)
    for (uint32_t spin = 0; __any(w == 0); ++spin) {
      if (spin >= kOpSpinCap) return false;
      __builtin_amdgcn_s_sleep(1);
      if (w == 0) w = op_ld(stat + k);
    }
    const uint64_t fin = __ballot(w >= kXcIncl);  // INCL or FAIL
    const uint32_t stop = fin ? (uint32_t)__builtin_ctzll(fin) : 64u;
    if (stop < 64 && __shfl(w, (int)stop, 64) == kXcFail) return false;
    uint64_t v = l <= stop ? (w & kXcVal) : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    sum += v;
    if (fin) break;
  }
  prefix = sum;
  return true;
}

// The emit pass, two forms.
// kOne = false, the two-pass write pass: records the size pass listed keep a
//   hole of the size the general writer measured (x.e.offs[r],
//   k_transcode.hip) and their output start in x.e.offs[r]; the general
//   writer fills the hole afterwards. Behind a single pass (x.gate set) it
//   runs only when that pass left work (a listed record or a failed wait).
// kOne = true, the single pass: decode, size, look back, emit; a record the
//   program cannot take is listed and opens the gate (the two-pass kernels
//   then redo the call from the tile sums left in e.block_sums).
template <class PS, class PD, uint32_t kRS, bool kOne>
__device__ __forceinline__ void xc_emit_tile(const XcodeArgs& x, const PS& Ps, const PD& Pd,
                                             uint32_t S, uint32_t wire_cap, uint32_t ocap,
                                             uint8_t* smem, EncodeShared& sm) {
  const DecodeArgs& a = x.d;
  const EncodeArgs& e = x.e;
  if ((uint64_t)blockIdx.x * kPT >= a.n) return;
  if constexpr (!kOne) {
    if (x.gate && *x.gate == 0) return;
  }
  uint8_t* wire = smem;
  uint8_t* rtile = smem + decode_wire_region(wire_cap);
  uint8_t* otile = rtile + xc_rec_region(S, kRS);
  const XcTile t = xc_stage(a, wire_cap, wire);
  __syncthreads();
  const bool stage_lists = Ps.has_lists() && Ps.protocol() == TGPU_PROTOCOL_BINARY && t.ok;
  const uint8_t* sb = xc_tile_base(wire, t);
  const uint8_t* lb = stage_lists ? sb : a.arena;
  const uint32_t r = threadIdx.x;
  alignas(8) uint8_t rbuf[kRS ? kRS : 8];
  uint8_t* rec = kRS ? rbuf : rtile + r * S;
  bool ok = false;
  unsigned long long sz = 0;
  if (r < t.nrec) {
    ok = xc_decode<PS, kRS>(a, Ps, t, wire, stage_lists, rec, S);
    if (ok) {
      bool v = true;
      sz = program_size(Pd, PtrRec{rec}, lb, v);
      if (kOne && !v) atomicMin(&e.res->first_fail, (unsigned long long)(t.r0 + r));
    } else if constexpr (kOne) {
      const unsigned long long k = atomicAdd(x.nirr, 1ull);
      x.irr[k] = t.r0 + r;
      op_st(x.xstat + ((a.n + kPT - 1) / kPT), 1);  // the gate
    } else {
      sz = e.offs[t.r0 + r];  // the general writer's size (0: not written)
    }
  }
  unsigned long long tile_total;
  const unsigned long long rel = block_exscan256(sz, sm.part, &tile_total);
  unsigned long long tile_base;
  if constexpr (kOne) {
    const uint64_t j = blockIdx.x;
    if (threadIdx.x == 0) {
      e.block_sums[j] = tile_total;  // (the two-pass kernels' input if the gate opens)
      op_st(x.xstat + j, (j == 0 ? kXcIncl : kXcAgg) | tile_total);
      if (j == 0) sm.base = 0;
    }
    if (j > 0 && threadIdx.x < 64) {
      uint64_t p = 0;
      const bool got = xc_look_back(x.xstat, j, p);
      if (threadIdx.x == 0) {
        op_st(x.xstat + j, got ? kXcIncl | (p + tile_total) : kXcFail);
        if (!got) op_st(x.xstat + ((a.n + kPT - 1) / kPT), 1);
        sm.base = got ? p : kNo;
      }
    }
    __syncthreads();
    tile_base = sm.base;
    if (tile_base == kNo) return;  // (the gate is open: the two passes redo the call)
  } else {
    tile_base = e.block_sums[blockIdx.x];
  }
  uint8_t* gtile = e.out + tile_base;
  const uint32_t osh = (uint32_t)((uintptr_t)gtile & 15);
  {
    const uint4 z = {0u, 0u, 0u, 0u};
    const uint32_t nz = (osh + (uint32_t)min(tile_total, (unsigned long long)ocap) + 4 + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nz; i += kPT) ((uint4*)otile)[i] = z;
  }
  if (r == 0) sm.lds_end = (unsigned int)min(tile_total, (unsigned long long)ocap);
  __syncthreads();
  bool fits = false;
  if (r < t.nrec && (ok || !kOne)) {
    const unsigned long long start = tile_base + rel;
    const bool over = start + sz > e.cap;
    // (every start when the caller asked for offsets; else the listed
    // records' and an overflowing one's, which the general writer and the
    // finish read)
    if (x.want_offs || !ok || over) e.offs[t.r0 + r] = start;
    if (over) {
      atomicMin(&e.res->first_fail, (unsigned long long)(t.r0 + r));
      atomicMin(&sm.lds_end, (unsigned int)min(rel, (unsigned long long)ocap));
    } else {
      fits = rel + sz <= ocap;
      if (!fits) atomicMin(&sm.lds_end, (unsigned int)rel);
    }
  }
  __syncthreads();
  if (r < t.nrec && ok) {
    if (fits && rel + sz <= sm.lds_end) {
      OrSink w((uint32_t*)otile, osh + (uint32_t)rel);
      program_emit(Pd, PtrRec{rec}, sb, lb, w);
    } else if (tile_base + rel + sz <= e.cap) {
      ByteSink w(gtile + rel);
      program_emit(Pd, PtrRec{rec}, sb, lb, w);
    }
  }
  __syncthreads();
  const uint32_t end = osh + sm.lds_end;
  const uint32_t nvec = (end + 15) >> 4;
  uint8_t* gb = gtile - osh;
  for (uint32_t i = threadIdx.x; i < nvec; i += kPT) {
    const uint32_t lo = i << 4, hi = lo + 16;
    if (lo >= osh && hi <= end) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(((const u32x4*)otile)[i], (u32x4*)gb + i);
    } else {
      for (uint32_t b = (lo < osh ? osh : lo); b < (hi < end ? hi : end); ++b) gb[b] = otile[b];
    }
  }
}

template <class PS, class PD, uint32_t kRS>
__device__ __forceinline__ void xc_write_tile(const XcodeArgs& x, const PS& Ps, const PD& Pd,
                                              uint32_t S, uint32_t wire_cap, uint32_t ocap,
                                              uint8_t* smem, EncodeShared& sm) {
  xc_emit_tile<PS, PD, kRS, false>(x, Ps, Pd, S, wire_cap, ocap, smem, sm);
}

template <class PS, class PD, uint32_t kRS>
__device__ __forceinline__ void xc_one_tile(const XcodeArgs& x, const PS& Ps, const PD& Pd,
                                            uint32_t S, uint32_t wire_cap, uint32_t ocap,
                                            uint8_t* smem, EncodeShared& sm) {
  xc_emit_tile<PS, PD, kRS, true>(x, Ps, Pd, S, wire_cap, ocap, smem, sm);
}

}  // namespace prog
}  // namespace tgpu
