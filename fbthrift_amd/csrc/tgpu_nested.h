// tgpu_nested.h — the compiled decode of nested programs: records whose
// lists / sets hold structs or scalar lists (list<Item>, list<list<i32>>),
// the schemas the general reader's frame machine (tgpu_device.h read_record)
// takes otherwise. Not part of the public ABI.
//
// The schema compiler (tgpu_jit.cpp gen_nested_source) writes the record's
// canonical form out as straight-line code with one counted loop per
// container level: every header byte, width and member offset a constant,
// no frames. A lane decodes one record of its workgroup's LDS wire tile; the
// containers take their element arrays from the record's arena region in
// wire order, exactly as the general reader allocates them (Arena::alloc,
// record regions: scale x the record's start, 8-byte aligned bumps), so the
// records, spans and arena bytes are the general reader's. A record that
// leaves the canonical form in any way is queued for the general decoder,
// which decides it with the full readNoXfer semantics
// (protocol_methods.h:358-503 for the containers).
#pragma once

#include "tgpu_prog_kernels.h"

namespace tgpu {
namespace prog {

// Arena::alloc of the record regions (tgpu_device.h)
__device__ __forceinline__ uint64_t region_alloc(uint64_t& bump, uint64_t bytes) {
  const uint64_t o = bump;
  bump = (bump + bytes + 7) & ~7ull;
  return o;
}

// A list / set header whose elements must be op.elem_ttype (Binary: type
// byte + BE i32; Compact: size nibble + ctype, size 15 -> varint;
// BinaryProtocol-inl.h:526-540, CompactProtocol-inl.h:692-715) and the
// count checks of check_container / the truncation check (n <= bytes left).
template <class Src>
__device__ __forceinline__ bool seq_header(const VOp op, const bool compact, const Src& src,
                                           const Ctx& c, uint32_t& p, const uint32_t end,
                                           int64_t& n) {
  if (compact) {
    if (p + 1 > end) return false;
    const uint32_t b = (uint32_t)(src.win8(p) & 0xff);
    const uint32_t ct = b & 0xf;
    const bool ok_ct = op.elem_ttype == TGPU_T_BOOL ? (ct == 1 || ct == 2) : ct == op.elem_ct;
    if (!ok_ct) return false;
    ++p;
    n = b >> 4;
    if (n == 15) {
      uint64_t z;
      if (!read_varint(src, p, end, 32, z)) return false;
      n = (int32_t)(uint32_t)z;
    }
  } else {
    if (p + 5 > end) return false;
    const uint64_t w = src.win8(p);
    if ((w & 0xff) != op.elem_ttype) return false;
    n = (int32_t)(uint32_t)bswap_n(w >> 8, 4);
    p += 5;
  }
  return n >= 0 && !(c.container_limit && n > c.container_limit) && n <= (int64_t)(end - p);
}

// VOP_SEQ: the container's element array (n x op.hdr bytes) from the region
// and its span at base + member; the caller loops over the elements.
template <class Src>
__device__ __forceinline__ bool seq_open(const VOp op, const bool compact, const Src& src,
                                         const Ctx& c, uint32_t& p, const uint32_t end,
                                         uint8_t* base, uint64_t& bump, uint32_t& n_out,
                                         uint8_t*& arr) {
  int64_t n;
  if (!seq_header(op, compact, src, c, p, end, n)) return false;
  tgpu_span* sp = (tgpu_span*)(base + op.member);
  n_out = (uint32_t)n;
  arr = nullptr;
  if (n == 0) {
    *sp = tgpu_span{0, 0, 0};
    return true;
  }
  const uint64_t bytes = (uint64_t)n * op.hdr;
  if (!c.arena) return false;
  const uint64_t aoff = region_alloc(bump, bytes);
  if (aoff + bytes > c.arena_cap) return false;
  arr = c.arena + aoff;
  *sp = tgpu_span{aoff, (uint32_t)n, 0};
  return true;
}

__device__ __forceinline__ void seq_close(const VOp op, uint8_t* base) {
  if (op.isset != 0xffff) base[op.isset] = 1;
}

// A default-constructed struct element (the general reader zeroes the slot
// before reading into it); ES is a compile-time constant.
template <uint32_t ES>
__device__ __forceinline__ void zero_slot(uint8_t* el) {
  if constexpr (ES % 8 == 0) {
#pragma unroll
    for (uint32_t b = 0; b < ES; b += 8) *(uint64_t*)(el + b) = 0;
  } else if constexpr (ES % 4 == 0) {
#pragma unroll
    for (uint32_t b = 0; b < ES; b += 4) *(uint32_t*)(el + b) = 0;
  } else {
#pragma unroll
    for (uint32_t b = 0; b < ES; ++b) el[b] = 0;
  }
}

// VOP_LIST of a nested program: scalar elements into the region (read_list,
// tgpu_device.h: allocated only when n > 0), span at base + member.
template <class Src>
__device__ __forceinline__ bool nlist(const VOp op, const bool compact, const Src& src,
                                      const Ctx& c, uint32_t& p, const uint32_t end,
                                      uint8_t* base, uint64_t& bump) {
  int64_t n;
  if (!seq_header(op, compact, src, c, p, end, n)) return false;
  const uint32_t es = op.width;
  uint64_t aoff = 0;
  if (n) {
    if (!c.arena) return false;
    aoff = region_alloc(bump, (uint64_t)n * es);
    if (aoff + (uint64_t)n * es > c.arena_cap) return false;
  }
  uint8_t* dst = c.arena + aoff;
  for (int64_t i = 0; i < n; ++i) {
    uint64_t v;
    if (op.elem_kind == VEL_VARINT) {
      uint64_t z;
      if (!read_varint(src, p, end, op.bits, z)) return false;
      v = unzigzag(z, op.bits);
    } else {
      const uint32_t wb = op.elem_kind == VEL_BOOL ? 1 : es;
      if (p + wb > end) return false;
      v = bswap_n(src.win8(p), wb);
      if (op.elem_kind == VEL_BOOL) {
        if (compact) v = v == 1;
        else if (v > 1) return false;
      }
      p += wb;
    }
    store_n(dst + (uint64_t)i * es, v, es);
  }
  *(tgpu_span*)(base + op.member) = tgpu_span{n ? aoff : 0, (uint32_t)n, 0};
  if (op.isset != 0xffff) base[op.isset] = 1;
  return true;
}

// One 256-record tile of an indexed stream: decode_tile's staging (wire bytes
// HBM -> LDS by LDS DMA, records built in an LDS record tile that leaves with
// 16-byte stores), each lane running the generated record function
//   bool R(const LdsSrc&, const Ctx&, uint32_t& p, uint32_t end, uint8_t* rec,
//          uint64_t& bump)
// with its region start in `bump`. Element arrays go straight to the arena.
template <class R>
__device__ __forceinline__ void nested_decode_tile(const DecodeArgs& a, const R& run, uint32_t S,
                                                   uint32_t wire_cap, uint64_t* __restrict__ irr,
                                                   unsigned long long* __restrict__ nirr,
                                                   uint8_t* smem) {
  uint8_t* wire = smem;
  uint8_t* rtile = smem + decode_wire_region(wire_cap);
  const uint64_t r0 = (uint64_t)blockIdx.x * kPT;
  const uint64_t n_all = a.n_dev ? min(a.n, (uint64_t)*a.n_dev) : a.n;
  if (r0 >= n_all) return;  // (whole workgroup)
  const uint32_t nrec = (uint32_t)min((uint64_t)kPT, n_all - r0);
  const uint64_t t0 = a.offs[r0], t1 = a.offs[r0 + nrec];
  const bool tile_ok = t1 >= t0 && t1 <= a.in_len && (t1 - t0) + 16 <= wire_cap;
  uint32_t sh = 0;
  if (tile_ok) {
    const uint8_t* g = a.in + t0;
    sh = (uint32_t)((uintptr_t)g & 15);
    const uint4* src = (const uint4*)(g - sh);
    const uint32_t nvec = (uint32_t)((t1 - t0) + sh + 15) >> 4;
    const uint32_t wave = threadIdx.x >> 6;
    for (uint32_t k = 0; k * kPT < nvec; ++k) {
      const uint32_t i = k * kPT + threadIdx.x;
      __builtin_amdgcn_global_load_lds(
          (const void*)(src + (i < nvec ? i : nvec - 1)),
          (__attribute__((address_space(3))) void*)(wire + (size_t)(k * kPT + wave * 64) * 16), 16,
          0, 0);
    }
    lds_dma_settle(wire, threadIdx.x, kPT, (nvec + kPT - 1) / kPT);
  }
  uint8_t* gout = a.recs + r0 * S;
  const uint32_t osh = (uint32_t)((uintptr_t)gout & 15);
  {
    const uint4 z = {0u, 0u, 0u, 0u};
    const uint32_t nz = (kPT * S + osh + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nz; i += kPT) ((uint4*)rtile)[i] = z;
  }
  __syncthreads();
  const uint32_t r = threadIdx.x;
  if (r < nrec) {
    uint8_t* rec = rtile + osh + r * S;
    bool ok = tile_ok;
    if (ok) {
      const uint64_t s = a.offs[r0 + r], e = a.offs[r0 + r + 1];
      ok = s >= t0 && e >= s && e <= t1;
      if (ok) {
        const Ctx c{t0 - sh, a.arena, a.arena_cap, a.string_limit, a.container_limit, nullptr};
        const LdsSrc src{(const uint32_t*)wire};
        uint32_t p = (uint32_t)(s - t0) + sh;
        const uint32_t pe = (uint32_t)(e - t0) + sh;
        uint64_t bump = (uint64_t)a.sc.bump_scale * s;  // record_arena: the record's region
        ok = run(src, c, p, pe, rec, bump) && p == pe;
      }
    }
    if (!ok) irr[atomicAdd(nirr, 1ull)] = r0 + r;  // the general decoder's list
  }
  __syncthreads();
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

// The same without staging (A/B, TGPU_NESTED_SRC=hbm): one lane per record,
// reading its bytes from HBM through 8-byte windows (HbmSrc) and writing the
// record in place — no LDS, so occupancy is set by registers alone.
template <class R>
__device__ __forceinline__ void nested_decode_hbm(const DecodeArgs& a, const R& run, uint32_t S,
                                                  uint64_t* __restrict__ irr,
                                                  unsigned long long* __restrict__ nirr) {
  const uint64_t i = (uint64_t)blockIdx.x * kPT + threadIdx.x;
  const uint64_t n_all = a.n_dev ? min(a.n, (uint64_t)*a.n_dev) : a.n;
  if (i >= n_all) return;
  uint8_t* rec = a.recs + i * S;
  if ((S & 7) == 0 && ((uintptr_t)rec & 7) == 0) {
    for (uint32_t b = 0; b < S; b += 8) *(uint64_t*)(rec + b) = 0;
  } else {
    for (uint32_t b = 0; b < S; ++b) rec[b] = 0;
  }
  const uint64_t s = a.offs[i], e = a.offs[i + 1];
  bool ok = e >= s && e <= a.in_len && e - s < (1ull << 31);
  if (ok) {
    const Ctx c{s, a.arena, a.arena_cap, a.string_limit, a.container_limit, nullptr};
    const HbmSrc src{a.in + s, (uint32_t)min(a.in_len - s, (uint64_t)0xffffffffu)};
    uint32_t p = 0;
    const uint32_t pe = (uint32_t)(e - s);
    uint64_t bump = (uint64_t)a.sc.bump_scale * s;
    ok = run(src, c, p, pe, rec, bump) && p == pe;
  }
  if (!ok) irr[atomicAdd(nirr, 1ull)] = i;
}

}  // namespace prog
}  // namespace tgpu
