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

// ---- field headers of the nested programs -----------------------------------
// Binary: type byte + BE i16 id (BinaryProtocol-inl.h:53-59).
template <class Src>
__device__ __forceinline__ bool bfield(const Src& src, uint32_t& p, const uint32_t end,
                                       uint32_t hdr) {
  if (p + 3 > end || (src.win8(p) & 0xffffff) != hdr) return false;
  p += 3;
  return true;
}

// Compact (CompactProtocol-inl.h:133-160): the header the writer emits for
// field `id` after field `last`: one byte (delta << 4 | ctype) when
// 0 < delta <= 15, else ctype + zigzag varint id. ct 0: a bool field, the
// byte's ctype 1 / 2 is its value (*val). On a match the header is
// consumed and last = id.
__device__ __forceinline__ void chdr_bytes(int32_t id, uint32_t ct, int32_t last, uint64_t& hb,
                                           uint32_t& len) {
  const int32_t d = id - last;
  if (d > 0 && d <= 15) {
    hb = ((uint32_t)d << 4) | ct;
    len = 1;
    return;
  }
  uint32_t zz = ((uint32_t)id << 1) ^ (uint32_t)(id >> 31);
  hb = ct;
  len = 1;
  do {
    hb |= (uint64_t)((zz & 0x7f) | (zz > 0x7f ? 0x80 : 0)) << (8 * len++);
    zz >>= 7;
  } while (zz);
}
template <class Src>
__device__ __forceinline__ bool cfield(const Src& src, uint32_t& p, const uint32_t end, int32_t id,
                                       uint32_t ct, int32_t& last) {
  uint64_t hb;
  uint32_t len;
  chdr_bytes(id, ct, last, hb, len);
  const uint64_t m = (1ull << (8 * len)) - 1;
  if (p + len > end || (src.win8(p) & m) != hb) return false;
  p += len;
  last = id;
  return true;
}
template <bool kStore = true, class Src>
__device__ __forceinline__ bool cbool_field(const Src& src, uint32_t& p, const uint32_t end,
                                            int32_t id, int32_t& last, uint8_t* member,
                                            uint8_t* isset) {
  uint64_t hb;
  uint32_t len;
  chdr_bytes(id, 0, last, hb, len);
  const uint64_t m = (1ull << (8 * len)) - 1;
  if (p + len > end) return false;
  const uint64_t w = src.win8(p) & m;
  const uint32_t ct = (uint32_t)(w & 0xf);
  if ((w & ~0xfull) != hb || (ct != 1 && ct != 2)) return false;
  if (kStore) {
    *member = ct == 1 ? 1 : 0;
    *isset = 1;
  }
  p += len;
  last = id;
  return true;
}
template <class Src>
__device__ __forceinline__ bool struct_stop(const Src& src, uint32_t& p, const uint32_t end) {
  if (p + 1 > end || (src.win8(p) & 0xff) != 0) return false;
  ++p;
  return true;
}

// VOP_SEQ: the container's element array (n x op.hdr bytes) from the region
// and its span at base + member; the caller loops over the elements.
// kStore false: measuring only (the stream index), nothing allocated or written
template <bool kStore = true, class Src>
__device__ __forceinline__ bool seq_open(const VOp op, const bool compact, const Src& src,
                                         const Ctx& c, uint32_t& p, const uint32_t end,
                                         uint8_t* base, uint64_t& bump, uint32_t& n_out,
                                         uint8_t*& arr) {
  int64_t n;
  if (!seq_header(op, compact, src, c, p, end, n)) return false;
  n_out = (uint32_t)n;
  arr = nullptr;
  if (!kStore) return true;
  tgpu_span* sp = (tgpu_span*)(base + op.member);
  if (n == 0) {
    *sp = tgpu_span{0, 0, 0};
    return true;
  }
  const uint64_t bytes = (uint64_t)n * op.hdr;
  if (!c.arena || c.pos_scale) return false;
  const uint64_t aoff = region_alloc(bump, bytes);
  if (aoff + bytes > c.arena_cap) return false;
  arr = c.arena + aoff;
  *sp = tgpu_span{aoff, (uint32_t)n, 0};
  return true;
}

__device__ __forceinline__ void seq_close(const VOp op, uint8_t* base) {
  if (op.isset != 0xffff) base[op.isset] = 1;
}

// VOP_MSEQ: a map header (Binary: key type, value type, BE i32; Compact:
// varint size, then the key/value ctype byte when size > 0;
// BinaryProtocol-inl.h:506-524, CompactProtocol-inl.h:662-690), the
// truncation check of two bytes a pair, the pairs from the region.
template <bool kStore = true, class Src>
__device__ __forceinline__ bool mseq_open(const VOp op, const bool compact, const Src& src,
                                          const Ctx& c, uint32_t& p, const uint32_t end,
                                          uint8_t* base, uint64_t& bump, uint32_t& n_out,
                                          uint8_t*& arr) {
  int64_t n;
  if (compact) {
    uint64_t z;
    if (!read_varint(src, p, end, 32, z)) return false;
    n = (int32_t)(uint32_t)z;
    if (n > 0) {
      if (p + 1 > end || (src.win8(p) & 0xff) != op.elem_ct) return false;
      ++p;
    }
  } else {
    if (p + 6 > end) return false;
    const uint64_t w = src.win8(p);
    if ((w & 0xff) != op.width || ((w >> 8) & 0xff) != op.elem_ttype) return false;
    n = (int32_t)(uint32_t)bswap_n(w >> 16, 4);
    p += 6;
  }
  if (n < 0 || (c.container_limit && n > c.container_limit) || 2 * n > (int64_t)(end - p))
    return false;
  n_out = (uint32_t)n;
  arr = nullptr;
  if (!kStore) return true;
  tgpu_span* sp = (tgpu_span*)(base + op.member);
  if (n == 0) {
    *sp = tgpu_span{0, 0, 0};
    return true;
  }
  const uint64_t bytes = (uint64_t)n * op.hdr;
  if (!c.arena || c.pos_scale) return false;
  const uint64_t aoff = region_alloc(bump, bytes);
  if (aoff + bytes > c.arena_cap) return false;
  arr = c.arena + aoff;
  *sp = tgpu_span{aoff, (uint32_t)n, 0};
  return true;
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

// VOP_BOX: a boxed struct field's object (SZ bytes) from the record's region
// (Arena::alloc at the struct's start, as the general reader allocates it),
// default-constructed; the caller reads it, then points the member to it.
template <uint32_t SZ>
__device__ __forceinline__ bool box_open(const Ctx& c, uint64_t& bump, uint64_t& aoff,
                                         uint8_t*& obj) {
  if (!c.arena || c.pos_scale) return false;
  aoff = region_alloc(bump, SZ);
  if (aoff + SZ > c.arena_cap) return false;
  obj = c.arena + aoff;
  zero_slot<SZ>(obj);
  return true;
}

// A struct slot built in registers (ES % 8 == 0) to its arena place.
template <uint32_t ES>
__device__ __forceinline__ void copy_slot(uint8_t* dst, const uint8_t* src) {
#pragma unroll
  for (uint32_t b = 0; b < ES; b += 8) *(uint64_t*)(dst + b) = *(const uint64_t*)(src + b);
}

// A struct slot (ES % 8 == 0) of an encoder's list base into registers: the
// slot's loads issued together instead of one dependent load per member
// (8-byte loads when the slot is 8-byte aligned, else 4-byte ones).
template <uint32_t ES>
__device__ __forceinline__ void load_slot(uint8_t* dst, const uint8_t* src) {
  if (((uintptr_t)src & 7) == 0) {
#pragma unroll
    for (uint32_t b = 0; b < ES; b += 8) *(uint64_t*)(dst + b) = *(const uint64_t*)(src + b);
  } else {
#pragma unroll
    for (uint32_t b = 0; b < ES; b += 4) *(uint32_t*)(dst + b) = *(const uint32_t*)(src + b);
  }
}

// VOP_LIST of a nested program: scalar elements into the region (read_list,
// tgpu_device.h: allocated only when n > 0), span at base + member.
template <bool kStore = true, class Src>
__device__ __forceinline__ bool nlist(const VOp op, const bool compact, const Src& src,
                                      const Ctx& c, uint32_t& p, const uint32_t end,
                                      uint8_t* base, uint64_t& bump) {
  int64_t n;
  if (!seq_header(op, compact, src, c, p, end, n)) return false;
  const uint32_t es = op.width;
  uint64_t aoff = 0;
  if (!kStore && op.elem_kind == VEL_FIXED) {  // measuring: fixed-width elements skipped
    if ((uint64_t)n * es > end - p) return false;
    p += (uint32_t)n * es;
    return true;
  }
  if (kStore && n) {
    if (!c.arena) return false;
    // the record's region, or the position rule (schemas without regions)
    aoff = c.pos_scale ? c.pos_scale * (c.gbase + p) : region_alloc(bump, (uint64_t)n * es);
    if (aoff + (uint64_t)n * es > c.arena_cap) return false;
  }
  uint8_t* dst = c.arena + aoff;
#ifndef TGPU_NLIST_SINGLE  // A/B (TGPU_JIT_DEFINES): one element per window
  if (kStore && !compact && op.elem_kind == VEL_FIXED && es == 4 && !c.pos_scale) {
    // Binary 4-byte elements two at a time: one window, one 8-byte store
    // (region arrays are 8-byte aligned)
    if ((uint64_t)n * 4 > end - p) return false;
    int64_t i = 0;
    for (; i + 1 < n; i += 2) {
      const uint64_t w = src.win8(p);
      const uint64_t v = (uint64_t)__builtin_bswap32((uint32_t)w) |
                         ((uint64_t)__builtin_bswap32((uint32_t)(w >> 32)) << 32);
      *(uint64_t*)(dst + (uint64_t)i * 4) = v;
      p += 8;
    }
    if (i < n) {
      *(uint32_t*)(dst + (uint64_t)i * 4) = __builtin_bswap32((uint32_t)src.win8(p));
      p += 4;
    }
    *(tgpu_span*)(base + op.member) = tgpu_span{n ? aoff : 0, (uint32_t)n, 0};
    if (op.isset != 0xffff) base[op.isset] = 1;
    return true;
  }
#endif
  for (int64_t i = 0; i < n; ++i) {
    uint64_t v;
    if (op.elem_kind == VEL_STRING) {  // read_elem: a view into the stream
      int64_t len;
      if (compact) {
        uint64_t z;
        if (!read_varint(src, p, end, 32, z)) return false;
        len = (int32_t)(uint32_t)z;
      } else {
        if (p + 4 > end) return false;
        len = (int32_t)(uint32_t)bswap_n(src.win8(p), 4);
        p += 4;
      }
      if (len < 0 || (c.string_limit > 0 && len > c.string_limit) || len > (int64_t)(end - p))
        return false;
      if (kStore)
        *(tgpu_span*)(dst + (uint64_t)i * es) = tgpu_span{len ? c.gbase + p : 0, (uint32_t)len, 0};
      p += (uint32_t)len;
      continue;
    }
    if (op.elem_kind == VEL_VARINT) {
      uint64_t z;
      if (!read_varint(src, p, end, op.bits, z)) return false;
      v = unzigzag(z, op.bits);
    } else {
      const uint32_t wb = op.elem_kind == VEL_BOOL ? 1 : es;
      if (p + wb > end) return false;
      v = fixed_n(src.win8(p), wb, op.elem_kind == VEL_FIXED && op.bits == kFixedLE);
      if (op.elem_kind == VEL_BOOL) {
        if (compact) v = v == 1;
        else if (v > 1) return false;
      }
      p += wb;
    }
    if (kStore) store_n(dst + (uint64_t)i * es, v, es);
  }
  if (kStore) {
    *(tgpu_span*)(base + op.member) = tgpu_span{n ? aoff : 0, (uint32_t)n, 0};
    if (op.isset != 0xffff) base[op.isset] = 1;
  }
  return true;
}

// The stream index's view of the LDS tile for a measuring walk
// (measure_lds): reads past lim are clamped and mark the walk undecided.
struct ClampSrc {
  const uint32_t* w32;
  uint32_t lim;
  bool* slow;
  __device__ __forceinline__ uint64_t win8(uint32_t p) const {
    if (p > lim) {
      *slow = true;
      p = lim;
    }
    return LdsSrc{w32}.win8(p);
  }
};

// One 256-record tile of an indexed stream: decode_tile's staging (wire bytes
// HBM -> LDS by LDS DMA, records built in an LDS record tile that leaves with
// 16-byte stores), each lane running the generated record function
//   bool R(const LdsSrc&, const Ctx&, uint32_t& p, uint32_t end, uint8_t* rec,
//          uint64_t& bump)
// with its region start in `bump`. Element arrays go straight to the arena.
// tgpu_schema_arena_scale of a schema without record regions (0: regions)
__device__ __forceinline__ uint64_t pos_scale(const DevSchema& sc, bool compact) {
  if (sc.bump_scale) return 0;
  return sc.str_elems ? (compact ? 16 : 4) : (compact ? 8 : 1);
}

// kRTile false (A/B, TGPU_NESTED_RTILE=0): no LDS record tile — each lane
// zeroes and fills its record in HBM, the workgroup's LDS is the wire tile.
template <bool kRTile = true, class R>
__device__ __forceinline__ void nested_decode_tile(const DecodeArgs& a, const R& run, uint32_t S,
                                                   bool compact,
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
  if (kRTile) {
    const uint4 z = {0u, 0u, 0u, 0u};
    const uint32_t nz = (kPT * S + osh + 15) >> 4;
    for (uint32_t i = threadIdx.x; i < nz; i += kPT) ((uint4*)rtile)[i] = z;
  }
  __syncthreads();
  const uint32_t r = threadIdx.x;
  if (r < nrec) {
    uint8_t* rec = kRTile ? rtile + osh + r * S : gout + (uint64_t)r * S;
    if (!kRTile) {
      if ((S & 7) == 0 && ((uintptr_t)rec & 7) == 0) {
        for (uint32_t b = 0; b < S; b += 8) *(uint64_t*)(rec + b) = 0;
      } else {
        for (uint32_t b = 0; b < S; ++b) rec[b] = 0;
      }
    }
    bool ok = tile_ok;
    if (ok) {
      const uint64_t s = a.offs[r0 + r], e = a.offs[r0 + r + 1];
      ok = s >= t0 && e >= s && e <= t1;
      if (ok) {
        const Ctx c{t0 - sh, a.arena, a.arena_cap, a.string_limit, a.container_limit, nullptr,
                    pos_scale(a.sc, compact)};
        const LdsSrc src{(const uint32_t*)wire};
        uint32_t p = (uint32_t)(s - t0) + sh;
        const uint32_t pe = (uint32_t)(e - t0) + sh;
        uint64_t bump = (uint64_t)a.sc.bump_scale * s;  // record_arena: the record's region
        ok = run(src, c, p, pe, rec, bump) && p == pe;
      }
    }
    if (!ok) irr[atomicAdd(nirr, 1ull)] = r0 + r;  // the general decoder's list
  }
  if (!kRTile) return;
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
                                                  bool compact,
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
    const Ctx c{s, a.arena, a.arena_cap, a.string_limit, a.container_limit, nullptr,
                pos_scale(a.sc, compact)};
    const HbmSrc src{a.in + s, (uint32_t)min(a.in_len - s, (uint64_t)0xffffffffu)};
    uint32_t p = 0;
    const uint32_t pe = (uint32_t)(e - s);
    uint64_t bump = (uint64_t)a.sc.bump_scale * s;
    ok = run(src, c, p, pe, rec, bump) && p == pe;
  }
  if (!ok) irr[atomicAdd(nirr, 1ull)] = i;
}

// ================================================================ encode ======
// The generated record writer runs twice: over Count (the size pass: bytes
// only) and over Out (the write pass). Either way the bytes are the general
// writer's (tgpu_device.h write_record: the generated write of every field in
// declaration order, serialize_struct.whisker:40-67), for records of the
// canonical kind these schemas have (every field unqualified / required): a
// value the writer rejects (a bool byte > 1, a length > INT32_MAX) fails the
// record, and the finish kernel diagnoses it with the general writer.
struct Count {
  static constexpr bool kCount = true;
  uint64_t n = 0;
  __device__ __forceinline__ void put(uint64_t, uint32_t k) { n += k; }
  __device__ __forceinline__ void bytes(const uint8_t*, uint32_t k) { n += k; }
};

// Bytes into HBM from an 8-byte accumulator: whole aligned words with one
// 8-byte store, the record's first and last partial words byte by byte (the
// neighbouring records own the rest of those words).
template <bool kLds>
struct OutT {
  static constexpr bool kCount = false;
  uint8_t* w;      // current aligned word
  uint64_t acc;    // its pending bytes (little-endian)
  uint32_t nb;     // bytes in acc (incl. the skipped head of the first word)
  uint32_t lo;     // first byte of the current word this record owns
  __device__ __forceinline__ OutT(uint8_t* out, uint64_t start) {
    const uintptr_t at = (uintptr_t)out + start;
    w = (uint8_t*)(at & ~(uintptr_t)7);
    nb = lo = (uint32_t)(at & 7);
    acc = 0;
  }
  __device__ __forceinline__ void emit(uint64_t x) {
    if (lo == 0) {
      *(uint64_t*)w = x;
    } else if constexpr (kLds) {  // a zero-filled LDS tile: OR in the bytes this record owns
      atomicOr((unsigned long long*)w, (unsigned long long)(x & (~0ull << (8 * lo))));
      lo = 0;
    } else {
      for (uint32_t b = lo; b < 8; ++b) w[b] = (uint8_t)(x >> (8 * b));
      lo = 0;
    }
    w += 8;
  }
  // the low k bytes of v (1 <= k <= 8), first byte lowest
  __device__ __forceinline__ void put(uint64_t v, uint32_t k) {
    if (k < 8) v &= (1ull << (8 * k)) - 1;
    acc |= v << (8 * nb);
    const uint32_t t = nb + k;
    if (t >= 8) {
      emit(acc);
      acc = nb ? v >> (8 * (8 - nb)) : 0;
      nb = t - 8;
    } else {
      nb = t;
    }
  }
  // k bytes from src (a string payload): 8 at a time from aligned loads (never
  // past the 8-byte words that hold src's bytes)
  __device__ __forceinline__ void bytes(const uint8_t* src, uint32_t k) {
    while (k) {
      const uint32_t m = k < 8 ? k : 8;
      const uintptr_t a = (uintptr_t)src;
      const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
      const uint32_t sh = (uint32_t)(a & 7);
      uint64_t x = q[0] >> (8 * sh);
      if (sh && sh + m > 8) x |= q[1] << (8 * (8 - sh));
      put(x, m);
      src += m;
      k -= m;
    }
  }
  __device__ __forceinline__ void flush() {
    if (nb <= lo) return;
    if constexpr (kLds) {
      const uint64_t m = (nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1)) & (~0ull << (8 * lo));
      atomicOr((unsigned long long*)w, (unsigned long long)(acc & m));
    } else {
      for (uint32_t b = lo; b < nb; ++b) w[b] = (uint8_t)(acc >> (8 * b));
    }
  }
};
using Out = OutT<false>;

__device__ __forceinline__ uint32_t lebn(uint64_t v) {  // LEB128 bytes of v
  const uint32_t bits = 64 - (uint32_t)__builtin_clzll(v | 1);
  return (bits + 6) / 7;
}

template <class O>
__device__ __forceinline__ void nput_varint(O& o, uint64_t v) {
  if constexpr (O::kCount) {
    o.n += lebn(v);
  } else {
    uint64_t x = 0;
    uint32_t n = 0;
    while (v >= 0x80 && n < 8) {
      x |= ((v & 0x7f) | 0x80) << (8 * n);
      v >>= 7;
      ++n;
    }
    if (n < 8) {
      o.put(x | (v << (8 * n)), n + 1);
      return;
    }
    o.put(x, 8);  // (a 9-10 byte i64 varint)
    x = 0;
    n = 0;
    while (v >= 0x80) {
      x |= ((v & 0x7f) | 0x80) << (8 * n);
      v >>= 7;
      ++n;
    }
    o.put(x | (v << (8 * n)), n + 1);
  }
}

// writeListBegin / writeSetBegin (BinaryProtocol-inl.h:69-96,
// CompactProtocol-inl.h:182-246) of n elements of op.elem_ttype
template <class O>
__device__ __forceinline__ bool put_list_header(O& o, const VOp op, const bool compact,
                                                uint32_t n) {
  if (n > 0x7fffffffu) return false;  // checked_container_size: WRITE_SIZE_LIMIT
  if (!compact) {
    o.put(op.elem_ttype, 1);
    o.put(__builtin_bswap32(n), 4);
  } else if (n <= 14) {
    o.put((n << 4) | op.elem_ct, 1);
  } else {
    o.put(0xf0 | op.elem_ct, 1);
    nput_varint(o, n);
  }
  return true;
}

// writeMapBegin (BinaryProtocol-inl.h:83-96, CompactProtocol-inl.h:219-246)
template <class O>
__device__ __forceinline__ bool put_map_header(O& o, const VOp op, const bool compact, uint32_t n) {
  if (n > 0x7fffffffu) return false;
  if (!compact) {
    o.put(op.width | ((uint32_t)op.elem_ttype << 8), 2);
    o.put(__builtin_bswap32(n), 4);
  } else if (n == 0) {
    o.put(0, 1);
  } else {
    nput_varint(o, n);
    o.put(op.elem_ct, 1);
  }
  return true;
}

// A fixed-width scalar of w bytes at p as the writer emits it
// (write_scalar): big-endian, a bool validated (0/1; Compact 1 / 2).
// (le: little-endian on the wire, kFixedLE — CompactV1 doubles)
template <class O>
__device__ __forceinline__ bool put_fixed(O& o, const bool compact, const uint8_t* p, uint32_t w,
                                          bool is_bool, bool le = false) {
  const uint64_t raw = load_member(p, w);
  if (is_bool) {
    if (raw > 1) return false;  // validate_bool: INVALID_BOOL_WRITE
    o.put(compact ? (raw ? 1 : 2) : raw, 1);
    return true;
  }
  o.put(le ? raw : __builtin_bswap64(raw) >> (64 - 8 * w), w);
  return true;
}

// One non-container op of the program (the ops run_op decodes).
template <class O>
__device__ __forceinline__ bool enc_op(const VOp op, const bool compact, const uint8_t* base,
                                       const uint8_t* sbase, const uint8_t* lbase, O& o) {
  switch (op.kind) {
    case VOP_CONST:
      o.put(op.hdr, op.hdr_len);
      return true;
    case VOP_CBOOL: {
      const uint32_t b = base[op.member];
      if (b > 1) return false;
      o.put(op.hdr | (b ? 1u : 2u), op.hdr_len);
      return true;
    }
    case VOP_FIXED:
      return put_fixed(o, compact, base + op.member, op.width, op.is_bool, op.bits == kFixedLE);
    case VOP_VARINT:
      nput_varint(o, zz_member(load_member(base + op.member, op.width), op.width, op.bits));
      return true;
    case VOP_STRING: {
      const tgpu_span sp = *(const tgpu_span*)(base + op.member);
      if (sp.length > 0x7fffffffu) return false;  // checkBinarySize
      if (compact) nput_varint(o, sp.length);
      else o.put(__builtin_bswap32(sp.length), 4);
      o.bytes(sbase + sp.offset, sp.length);
      return true;
    }
    case VOP_LIST: {
      const tgpu_span sp = *(const tgpu_span*)(base + op.member);
      if (!put_list_header(o, op, compact, sp.length)) return false;
      const uint8_t* e = lbase + sp.offset;
      const uint32_t es = op.width;
      if constexpr (O::kCount) {
        if (op.elem_kind == VEL_FIXED) {
          o.n += (uint64_t)sp.length * es;
          return true;
        }
      }
#ifndef TGPU_NLIST_ENC_SINGLE  // A/B (TGPU_JIT_DEFINES): one element per load
      if constexpr (!O::kCount) {
        // Binary 4- / 8-byte elements from an 8-byte aligned array: whole
        // 8-byte words, four loads in flight, one put each
        if (!compact && op.elem_kind == VEL_FIXED && (es == 4 || es == 8) &&
            ((uintptr_t)e & 7) == 0) {
          const uint64_t* q = (const uint64_t*)e;
          const uint32_t nw = es == 4 ? sp.length / 2 : sp.length;
          auto be = [es](uint64_t w) -> uint64_t {
            return es == 8 ? __builtin_bswap64(w)
                           : (uint64_t)__builtin_bswap32((uint32_t)w) |
                                 ((uint64_t)__builtin_bswap32((uint32_t)(w >> 32)) << 32);
          };
          uint32_t k = 0;
          for (; k + 4 <= nw; k += 4) {
            const uint64_t w0 = q[k], w1 = q[k + 1], w2 = q[k + 2], w3 = q[k + 3];
            o.put(be(w0), 8);
            o.put(be(w1), 8);
            o.put(be(w2), 8);
            o.put(be(w3), 8);
          }
          for (; k < nw; ++k) o.put(be(q[k]), 8);
          if (es == 4 && (sp.length & 1))
            o.put(__builtin_bswap32(((const uint32_t*)e)[sp.length - 1]), 4);
          return true;
        }
      }
#endif
      for (uint32_t i = 0; i < sp.length; ++i) {
        const uint8_t* p = e + (uint64_t)i * es;
        if (op.elem_kind == VEL_STRING) {
          const tgpu_span st = *(const tgpu_span*)p;
          if (st.length > 0x7fffffffu) return false;  // checkBinarySize
          if (compact) nput_varint(o, st.length);
          else o.put(__builtin_bswap32(st.length), 4);
          o.bytes(sbase + st.offset, st.length);
        } else if (op.elem_kind == VEL_VARINT) {
          nput_varint(o, zz_member(load_member(p, es), es, op.bits));
        } else if (!put_fixed(o, compact, p, es, op.elem_kind == VEL_BOOL,
                              op.elem_kind == VEL_FIXED && op.bits == kFixedLE)) {
          return false;
        }
      }
      return true;
    }
    default:
      return true;  // VOP_ISSET, VOP_SEQ_END: no bytes
  }
}

// Field headers on encode: Compact delta / long form from the struct's last
// field; a bool's value in the header (validate_bool).
template <class O>
__device__ __forceinline__ void put_cfield(O& o, int32_t id, uint32_t ct, int32_t& last) {
  uint64_t hb;
  uint32_t len;
  chdr_bytes(id, ct, last, hb, len);
  o.put(hb, len);
  last = id;
}
template <class O>
__device__ __forceinline__ bool put_cbool_field(O& o, int32_t id, int32_t& last, uint32_t v) {
  if (v > 1) return false;
  put_cfield(o, id, v ? 1u : 2u, last);
  return true;
}

// op::isEmpty of a terse member (Clear.h:98-127): a scalar of w bytes all
// zero bits (-0.0 is not empty), a string / container (w 0) of length 0.
__device__ __forceinline__ bool terse_leaf_empty(const uint8_t* m, uint32_t w) {
  if (!w) return ((const tgpu_span*)m)->length == 0;
  uint32_t any = 0;
  for (uint32_t b = 0; b < w; ++b) any |= m[b];
  return any == 0;
}

// VOP_SEQ: the header; the caller loops over the elements of the span
__device__ __forceinline__ tgpu_span seq_span(const VOp op, const uint8_t* base) {
  return *(const tgpu_span*)(base + op.member);
}

// Size pass: per-record sizes into a.offs, tile sums into a.block_sums (the
// general encode's layout, k_general.hip encode_size_kernel).
template <class E>
__device__ __forceinline__ void nested_size_tile(const EncodeArgs& a, const E& enc,
                                                 unsigned long long* part) {
  const uint64_t i = (uint64_t)blockIdx.x * kET + threadIdx.x;
  unsigned long long sz = 0;
  if (i < a.n) {
    Count o;
    if (enc(a.recs + i * a.rec_size, a.sbase, a.lbase, o)) {
      sz = o.n;
    } else {
#ifdef TGPU_NESTED_DEFER
      // a recursive schema's record nesting past the unrolled levels (or a
      // value the writer rejects): the general writer's deep pass sizes and
      // writes it, or reports it (deep_size_kernel / deep_write_kernel); the
      // write pass leaves its bytes to that pass
      a.deep.list[atomicAdd(a.deep.count, 1ull)] = i;
      atomicAdd(&a.res->n_irregular, 1ull);
#else
      atomicMin(&a.res->first_fail, (unsigned long long)i);
#endif
    }
    a.offs[i] = sz;
  }
  unsigned long long total;
  (void)block_exscan256(sz, part, &total);
  if (threadIdx.x == 0) a.block_sums[blockIdx.x] = total;
}

// Write pass: record starts from the scanned tile sums (encode_write_kernel).
// The tile's output (cap bytes of dynamic LDS, zero-filled) is built in LDS
// — whole words stored, each record's two edge words OR-ed in — and leaves
// with 16-byte stores, byte stores only in the two vectors shared with the
// neighbouring tiles; a tile larger than cap writes its records straight to
// the stream.
template <class E>
__device__ __forceinline__ void nested_write_tile(const EncodeArgs& a, const E& enc,
                                                  unsigned long long* part, uint8_t* tile,
                                                  uint32_t cap) {
  const uint64_t i = (uint64_t)blockIdx.x * kET + threadIdx.x;
  const unsigned long long sz = i < a.n ? a.offs[i] : 0;
  unsigned long long total;
  const unsigned long long t0 = a.block_sums[blockIdx.x];
  const unsigned long long start = t0 + block_exscan256(sz, part, &total);
  const uint32_t sh = (uint32_t)(((uintptr_t)a.out + t0) & 15);
  const bool staged = cap && total + sh + 16 <= cap && t0 + total <= a.cap;
  if (staged) {
    const uint4 z = {0u, 0u, 0u, 0u};
    const uint32_t nz = (uint32_t)((sh + total + 15) >> 4);
    for (uint32_t k = threadIdx.x; k < nz; k += kET) ((uint4*)tile)[k] = z;
  }
  __syncthreads();
  if (i < a.n) {
    a.offs[i] = start;
    if (start + sz > a.cap) {
      atomicMin(&a.res->first_fail, (unsigned long long)i);
    } else if (sz) {  // (sz 0: a record the size pass failed; the finish kernel reports it)
      if (staged) {
        OutT<true> o(tile + sh - (uintptr_t)0, start - t0);
        if (enc(a.recs + i * a.rec_size, a.sbase, a.lbase, o)) o.flush();
      } else {
        Out o(a.out, start);
        if (enc(a.recs + i * a.rec_size, a.sbase, a.lbase, o)) o.flush();
      }
    }
  }
  if (!staged) return;  // (uniform per workgroup)
  __syncthreads();
  uint8_t* base = a.out + t0 - sh;  // 16-byte aligned
  const uint32_t end = sh + (uint32_t)total;
  for (uint32_t k = threadIdx.x; k < ((end + 15) >> 4); k += kET) {
    const uint32_t lo = k << 4, hi = lo + 16;
    if (lo >= sh && hi <= end) {
      ((uint4*)base)[k] = ((const uint4*)tile)[k];
    } else {
      for (uint32_t b = (lo < sh ? sh : lo); b < (hi < end ? hi : end); ++b) base[b] = tile[b];
    }
  }
}

}  // namespace prog
}  // namespace tgpu
