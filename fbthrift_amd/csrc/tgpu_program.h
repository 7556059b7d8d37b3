// tgpu_program.h — the compiled-record-program codec shared by the indexed
// decode, the variable-length encode and the stream indexer. Not part of the
// public ABI.
//
// A VProgram (tgpu_api.cpp build_program) is the canonical wire form of one
// record of an all-unqualified schema: the header the generated readNoXfer
// expects next at each step (advanceToNextField's fast path,
// BinaryProtocol-inl.h:586-621 / CompactProtocol-inl.h:811-872) and the value
// that follows. run_program either accepts a record in exactly that form or
// reports it irregular (never an error): irregular records go to the general
// reader (tgpu_device.h), which has the full readNoXfer semantics.
//
// The program reaches the code through an accessor:
//   DynProg  — a device-resident VProgram read through the scalar cache; one
//              build of the kernels interprets any schema (the AOT library);
//   a static accessor (kStatic) — the same ops as compile-time constants, in
//              kernels the library generates and compiles for one schema at
//              run time (tgpu_jit.cpp), the way the reference's thrift1
//              compiler emits one readNoXfer/write per struct
//              (deserialize_struct.whisker:19-160, serialize_struct.whisker:40-67):
//              the op loop unrolls and every header, width and offset folds.
#pragma once

#include "tgpu_internal.h"

namespace tgpu {
namespace prog {

// ---- fixed-stride exceptions ----------------------------------------------------
// A fixed-stride batch (record i at i * L): record i is one the fast kernel
// could not take. It latches first_irregular and joins the exception list
// (irr[0 .. cap), count in n_irregular) that fixed_exception_kernel reads at
// the record's stride position. Called by the active lanes of a wave together
// (a lane passes flag = false when it has nothing), with i non-decreasing with
// the lane: one atomic per wave, the lowest flagged lane's i is the minimum.
// A record may be listed more than once (the reads are idempotent).
__device__ __forceinline__ void note_exception(bool flag, uint64_t i, DevResult* res,
                                               uint64_t* irr, uint64_t cap) {
  const uint64_t m = __ballot(flag);
  if (!m) return;
  const uint32_t lane = __lane_id();
  const uint32_t leader = (uint32_t)__builtin_ctzll(m);
  unsigned long long base = 0;
  if (lane == leader) {
    base = atomicAdd(&res->n_irregular, (unsigned long long)__popcll(m));
    atomicMin(&res->first_irregular, (unsigned long long)i);
  }
  base = __shfl(base, (int)leader, 64);
  if (flag) {
    const uint64_t k = base + (uint64_t)__popcll(m & ((1ull << lane) - 1));
    if (k < cap) irr[k] = i;
  }
}

// ---- LDS-DMA settle ------------------------------------------------------------
// After a wave's global_load_lds writes, `s_waitcnt vmcnt(0)` + `s_barrier`
// alone did not make them visible to the workgroup's other waves in the
// stream index's tiles: measured (TGPU_SPEC_LATE), 900-4400 threads per
// config-5 call saw their staged words change AFTER the staging barrier
// (round 2's "broken chains", hidden by the repair passes), while a
// standalone probe of the same staging never did (tools/glds_probe.hip).
// Each lane reading back one word of every vector it DMA'd, after
// vmcnt(0), made every such call clean (as did a 128-cycle pause, or
// staging through registers, which costs 0.2 ms per call); the caller's
// barrier then waits for these reads (lgkmcnt(0)). One read of the lane's
// last DMA'd vector is enough: zero repairs on config 5 and the whole GPU
// suite green with it, and 1-3 % off every LDS-DMA decode against a read per
// vector (TGPU_SETTLE_EACH, A/B). Round 5: the read is not
// what orders — the wait alone placed early (TGPU_SETTLE_WAIT_ONLY,
// TGPU_SETTLE_VMLGKM) is as clean, expcnt plays no part (TGPU_SETTLE_EXPCNT)
// and idle cycles before the wait do not help (TGPU_SETTLE_NOPS): what every
// clean form has is work between the wave's vmcnt reaching zero and the
// readers' first LDS read. `first` = the lane's first vector index, `step` =
// the vector stride between its DMAs, `n` = its DMAs.
__device__ __forceinline__ void lds_dma_settle(const uint8_t* lds, uint32_t first, uint32_t step,
                                               uint32_t n) {
#if defined(TGPU_SETTLE_EXPCNT)  // diagnostics: expcnt(0) alone (inline asm: the
  // compiler's wait pass would merge a builtin into its own full wait)
  asm volatile("s_waitcnt expcnt(0)" ::: "memory");
  (void)lds;
  (void)first;
  (void)step;
  (void)n;
  return;
#elif defined(TGPU_SETTLE_VMLGKM)  // diagnostics: vmcnt(0) lgkmcnt(0), expcnt left open
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  (void)lds;
  (void)first;
  (void)step;
  (void)n;
  return;
#elif defined(TGPU_SETTLE_NOPS)  // diagnostics: ~40 idle cycles, no wait (the
  // compiler's own vmcnt(0) lgkmcnt(0) stays right before the barrier)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  (void)lds;
  (void)first;
  (void)step;
  (void)n;
  return;
#endif
  __builtin_amdgcn_s_waitcnt(0);  // (vmcnt(0) expcnt(0) lgkmcnt(0))
#if defined(TGPU_SETTLE_WAIT_ONLY)  // diagnostics: the full wait alone
  (void)lds;
  (void)first;
  (void)step;
  (void)n;
#elif defined(TGPU_SETTLE_SLEEP)  // diagnostics: the wait, then ~4k cycles, no read
  (void)lds;
  (void)first;
  (void)step;
  (void)n;
  for (int k = 0; k < 64; ++k) __builtin_amdgcn_s_sleep(1);
#elif defined(TGPU_SETTLE_DSREAD)  // diagnostics: the read through the LDS address space
  if (n) {
    const __attribute__((address_space(3))) volatile uint32_t* l3 =
        (const __attribute__((address_space(3))) volatile uint32_t*)(lds);
    (void)l3[(first + (n - 1) * step) * 4];
  }
#elif !defined(TGPU_SETTLE_EACH)
  if (n) (void)((const volatile uint32_t*)lds)[(first + (n - 1) * step) * 4];
#else
  for (uint32_t k = 0; k < n; ++k)
    (void)((const volatile uint32_t*)lds)[(first + k * step) * 4];
#endif
}

// ---- program accessors --------------------------------------------------------
struct DynProg {
  static constexpr bool kStatic = false;
  static constexpr uint32_t kN = 0;
  static constexpr uint32_t kLists = 0;  // (the block rule's packing tile: compiled programs only)
  const VProgram* __restrict__ p;
  __device__ __forceinline__ uint32_t n_ops() const { return p->n_ops; }
  __device__ __forceinline__ uint32_t protocol() const { return p->protocol; }
  __device__ __forceinline__ bool has_lists() const { return p->has_list != 0; }
  __device__ __forceinline__ VOp op(uint32_t k) const { return p->ops[k]; }
};

// f(op) for every op in order; stops at the first op for which f returns false.
// Compiled programs expand the ops as a fold over a constant index sequence:
// every op is a constant and every call its own straight-line copy. (A
// `#pragma unroll` loop was left rolled by the compiler for large bodies —
// the write pass's emitter read the op table at run time.)
template <class T, T... K>
struct OpSeq {};
template <class PP, class F, uint32_t... K>
__device__ __forceinline__ bool all_ops_seq(const PP& P, F& f, OpSeq<uint32_t, K...>) {
  bool go = true;
  ((go = go && f(P.op(K))), ...);
  return go;
}
template <class PP, class F>
__device__ __forceinline__ bool all_ops(const PP& P, F&& f) {
  if constexpr (PP::kStatic) {
    return all_ops_seq(P, f, __make_integer_seq<OpSeq, uint32_t, PP::kN>{});
  } else {
    const uint32_t n = P.n_ops();
    for (uint32_t k = 0; k < n; ++k)
      if (!f(P.op(k))) return false;
  }
  return true;
}

// ---- byte sources: 8 bytes at position p, little-endian packed -------------
struct LdsSrc {
  const uint32_t* w32;  // LDS tile (at least 8 readable bytes past any position)
  __device__ __forceinline__ uint64_t win8(uint32_t p) const {
    const uint32_t d = p >> 2, s = p & 3;
    const uint32_t W0 = w32[d], W1 = w32[d + 1], W2 = w32[d + 2];
    const uint32_t lo = __builtin_amdgcn_alignbyte(W1, W0, s);
    const uint32_t hi = __builtin_amdgcn_alignbyte(W2, W1, s);
    return ((uint64_t)hi << 32) | lo;
  }
};

struct HbmSrc {
  const uint8_t* base;  // position 0
  uint32_t avail;       // readable bytes from base
  __device__ __forceinline__ uint64_t win8(uint32_t p) const {
    if ((uint64_t)p + 16 <= avail) {
      // two aligned 8-byte loads (never leave the 8-byte words around the window)
      const uintptr_t a = (uintptr_t)(base + p);
      const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
      const uint32_t s = (uint32_t)(a & 7) * 8;
      const uint64_t lo = q[0], hi = q[1];
      return s ? (lo >> s) | (hi << (64 - s)) : lo;
    }
    uint64_t v = 0;
    for (uint32_t i = 0; i < 8; ++i)
      if ((uint64_t)p + i < avail) v |= (uint64_t)base[p + i] << (8 * i);
    return v;
  }
};

__device__ __forceinline__ uint64_t bswap_n(uint64_t x, uint32_t width) {
  // the first `width` bytes of x (little-endian packed) as a big-endian number
  const uint64_t b = __builtin_bswap64(x);
  return width == 8 ? b : (b >> (64 - 8 * width));
}
// A FIXED value of `width` bytes: big-endian, or little-endian when the op
// says so (kFixedLE: CompactV1 doubles)
__device__ __forceinline__ uint64_t fixed_n(uint64_t x, uint32_t width, bool le) {
  if (!le) return bswap_n(x, width);
  return width == 8 ? x : (x & ((1ull << (8 * width)) - 1));
}

// LEB128 at p (VarintUtils-inl.h:94-134): up to 8 bytes from one window,
// 9-10 byte i64 varints byte-wise. Returns false (irregular) on anything the
// fast path does not take (past `end`, more than ceil(bits/7) bytes).
// w: the 8 bytes at p (a caller's cached window), or read here.
template <class Src>
__device__ __forceinline__ bool read_varint_w(const Src& src, uint64_t w, uint32_t& p,
                                              uint32_t end, uint32_t bits, uint64_t& v);
template <class Src>
__device__ __forceinline__ bool read_varint(const Src& src, uint32_t& p, uint32_t end,
                                            uint32_t bits, uint64_t& v) {
  return read_varint_w(src, src.win8(p), p, end, bits, v);
}
template <class Src>
__device__ __forceinline__ bool read_varint_w(const Src& src, uint64_t w, uint32_t& p,
                                              uint32_t end, uint32_t bits, uint64_t& v) {
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
    const uint64_t b = (src.win8(p + i) & 0xff);
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
// VarintUtils-inl.h:630-636
__device__ __forceinline__ uint32_t i32_to_zz(int32_t n) {
  return ((uint32_t)n << 1) ^ (uint32_t)(n >> 31);
}
__device__ __forceinline__ uint64_t i64_to_zz(int64_t n) {
  return ((uint64_t)n << 1) ^ (uint64_t)(n >> 63);
}

struct Ctx {
  uint64_t gbase;  // stream offset of source position 0
  uint8_t* arena;
  uint64_t arena_cap;
  int32_t string_limit, container_limit;
  // Binary decode tile: list elements are converted in place in the LDS
  // wire tile (an element's arena slot is its own wire bytes, scale 1) and
  // the tile is copied to the arena with coalesced stores afterwards
  uint8_t* lds_wire;
  // nested programs of schemas without record regions: the position rule's
  // scale (an element array at scale x its first element's stream offset)
  uint64_t pos_scale = 0;
};

// At the root STOP (kStopSkipsUnknown) a field header instead of STOP: up to
// kMaxUnknownTail fields with ids above the schema's, each a scalar or a
// string within the limits, are skipped (the general reader's unknown-field
// path, BinaryProtocol.cpp skip / Protocol.h:187-344, for these types), then
// the STOP. Anything else is irregular (the general reader decides).
constexpr uint32_t kMaxUnknownTail = 8;

template <class Src>
__device__ __forceinline__ bool skip_unknown_tail(const VOp op, const bool compact,
                                                            const Src src, const Ctx c,
                                                            uint32_t& pos, const uint32_t end) {
  const int32_t max_id = (int16_t)op.member;
  int32_t prev = (int16_t)(uint16_t)(op.hdr >> 8);
  uint32_t p = pos;
  for (uint32_t k = 0; k <= kMaxUnknownTail; ++k) {
    if (p + 1 > end) return false;
    const uint64_t w = src.win8(p);
    const uint32_t b = (uint32_t)(w & 0xff);
    if (b == 0) {  // STOP
      pos = p + 1;
      return true;
    }
    if (k == kMaxUnknownTail) return false;
    int32_t id;
    uint32_t t;
    if (!compact) {
      if (p + 3 > end) return false;
      t = b;
      id = (int16_t)(uint16_t)(((w >> 8) & 0xff) << 8 | ((w >> 16) & 0xff));
      p += 3;
    } else {
      t = b & 0xf;
      const uint32_t d = b >> 4;
      ++p;
      if (d) {
        id = prev + (int32_t)d;
      } else {
        uint64_t z;
        if (!read_varint(src, p, end, 32, z)) return false;
        const int64_t v = (int64_t)unzigzag(z, 32);
        if (v < -32768 || v > 32767) return false;
        id = (int32_t)v;
      }
      prev = id;
    }
    if (id <= max_id) return false;  // a schema id (or below): not a plain append
    int64_t n;  // value bytes
    if (!compact) {
      switch (t) {
        case TGPU_T_BOOL:
          if (p + 1 > end || (src.win8(p) & 0xff) > 1) return false;
          n = 1;
          break;
        case TGPU_T_BYTE: n = 1; break;
        case TGPU_T_I16: n = 2; break;
        case TGPU_T_I32: case TGPU_T_FLOAT: n = 4; break;
        case TGPU_T_I64: case TGPU_T_DOUBLE: n = 8; break;
        case TGPU_T_STRING:
          if (p + 4 > end) return false;
          n = (int32_t)(uint32_t)bswap_n(src.win8(p), 4);
          p += 4;
          if (n < 0 || (c.string_limit > 0 && n > c.string_limit)) return false;
          break;
        default: return false;
      }
    } else {
      switch (t) {
        case 1: case 2: n = 0; break;  // bool in the header
        case 3: n = 1; break;          // byte
        case 4: case 5: case 6: {      // i16 / i32 / i64 varints
          uint64_t z;
          if (!read_varint(src, p, end, t == 6 ? 64 : 32, z)) return false;
          n = 0;
          break;
        }
        case 7: n = 8; break;   // double
        case 13: n = 4; break;  // float
        case 8: {               // binary
          uint64_t z;
          if (!read_varint(src, p, end, 32, z)) return false;
          n = (int32_t)(uint32_t)z;
          if (n < 0 || (c.string_limit > 0 && n > c.string_limit)) return false;
          break;
        }
        default: return false;
      }
    }
    if (n > (int64_t)(end - p)) return false;
    p += (uint32_t)n;
  }
  return false;
}

// The last 8-byte window a record's walk read. With TGPU_WINCACHE an op whose
// bytes lie inside it takes them from there (a Compact field header and its
// varint share one window: about one dependent LDS read per field instead of
// one per op). Measured slower (decode config 3 1.47 -> 1.51 ms, config 4
// 2.50 -> 2.69, config 5 6.70 -> 6.88; tools/kbench_jit.py), so off: every op
// reads its own window.
//
// TGPU_CARRY: a CONST header's window also serves the op right after it when
// that op's bytes (need) fit in the 8 - hdr_len left (decided by the op kinds
// alone, so it folds away in the compiled programs). Measured: config 3
// decode 1.468 vs 1.473 ms, config 4 2.68 vs 1.84 ms (slower), so off here;
// the index's branch-free walk (measure_lds) keeps it.
struct Win {
  uint64_t w = 0;
  uint32_t wp = 0;
  bool valid = false;
  uint32_t carry = 0;  // hdr_len of the CONST just read (its window is w)
  template <class Src>
  __device__ __forceinline__ uint64_t at(const Src& src, uint32_t p, uint32_t need) {
    const uint32_t h = carry;
    carry = 0;
#ifdef TGPU_CARRY
    if (h && h + need <= 8) return w >> (8 * h);
#else
    (void)h;
#endif
#ifdef TGPU_WINCACHE
    const uint32_t d = p - wp;
    if (valid && d + need <= 8) return w >> (8 * d);
#endif
    w = src.win8(p);
    wp = p;
    valid = true;
    return w;
  }
};

// One op of the program at p (bounded by end); false = irregular.
template <bool kStore, class Src>
__device__ __forceinline__ bool run_op(const VOp op, const bool compact, const Src& src,
                                       const Ctx& c, uint32_t& p, uint32_t end, uint8_t* rec,
                                       Win& W) {
  switch (op.kind) {
    case VOP_CONST: {
      if (p + op.hdr_len > end) return false;
      const uint32_t lo = (uint32_t)W.at(src, p, 8);
      const uint32_t mask = op.hdr_len >= 4 ? 0xffffffffu : ((1u << (8 * op.hdr_len)) - 1);
      if ((lo ^ op.hdr) & mask) {
#ifdef TGPU_NO_TAILS  // a compiled strict program (tgpu_jit.cpp)
        return false;
#else
        if (op.elem_kind != kStopSkipsUnknown) return false;
        if (!skip_unknown_tail(op, compact, src, c, p, end)) return false;
        break;
#endif
      }
      p += op.hdr_len;
      W.carry = op.hdr_len;
      break;
    }
    case VOP_CBOOL: {
      if (p + op.hdr_len > end) return false;
      const uint32_t lo = (uint32_t)W.at(src, p, op.hdr_len);
      const uint32_t mask = (op.hdr_len >= 4 ? 0xffffffffu : ((1u << (8 * op.hdr_len)) - 1)) & ~0xfu;
      const uint32_t ct = lo & 0xf;
      if (((lo ^ op.hdr) & mask) || (ct != 1 && ct != 2)) return false;
      if (kStore) rec[op.member] = ct == 1 ? 1 : 0;
      p += op.hdr_len;
      break;
    }
    case VOP_FIXED: {
      if (p + op.width > end) return false;
      uint64_t v = fixed_n(W.at(src, p, op.width), op.width, op.bits == kFixedLE);
      // a bool: Binary readBool throws on a byte >= 2 (general path); a
      // Compact container bool is byte == 1 (nested programs' map keys / values)
      if (op.is_bool && !compact && v > 1) return false;
      if (op.is_bool && compact) v = v == 1;
      if (kStore) store_n(rec + op.member, v, op.width);
      p += op.width;
      break;
    }
    case VOP_VARINT: {
      uint64_t z;
      if (!read_varint_w(src, W.at(src, p, op.bits == 32 ? 5 : 8), p, end, op.bits, z))
        return false;
      if (kStore) store_n(rec + op.member, unzigzag(z, op.bits), op.width);
      break;
    }
    case VOP_STRING: {
      int64_t len;
      if (compact) {
        uint64_t z;
        if (!read_varint_w(src, W.at(src, p, 5), p, end, 32, z)) return false;
        len = (int32_t)(uint32_t)z;
      } else {
        if (p + 4 > end) return false;
        len = (int32_t)(uint32_t)bswap_n(W.at(src, p, 4), 4);
        p += 4;
      }
      if (len < 0 || (c.string_limit > 0 && len > c.string_limit) || len > (int64_t)(end - p))
        return false;
      if (kStore) {
        tgpu_span* sp = (tgpu_span*)(rec + op.member);
        sp->offset = len ? c.gbase + p : 0;
        sp->length = (uint32_t)len;
        sp->reserved = 0;
      }
      p += (uint32_t)len;
      break;
    }
    case VOP_LIST: {
      int64_t n;
      if (compact) {
        if (p + 1 > end) return false;
        const uint32_t b = (uint32_t)(W.at(src, p, 1) & 0xff);
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
        const uint64_t w = W.at(src, p, 5);
        if ((w & 0xff) != op.elem_ttype) return false;
        n = (int32_t)(uint32_t)bswap_n(w >> 8, 4);
        p += 5;
      }
      if (n < 0 || (c.container_limit && n > c.container_limit) || n > (int64_t)(end - p))
        return false;
      const uint64_t scale = compact ? 8 : 1;
      const uint64_t aoff = scale * (c.gbase + p);
      const uint32_t es = op.width;
      if (kStore && n && (!c.arena || aoff + (uint64_t)n * es > c.arena_cap)) return false;
      if (!kStore && op.elem_kind == VEL_FIXED) {
        if ((uint64_t)n * es > end - p) return false;
        p += (uint32_t)n * es;
      } else {
        for (int64_t i = 0; i < n; ++i) {
          uint64_t v;
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
            if (kStore && c.lds_wire) store_n(c.lds_wire + p, v, wb);  // in place (wb == es)
            p += wb;
          }
#ifndef TGPU_NO_ARENA_STORE  // A/B only (tools/kbench_jit.py): cost of the element stores
          if (kStore && !c.lds_wire) store_n(c.arena + aoff + (uint64_t)i * es, v, es);
#endif
        }
      }
      if (kStore) {
        tgpu_span* sp = (tgpu_span*)(rec + op.member);
        sp->offset = n ? aoff : 0;
        sp->length = (uint32_t)n;
        sp->reserved = 0;
      }
      break;
    }
    case VOP_ISSET:
      break;
    default:
      return false;
  }
  if (kStore && op.isset != 0xffff) rec[op.isset] = 1;
  return true;
}

// ---- branch-free measuring walk (stream index) ---------------------------------
// run_program<false> decides each op with an early return; in the index's
// speculation (every lane walking its slice's records, most of them
// different lengths) each return is a divergent branch: the compiled config-5
// speculation kernel ran ~1,500 SALU (exec-mask) instructions per wave. Here
// every op is straight-line: the checks AND into `ok` and the walk carries on
// over whatever bytes follow (reads clamped into the staged tile), so a wave
// runs the record's ops once, in lockstep. Accepts exactly what
// run_program<false> accepts with the same end position, for every record
// whose reads stay inside the staged bytes (position <= lim); anything it
// does not decide here sets `slow` (a read past lim, a 9-10 byte i64
// varint, element loops, the tolerant programs' appended fields) and the
// caller runs run_program on the record instead.
template <class PP>
__device__ __forceinline__ bool measure_lds(const PP& P, const uint32_t* w32, uint32_t lim,
                                            const Ctx& c, uint32_t& pos, uint32_t end, bool& slow) {
  const bool compact = P.protocol() != TGPU_PROTOCOL_BINARY;
  const LdsSrc src{w32};
  uint32_t p = pos;
  bool ok = true, sl = false;
  auto rd = [&](uint32_t q) {
    sl |= ok && q > lim;
    return src.win8(q > lim ? lim : q);
  };
  // LEB128 of a 32-bit value in w (read_varint_w's fast form): length, value
  auto var32 = [&](uint64_t w, uint32_t& len) {
    const uint64_t stop = ~w & 0x8080808080808080ull;
    len = stop ? ((uint32_t)__builtin_ctzll(stop) >> 3) + 1 : 8;
    ok &= stop != 0 && len <= 5;
    uint64_t x = w & ((len >= 8 ? 0 : (1ull << (8 * len))) - 1) & 0x7f7f7f7f7f7f7f7full;
    x = ((x & 0x7f007f007f007f00ull) >> 1) | (x & 0x007f007f007f007full);
    x = ((x & 0x3fff00003fff0000ull) >> 2) | (x & 0x00003fff00003fffull);
    x = ((x & 0x0fffffff00000000ull) >> 4) | (x & 0x000000000fffffffull);
    return (uint32_t)x;
  };
  // A header's window also holds the value right after it: the op after a
  // CONST of hdr_len h takes the window shifted by h when the bytes it may
  // look at (need) fit in the 8 - h left, instead of a dependent LDS read.
  // (Whether it does is decided by the op kinds alone, so in the compiled
  // programs it folds away.) A Compact {header, varint} field is one read.
  uint64_t cw = 0;
  uint32_t carry = 0;  // hdr_len of the previous op when it was a CONST, else 0
  auto rdv = [&](uint32_t need) {
    const uint32_t h = carry;
    carry = 0;
    if (h && h + need <= 8) return cw >> (8 * h);
    return rd(p);
  };
  all_ops(P, [&](const VOp op) {
    switch (op.kind) {
      case VOP_CONST: {
        const uint64_t w = rdv(8);
        const uint32_t lo = (uint32_t)w;
        const uint32_t mask = op.hdr_len >= 4 ? 0xffffffffu : ((1u << (8 * op.hdr_len)) - 1);
        const bool hit = ((lo ^ op.hdr) & mask) == 0;
#ifndef TGPU_NO_TAILS
        if (op.elem_kind == kStopSkipsUnknown) sl |= ok && !hit;
#endif
        ok &= p + op.hdr_len <= end && hit;
        p += op.hdr_len;
        cw = w;
        carry = op.hdr_len;
        break;
      }
      case VOP_CBOOL: {
        const uint32_t lo = (uint32_t)rdv(8);
        const uint32_t mask =
            (op.hdr_len >= 4 ? 0xffffffffu : ((1u << (8 * op.hdr_len)) - 1)) & ~0xfu;
        const uint32_t ct = lo & 0xf;
        ok &= p + op.hdr_len <= end && ((lo ^ op.hdr) & mask) == 0 && (ct == 1 || ct == 2);
        p += op.hdr_len;
        break;
      }
      case VOP_FIXED: {
        const uint64_t v = bswap_n(rdv(op.width), op.width);
        ok &= p + op.width <= end && !(op.is_bool && !compact && v > 1);
        p += op.width;
        break;
      }
      case VOP_VARINT: {
        // (an i32 varint's verdict needs its first 5 bytes: a longer one
        // fails either way; an i64's needs the whole window)
        const uint64_t w = rdv(op.bits == 32 ? 5 : 8);
        const uint64_t stop = ~w & 0x8080808080808080ull;
        const uint32_t len = stop ? ((uint32_t)__builtin_ctzll(stop) >> 3) + 1 : 8;
        if (op.bits == 32) {
          ok &= stop != 0 && len <= 5;
        } else {
          sl |= ok && stop == 0;  // 9-10 byte i64 varint
        }
        ok &= p + len <= end;
        p += len;
        break;
      }
      case VOP_STRING: {
        const uint64_t w = rdv(compact ? 5 : 4);
        uint32_t hl, n;
        if (compact) {
          n = var32(w, hl);
        } else {
          hl = 4;
          n = (uint32_t)bswap_n(w, 4);
        }
        ok &= p + hl <= end;
        p += hl;
        const int64_t len = (int32_t)n;
        ok &= len >= 0 && !(c.string_limit > 0 && len > c.string_limit) &&
              len <= (int64_t)end - (int64_t)p;
        p += ok ? (uint32_t)len : 0u;
        break;
      }
      case VOP_LIST: {
        const uint64_t w = rdv(compact ? 1 : 5);
        int64_t n;
        if (compact) {
          const uint32_t b = (uint32_t)(w & 0xff);
          const uint32_t ct = b & 0xf;
          ok &= p + 1 <= end &&
                (op.elem_ttype == TGPU_T_BOOL ? (ct == 1 || ct == 2) : ct == op.elem_ct);
          p += 1;
          n = b >> 4;
          if (n == 15) {  // count in a varint (uniform per op: rare, branch kept)
            uint32_t vl;
            const uint32_t z = var32(rd(p), vl);
            ok &= p + vl <= end;
            p += vl;
            n = (int32_t)z;
          }
        } else {
          ok &= p + 5 <= end && (w & 0xff) == op.elem_ttype;
          n = (int32_t)(uint32_t)bswap_n(w >> 8, 4);
          p += 5;
        }
        ok &= n >= 0 && !(c.container_limit && n > c.container_limit) &&
              n <= (int64_t)end - (int64_t)p;
        const bool fixed = op.elem_kind == VEL_FIXED || (compact && op.elem_kind == VEL_BOOL);
        if (fixed) {
          const uint64_t bytes = (uint64_t)(ok ? n : 0) * (op.elem_kind == VEL_BOOL ? 1u : op.width);
          ok &= bytes <= (uint64_t)end - p;
          p += ok ? (uint32_t)bytes : 0u;
        } else {
          sl |= ok && n > 0;  // element loops: run_program
        }
        break;
      }
      case VOP_ISSET:
        break;  // (no bytes: a carried window stays valid)
      default:
        sl |= ok;
        carry = 0;
        break;
    }
    return true;
  });
  slow = sl;
  if (ok && !sl) pos = p;
  return ok;
}

// Runs the program from pos over at most [pos, end). On success pos is the
// end of the record. kStore: write members / isset / spans into rec and list
// elements into the arena; otherwise only measure and validate.
template <bool kStore, class PP, class Src>
__device__ __forceinline__ bool run_program(const PP& P, const Src& src, const Ctx& c,
                                            uint32_t& pos, uint32_t end, uint8_t* rec) {
  const bool compact = P.protocol() == TGPU_PROTOCOL_COMPACT;
  uint32_t p = pos;
  Win W;
  if (!all_ops(P, [&](const VOp op) { return run_op<kStore>(op, compact, src, c, p, end, rec, W); }))
    return false;
  pos = p;
  return true;
}

}  // namespace prog
}  // namespace tgpu
