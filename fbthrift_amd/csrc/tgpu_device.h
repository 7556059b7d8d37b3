// tgpu_device.h — per-lane Binary/Compact reader and writer used by the
// general (table-driven) gfx950 kernels. One lane parses or emits one record.
//
// Semantics follow the reference exactly (file:line in the fbthrift tree):
//   field headers   BinaryProtocol-inl.h:586-632; CompactProtocol-inl.h:811-910
//   scalar reads    BinaryProtocol-inl.h:489-533; CompactProtocol-inl.h:692-740
//   varints         VarintUtils-inl.h:94-134 (max ceil(bits/7) bytes, junk high
//                   bits dropped, overlong zeros accepted), :648-663 zigzag
//   strings         Protocol.h:435-449 readStringBody (truncation checked first)
//   lists           protocol_methods.h:389-467 (reset, type-mismatch skip_n,
//                   canReadNElements, element reads)
//   skip            BinaryProtocol.cpp:140-225; Protocol.h:187-344 (Compact)
//   depth           Protocol.h:59-78 descend/ascend (height = max_depth + 1)
//   struct driver   deserialize_struct.whisker:19-160 (any order, unknown and
//                   type-mismatched fields skipped, isset set after the read)
//   writers         BinaryProtocol-inl.h:41-222; CompactProtocol-inl.h:91-383;
//                   serialize_struct.whisker:40-67
// Device code cannot throw: the first error is latched in the reader/writer
// (code + byte offset) and every later operation becomes a no-op.
#pragma once

#include "tgpu_internal.h"

namespace tgpu {
namespace dev {

__device__ __forceinline__ bool is_scalar(uint32_t t) {
  return t == TGPU_T_BOOL || t == TGPU_T_BYTE || t == TGPU_T_I16 || t == TGPU_T_I32 ||
         t == TGPU_T_I64 || t == TGPU_T_DOUBLE || t == TGPU_T_FLOAT;
}
__device__ __forceinline__ uint32_t scalar_size(uint32_t t) {
  return (t == TGPU_T_BOOL || t == TGPU_T_BYTE) ? 1
         : t == TGPU_T_I16                      ? 2
         : (t == TGPU_T_I32 || t == TGPU_T_FLOAT) ? 4
                                                  : 8;
}
// Container elements: scalars in native layout, strings and containers as
// tgpu_span (structs: slot_size).
__device__ __forceinline__ uint32_t elem_size(uint32_t t) {
  return (t == TGPU_T_STRING || t == TGPU_T_LIST || t == TGPU_T_SET || t == TGPU_T_MAP)
             ? 16 : scalar_size(t);
}
// CompactProtocol-inl.h:48-86
__device__ __forceinline__ uint32_t ctype_to_ttype(uint32_t ct) {
  // packed nibble table for ct 0..13
  constexpr uint8_t tbl[14] = {TGPU_T_STOP, TGPU_T_BOOL, TGPU_T_BOOL, TGPU_T_BYTE,
                               TGPU_T_I16,  TGPU_T_I32,  TGPU_T_I64,  TGPU_T_DOUBLE,
                               TGPU_T_STRING, TGPU_T_LIST, TGPU_T_SET, TGPU_T_MAP,
                               TGPU_T_STRUCT, TGPU_T_FLOAT};
  return tbl[ct];
}
__device__ __forceinline__ uint32_t ttype_to_ctype(uint32_t t) {
  switch (t) {
    case TGPU_T_BOOL: return 1;
    case TGPU_T_BYTE: return 3;
    case TGPU_T_I16: return 4;
    case TGPU_T_I32: return 5;
    case TGPU_T_I64: return 6;
    case TGPU_T_DOUBLE: return 7;
    case TGPU_T_STRING: return 8;
    case TGPU_T_LIST: return 9;
    case TGPU_T_SET: return 10;
    case TGPU_T_MAP: return 11;
    case TGPU_T_STRUCT: return 12;
    case TGPU_T_FLOAT: return 13;
    default: return 0;
  }
}
__device__ __forceinline__ int32_t zz_to_i32(uint32_t n) {
  return (n & 1) ? (int32_t)~(n >> 1) : (int32_t)(n >> 1);
}
__device__ __forceinline__ int64_t zz_to_i64(uint64_t n) {
  return (n & 1) ? (int64_t)~(n >> 1) : (int64_t)(n >> 1);
}
__device__ __forceinline__ uint32_t i32_to_zz(int32_t n) {
  return ((uint32_t)n << 1) ^ (uint32_t)(n >> 31);
}
__device__ __forceinline__ uint64_t i64_to_zz(int64_t n) {
  return ((uint64_t)n << 1) ^ (uint64_t)(n >> 63);
}

// ------------------------------------------------------------------ reader --
struct Reader {
  const uint8_t* p;  // byte at stream position x: p[x - base]
  uint64_t base;     // 0, or the stream position of an LDS copy's first byte
  uint64_t pos, end;
  int64_t height;
  int32_t string_limit, container_limit, max_depth;
  int32_t err;
  uint64_t err_off;
  bool has_bool, bool_val;  // Compact boolValue_ latch
  // skip frames past the private kMaxSkipDepth (nullptr: kErrDeep instead)
  uint8_t* deep;
  uint64_t deep_cap;  // frames at `deep`
  bool deep_more;     // a larger slab follows (the wide tier): full is kErrDeep

  __device__ __forceinline__ bool ok() const { return err == 0; }
  __device__ __forceinline__ void fail(int32_t code, uint64_t off) {
    if (!err) {
      err = code;
      err_off = off;
    }
  }
  __device__ __forceinline__ uint32_t read8() {
    if (pos >= end) {
      fail(TGPU_ERR_UNDERFLOW, pos);
      return 0;
    }
    return p[pos++ - base];
  }
  __device__ __forceinline__ uint64_t readBE(uint32_t nbytes) {
    if (end - pos < nbytes) {
      fail(TGPU_ERR_UNDERFLOW, pos);
      pos = end;
      return 0;
    }
    uint64_t v = 0;
    for (uint32_t i = 0; i < nbytes; ++i) v = (v << 8) | p[pos - base + i];
    pos += nbytes;
    return v;
  }
  __device__ __forceinline__ void skip_bytes(uint64_t n) {
    if (end - pos < n) {
      fail(TGPU_ERR_UNDERFLOW, pos);
      pos = end;
      return;
    }
    pos += n;
  }
  // LEB128 with kMax = ceil(bits/7) bytes; value truncated to `bits`.
  __device__ __forceinline__ uint64_t varint(uint32_t bits) {
    const uint32_t kmax = (bits + 6) / 7;
    const uint64_t start = pos;
    uint64_t r = 0;
    for (uint32_t i = 0; i < kmax; ++i) {
      if (pos >= end) {
        fail(TGPU_ERR_UNDERFLOW, pos);
        return 0;
      }
      const uint64_t b = p[pos++ - base];
      r |= (b & 0x7f) << (7 * i);
      if (!(b & 0x80)) return bits < 64 ? (r & ((1ull << bits) - 1)) : r;
    }
    fail(TGPU_ERR_INVALID_VARINT, start);
    return 0;
  }
  __device__ __forceinline__ void descend(uint64_t off) {
    if (!--height) fail(TGPU_ERR_DEPTH_LIMIT, off);
  }
  __device__ __forceinline__ void ascend() { ++height; }
};

// A reader at `pos` of in[0..end) with the call's limits; height is
// ProtocolBase::setHeight (0 = max_depth, Protocol.h:59-78) plus the root.
__device__ __forceinline__ Reader make_reader(const uint8_t* in, uint64_t pos, uint64_t end,
                                             int32_t string_limit, int32_t container_limit,
                                             int32_t max_depth, int32_t height) {
  Reader r;
  r.p = in;
  r.base = 0;
  r.pos = pos;
  r.end = end;
  r.height = (int64_t)(height ? height : max_depth) + 1;
  r.string_limit = string_limit;
  r.container_limit = container_limit;
  r.max_depth = max_depth;
  r.err = 0;
  r.err_off = 0;
  r.has_bool = false;
  r.bool_val = false;
  r.deep = nullptr;
  r.deep_cap = 0;
  r.deep_more = false;
  return r;
}

template <int P>
struct Proto;

// ---------------------------------------------------------------- Binary ----
template <>
struct Proto<TGPU_PROTOCOL_BINARY> {
  static constexpr uint64_t kArenaScale = 1;
  // returns false on STOP (or error)
  static __device__ __forceinline__ bool field_header(Reader& r, int32_t /*prev*/,
                                                      uint32_t& type, int32_t& id) {
    type = r.read8();
    if (!r.ok() || type == TGPU_T_STOP) return false;
    id = (int16_t)r.readBE(2);
    return r.ok();
  }
  static __device__ __forceinline__ uint32_t read_bool(Reader& r) {
    const uint64_t off = r.pos;
    const uint32_t b = r.read8();
    if (b >= 2) r.fail(TGPU_ERR_BOOL_VALUE, off);
    return b ? 1 : 0;
  }
  static __device__ __forceinline__ void check_container(Reader& r, int32_t size, uint64_t off) {
    if (size < 0) r.fail(TGPU_ERR_NEGATIVE_SIZE, off);
    else if (r.container_limit && size > r.container_limit) r.fail(TGPU_ERR_SIZE_LIMIT, off);
  }
  static __device__ __forceinline__ void list_begin(Reader& r, uint32_t& elem, int32_t& size) {
    r.descend(r.pos);
    if (!r.ok()) return;
    elem = r.read8();
    const uint64_t soff = r.pos;
    size = (int32_t)(uint32_t)r.readBE(4);
    if (r.ok()) check_container(r, size, soff);
  }
  static __device__ __forceinline__ void map_begin(Reader& r, uint32_t& k, uint32_t& v, int32_t& size) {
    r.descend(r.pos);
    if (!r.ok()) return;
    k = r.read8();
    v = r.read8();
    const uint64_t soff = r.pos;
    size = (int32_t)(uint32_t)r.readBE(4);
    if (r.ok()) check_container(r, size, soff);
  }
  static __device__ __forceinline__ void read_string(Reader& r, uint64_t& view, uint32_t& len) {
    const uint64_t off = r.pos;
    const int32_t size = (int32_t)(uint32_t)r.readBE(4);
    if (!r.ok()) return;
    if (size < 0) return r.fail(TGPU_ERR_NEGATIVE_SIZE, off);
    if (r.string_limit > 0 && size > r.string_limit) return r.fail(TGPU_ERR_SIZE_LIMIT, off);
    if (r.end - r.pos < (uint64_t)size) return r.fail(TGPU_ERR_TRUNCATED, r.pos);
    view = r.pos;
    len = (uint32_t)size;
    r.pos += (uint64_t)size;
  }
  static __device__ __forceinline__ uint32_t fixed_in_container(uint32_t t) {
    return (t == TGPU_T_BOOL || t == TGPU_T_BYTE) ? 1
           : t == TGPU_T_I16                      ? 2
           : (t == TGPU_T_I32 || t == TGPU_T_FLOAT) ? 4
           : (t == TGPU_T_I64 || t == TGPU_T_DOUBLE) ? 8
                                                     : 0;
  }
  // Skip of a leaf value; returns false if `t` is a container/struct that
  // needs a frame (handled by the caller's explicit stack).
  static __device__ __forceinline__ bool skip_leaf(Reader& r, uint32_t t) {
    switch (t) {
      case TGPU_T_BYTE: case TGPU_T_BOOL: r.skip_bytes(1); return true;
      case TGPU_T_I16: r.skip_bytes(2); return true;
      case TGPU_T_FLOAT: case TGPU_T_I32: r.skip_bytes(4); return true;
      case TGPU_T_DOUBLE: case TGPU_T_U64: case TGPU_T_I64: r.skip_bytes(8); return true;
      case TGPU_T_UTF8: case TGPU_T_UTF16: case TGPU_T_STRING: {
        const uint64_t before = r.pos;
        const int32_t size = (int32_t)(uint32_t)r.readBE(4);
        if (!r.ok()) return true;
        // canAdvance from the cursor copy taken before the length
        const uint64_t want = (uint64_t)(int64_t)size;
        if (r.end - before < want) {
          r.fail(TGPU_ERR_TRUNCATED, r.pos);
          return true;
        }
        r.skip_bytes((uint64_t)(uint32_t)size);
        return true;
      }
      default: return false;
    }
  }
  static __device__ __forceinline__ void read_scalar(Reader& r, uint32_t t, uint8_t* dst) {
    switch (t) {
      case TGPU_T_BOOL: { const uint32_t v = read_bool(r); if (r.ok()) *dst = (uint8_t)v; break; }
      case TGPU_T_BYTE: { const uint32_t v = r.read8(); if (r.ok()) *dst = (uint8_t)v; break; }
      case TGPU_T_I16: { const uint16_t v = (uint16_t)r.readBE(2); if (r.ok()) *(uint16_t*)dst = v; break; }
      case TGPU_T_I32:
      case TGPU_T_FLOAT: { const uint32_t v = (uint32_t)r.readBE(4); if (r.ok()) *(uint32_t*)dst = v; break; }
      default: { const uint64_t v = r.readBE(8); if (r.ok()) *(uint64_t*)dst = v; break; }
    }
  }
};

// --------------------------------------------------------------- Compact ----
template <>
struct Proto<TGPU_PROTOCOL_COMPACT> {
  static constexpr uint64_t kArenaScale = 8;
  static __device__ __forceinline__ uint32_t get_type(Reader& r, uint32_t ct, uint64_t off) {
    if (ct >= 14) {
      r.fail(TGPU_ERR_BAD_TYPE, off);
      return TGPU_T_STOP;
    }
    return ctype_to_ttype(ct);
  }
  static __device__ __forceinline__ bool field_header(Reader& r, int32_t prev, uint32_t& type,
                                                      int32_t& id) {
    const uint64_t off = r.pos;
    const uint32_t b = r.read8();
    if (!r.ok() || (b & 0x0f) == 0) return false;  // STOP
    const int32_t mod = (int32_t)(b >> 4);
    if (mod) id = (int16_t)(prev + mod);
    else id = (int16_t)zz_to_i32((uint32_t)r.varint(32));
    if (!r.ok()) return false;
    const uint32_t ct = b & 0x0f;
    type = get_type(r, ct, off);
    if (ct == 1 || ct == 2) {
      r.has_bool = true;
      r.bool_val = ct == 1;
    }
    return r.ok();
  }
  static __device__ __forceinline__ uint32_t read_bool(Reader& r) {
    if (r.has_bool) {
      r.has_bool = false;
      return r.bool_val ? 1 : 0;
    }
    return r.read8() == 1 ? 1 : 0;
  }
  static __device__ __forceinline__ void list_begin(Reader& r, uint32_t& elem, int32_t& size) {
    const uint64_t off = r.pos;
    r.descend(off);
    if (!r.ok()) return;
    const uint32_t b = r.read8();
    if (!r.ok()) return;
    int32_t lsize = (int32_t)((b >> 4) & 0x0f);
    if (lsize == 15) lsize = (int32_t)(uint32_t)r.varint(32);
    if (!r.ok()) return;
    if (lsize < 0) return r.fail(TGPU_ERR_NEGATIVE_SIZE, off);
    if (r.container_limit && lsize > r.container_limit) return r.fail(TGPU_ERR_SIZE_LIMIT, off);
    elem = get_type(r, b & 0x0f, off);
    size = lsize;
  }
  static __device__ __forceinline__ void map_begin(Reader& r, uint32_t& k, uint32_t& v, int32_t& size) {
    const uint64_t off = r.pos;
    r.descend(off);
    if (!r.ok()) return;
    uint32_t kv = 0;
    const int32_t msize = (int32_t)(uint32_t)r.varint(32);
    if (!r.ok()) return;
    if (msize != 0) kv = r.read8();
    if (!r.ok()) return;
    if (msize < 0) return r.fail(TGPU_ERR_NEGATIVE_SIZE, off);
    if (r.container_limit && msize > r.container_limit) return r.fail(TGPU_ERR_SIZE_LIMIT, off);
    k = get_type(r, kv >> 4, off);
    v = get_type(r, kv & 0xf, off);
    size = msize;
  }
  static __device__ __forceinline__ void read_string(Reader& r, uint64_t& view, uint32_t& len) {
    const uint64_t off = r.pos;
    const int32_t size = (int32_t)(uint32_t)r.varint(32);
    if (!r.ok()) return;
    if (size < 0) return r.fail(TGPU_ERR_NEGATIVE_SIZE, off);
    if (r.string_limit > 0 && size > r.string_limit) return r.fail(TGPU_ERR_SIZE_LIMIT, off);
    if (size == 0) {
      view = 0;
      len = 0;
      return;
    }
    if (r.end - r.pos < (uint64_t)size) return r.fail(TGPU_ERR_TRUNCATED, r.pos);
    view = r.pos;
    len = (uint32_t)size;
    r.pos += (uint64_t)size;
  }
  static __device__ __forceinline__ uint32_t fixed_in_container(uint32_t t) {
    return (t == TGPU_T_BOOL || t == TGPU_T_BYTE) ? 1
           : t == TGPU_T_FLOAT                    ? 4
           : t == TGPU_T_DOUBLE                   ? 8
                                                  : 0;
  }
  static __device__ __forceinline__ bool skip_leaf(Reader& r, uint32_t t) {
    switch (t) {
      case TGPU_T_BOOL: read_bool(r); return true;
      case TGPU_T_BYTE: r.read8(); return true;
      case TGPU_T_I16: case TGPU_T_I32: r.varint(32); return true;
      case TGPU_T_U64: case TGPU_T_I64: r.varint(64); return true;
      case TGPU_T_DOUBLE: r.readBE(8); return true;
      case TGPU_T_FLOAT: r.readBE(4); return true;
      case TGPU_T_UTF8: case TGPU_T_UTF16: case TGPU_T_STRING: {
        uint64_t v;
        uint32_t l;
        read_string(r, v, l);
        return true;
      }
      default: return false;
    }
  }
  static __device__ __forceinline__ void read_scalar(Reader& r, uint32_t t, uint8_t* dst) {
    switch (t) {
      case TGPU_T_BOOL: { const uint32_t v = read_bool(r); if (r.ok()) *dst = (uint8_t)v; break; }
      case TGPU_T_BYTE: { const uint32_t v = r.read8(); if (r.ok()) *dst = (uint8_t)v; break; }
      case TGPU_T_I16: { const int16_t v = (int16_t)zz_to_i32((uint32_t)r.varint(32)); if (r.ok()) *(int16_t*)dst = v; break; }
      case TGPU_T_I32: { const int32_t v = zz_to_i32((uint32_t)r.varint(32)); if (r.ok()) *(int32_t*)dst = v; break; }
      case TGPU_T_I64: { const int64_t v = zz_to_i64(r.varint(64)); if (r.ok()) *(int64_t*)dst = v; break; }
      case TGPU_T_FLOAT: { const uint32_t v = (uint32_t)r.readBE(4); if (r.ok()) *(uint32_t*)dst = v; break; }
      default: { const uint64_t v = r.readBE(8); if (r.ok()) *(uint64_t*)dst = v; break; }
    }
  }
};

// ----------------------------------------------------------- Compact V1 ----
// CompactV1Protocol.h: the Compact reader with readDouble as readLE
// (CompactV1Protocol-inl.h:73-79); skip, sizes and everything else inherited.
template <>
struct Proto<TGPU_PROTOCOL_COMPACT_V1> : Proto<TGPU_PROTOCOL_COMPACT> {
  static __device__ __forceinline__ void read_scalar(Reader& r, uint32_t t, uint8_t* dst) {
    if (t == TGPU_T_DOUBLE) {
      const uint64_t v = __builtin_bswap64(r.readBE(8));
      if (r.ok()) *(uint64_t*)dst = v;
      return;
    }
    Proto<TGPU_PROTOCOL_COMPACT>::read_scalar(r, t, dst);
  }
};

// -------------------------------------------------------------------- skip --
// Iterative skip with an explicit frame stack (no recursion on the GPU).
// Frame kinds: struct (Binary: no delta; Compact: last field id), list/set
// (remaining elements), map (remaining pairs, key/value phase).
struct SkipFrame {
  uint8_t kind;  // 1 struct, 2 list, 3 map
  uint8_t t0, t1, phase;
  int32_t last_or_remaining;
  int32_t depth;  // depth of the values inside this frame
};
static_assert(sizeof(SkipFrame) == kSkipFrameBytes, "slab layout (tgpu_internal.h)");

// Frames live in the lane's private array, or all of them in the reader's
// HBM slab when it has one (deep-pass lanes). Running out of private frames
// is kErrDeep (the caller defers the record to the deep pass); out of slab
// frames (past kMaxDeepFrames) TGPU_ERR_UNSUPPORTED.
template <int P>
__device__ void skip(Reader& r, uint32_t type, int32_t depth) {
  using Pr = Proto<P>;
  SkipFrame priv[kMaxSkipDepth];
  SkipFrame* const st = r.deep ? (SkipFrame*)r.deep : priv;
  const uint64_t cap = r.deep ? r.deep_cap : (uint64_t)kMaxSkipDepth;
  const int32_t full = r.deep && !r.deep_more ? TGPU_ERR_UNSUPPORTED : kErrDeep;
  int sp = 0;
  uint32_t cur = type;
  int32_t cdepth = depth;
  bool have = true;  // a value of type `cur` at `cdepth` is to be skipped
  while (r.ok()) {
    if (have) {
      have = false;
      if (cdepth >= r.max_depth) return r.fail(TGPU_ERR_DEPTH_LIMIT, r.pos);
      if (!Pr::skip_leaf(r, cur)) {
        if (cur == TGPU_T_STRUCT) {
          r.descend(r.pos);  // readStructBegin
          if (!r.ok()) return;
          if ((uint64_t)sp >= cap) return r.fail(full, r.pos);
          st[sp++] = SkipFrame{1, 0, 0, 0, 0, cdepth + 1};
        } else if (cur == TGPU_T_LIST || cur == TGPU_T_SET || cur == TGPU_T_MAP) {
          uint32_t a = 0, b = 0;
          int32_t n = 0;
          const bool is_map = cur == TGPU_T_MAP;
          if (is_map) Pr::map_begin(r, a, b, n);
          else Pr::list_begin(r, a, n);
          if (!r.ok()) return;
          // skip_n(n, types, depth + 1) (Protocol.h:317-344)
          if (cdepth + 1 >= r.max_depth) return r.fail(TGPU_ERR_DEPTH_LIMIT, r.pos);
          const uint32_t fa = Pr::fixed_in_container(a);
          const uint32_t fb = is_map ? Pr::fixed_in_container(b) : 1;
          if (fa && fb) {
            const uint64_t sum = fa + (is_map ? fb : 0);
            r.skip_bytes(sum * (uint64_t)(uint32_t)n);
            r.ascend();
          } else {
            if ((uint64_t)sp >= cap) return r.fail(full, r.pos);
            st[sp++] = SkipFrame{(uint8_t)(is_map ? 3 : 2), (uint8_t)a, (uint8_t)b, 0, n,
                                 cdepth + 2};
          }
        } else {
          return r.fail(TGPU_ERR_INVALID_SKIP_TYPE, r.pos);
        }
      }
      continue;
    }
    if (sp == 0) return;
    SkipFrame& f = st[sp - 1];
    if (f.kind == 1) {
      uint32_t ft;
      int32_t fid = 0;
      if (P == TGPU_PROTOCOL_BINARY) {
        // BinaryProtocolReader::skip: readByte, STOP?, skipBytes(2)
        ft = r.read8();
        if (!r.ok()) return;
        if (ft == TGPU_T_STOP) {
          r.ascend();
          --sp;
          continue;
        }
        r.skip_bytes(2);
        if (!r.ok()) return;
      } else {
        if (!Pr::field_header(r, f.last_or_remaining, ft, fid)) {
          if (!r.ok()) return;
          r.ascend();
          --sp;
          continue;
        }
        f.last_or_remaining = fid;
      }
      cur = ft;
      cdepth = f.depth;
      have = true;
    } else {
      if (f.last_or_remaining == 0 && f.phase == 0) {
        r.ascend();
        --sp;
        continue;
      }
      if (f.kind == 2) {
        --f.last_or_remaining;
        cur = f.t0;
      } else {
        if (f.phase == 0) {
          --f.last_or_remaining;
          cur = f.t0;
          f.phase = 1;
        } else {
          cur = f.t1;
          f.phase = 0;
        }
      }
      cdepth = f.depth;
      have = true;
    }
  }
}

// ------------------------------------------------------------ struct read ---
// Stores in the widest units the alignment allows: the general reader's slots
// (records, arena elements, pairs) are 8-byte aligned with sizes that are
// mostly multiples of 8, and byte stores to them were its main cost (the
// nested leg's decode).
__device__ __forceinline__ void zero_bytes(uint8_t* p, uint32_t n) {
  uint32_t b = 0;
  if (((uintptr_t)p & 7) == 0)
    for (; b + 8 <= n; b += 8) *(uint64_t*)(p + b) = 0;
  for (; b < n; ++b) p[b] = 0;
}
// dst <- src for n bytes (src: a private buffer, 8-byte aligned).
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, uint32_t n) {
  uint32_t b = 0;
  const uintptr_t a = (uintptr_t)dst;
  if ((a & 7) == 0) {
    for (; b + 8 <= n; b += 8) *(uint64_t*)(dst + b) = *(const uint64_t*)(src + b);
  } else if ((a & 3) == 0) {
    for (; b + 4 <= n; b += 4) *(uint32_t*)(dst + b) = *(const uint32_t*)(src + b);
  }
  if (((a + b) & 1) == 0)
    for (; b + 2 <= n; b += 2) *(uint16_t*)(dst + b) = *(const uint16_t*)(src + b);
  for (; b < n; ++b) dst[b] = src[b];
}

// A container's element (list/set) or key/value (map) types, from a
// container field or from a type-table node (tgpu_type_desc).
struct CType {
  uint32_t ttype, elem, val;
  int32_t si;   // struct of the elements / values (T_STRUCT)
  uint32_t ti;  // 1 + type node of container elements / values
  uint32_t ki;  // map: 1 + type node of a struct / container key
};
__device__ __forceinline__ CType ctype_of(const tgpu_field_desc& f) {
  return CType{f.ttype, f.elem_ttype, f.val_ttype, f.struct_index, f.type_index, f.key_index};
}
__device__ __forceinline__ CType ctype_node(const DevSchema& sc, uint32_t ti) {
  const tgpu_type_desc t = sc.t[ti - 1];
  return CType{t.ttype, t.elem_ttype, t.val_ttype, t.struct_index, t.type_index, t.key_index};
}
__device__ __forceinline__ bool is_container(uint32_t t) {
  return t == TGPU_T_LIST || t == TGPU_T_SET || t == TGPU_T_MAP;
}
__device__ __forceinline__ bool is_complex(uint32_t t) {
  return t == TGPU_T_STRUCT || is_container(t);
}
// Bytes of one element / key / value in the arena.
__device__ __forceinline__ uint32_t slot_size(const DevSchema& sc, uint32_t t, int32_t si) {
  return t == TGPU_T_STRUCT ? sc.s[si].size : elem_size(t);
}

// Where containers put their elements (tgpu_schema_arena_scale):
//   position rule (schemas without nested containers): scale x the wire
//     position of the first element, so every slot is computable without a
//     scan;
//   record regions (nested schemas): each record's containers are allocated
//     in wire order from scale x its start, 8-byte aligned;
//   measure only (base null, cap kDiscardArena: the stream indexer): simple
//     containers are validated without storing; a container of structs or
//     containers reads each element into one reused slot per nesting level.
struct Arena {
  uint8_t* base;
  uint64_t cap;
  uint64_t scale;
  uint64_t bump;    // next free offset (record regions)
  bool regions;
  uint8_t* nest;    // measure only: the element slot every level shares
  uint32_t nest_slot;
  __device__ __forceinline__ bool discard() const { return !base && cap == kDiscardArena; }
  __device__ __forceinline__ uint64_t alloc(uint64_t first_elem_pos, uint64_t bytes) {
    if (!regions) return scale * first_elem_pos;
    const uint64_t o = bump;
    bump = (bump + bytes + 7) & ~7ull;
    return o;
  }
};

// One container element: a scalar, or a string as a span into the stream
// (the string field rule, Protocol.h:96-99).
template <int P>
__device__ __forceinline__ void read_elem(Reader& r, uint32_t t, uint8_t* dst) {
  if (t == TGPU_T_STRING) {
    uint64_t v = 0;
    uint32_t l = 0;
    Proto<P>::read_string(r, v, l);
    if (r.ok()) {
      const tgpu_span e{l ? v : 0, l, 0};
      copy_bytes(dst, (const uint8_t*)&e, 16);
    }
    return;
  }
  Proto<P>::read_scalar(r, t, dst);
}

// Arena slots of the position rule: scale x (wire position of the first
// element). Scalars need scale 1 (Binary) / 8 (Compact); 16-byte string
// spans from >= 4 (Binary) or >= 1 (Compact) wire bytes need 4 / 16.
template <int P>
__device__ __forceinline__ uint64_t arena_scale(const DevSchema& sc) {
  return sc.str_elems ? (P == TGPU_PROTOCOL_BINARY ? 4 : 16) : Proto<P>::kArenaScale;
}

__device__ __forceinline__ bool at_ok(uint64_t aoff, int32_t i, uint32_t es, uint64_t cap) {
  return aoff + ((uint64_t)i + 1) * es <= cap;
}

// protocol_methods<list>::read (protocol_methods.h:389-467) of scalar or
// string elements: the member is reset, a type mismatch skips the list
// (skip_n), canReadNElements, then the elements.
template <int P>
__device__ void read_list(Reader& r, const CType& c, uint8_t* m, Arena& A) {
  using Pr = Proto<P>;
  tgpu_span sp{0, 0, 0};
  *(tgpu_span*)m = sp;
  uint32_t reported = 0;
  int32_t n = 0;
  Pr::list_begin(r, reported, n);
  if (!r.ok()) return;
  if (reported != c.elem) {
    // skip_n(protocol, n, {reported}) with depth 0
    if (0 >= r.max_depth) return r.fail(TGPU_ERR_DEPTH_LIMIT, r.pos);
    const uint32_t fs = Pr::fixed_in_container(reported);
    if (fs) {
      r.skip_bytes((uint64_t)fs * (uint32_t)n);
    } else {
      for (int32_t i = 0; i < n && r.ok(); ++i) skip<P>(r, reported, 1);
    }
  } else {
    if (r.end - r.pos < (uint64_t)(uint32_t)n) return r.fail(TGPU_ERR_TRUNCATED, r.pos);
    const uint32_t es = elem_size(c.elem);
    if (n > 0 && A.discard()) {
      // measuring only (stream indexer): validate and consume, store nothing
      uint8_t tmp[16];
      for (int32_t i = 0; i < n && r.ok(); ++i) read_elem<P>(r, c.elem, tmp);
    } else if (n > 0) {
      if (!A.base) return r.fail(TGPU_ERR_OUTPUT_OVERFLOW, r.pos);
      uint8_t* arena = A.base;
      const uint64_t arena_cap = A.cap;
      const uint64_t aoff = A.alloc(r.pos, (uint64_t)(uint32_t)n * es);
      // the list is resized to n before the element reads
      sp.offset = aoff;
      sp.length = (uint32_t)n;
      *(tgpu_span*)m = sp;
      int32_t i = 0;
      for (; i < n; ++i) {
        // read first: a truncated stream fails as the reader does, and an
        // element that was read always fits an arena of the documented size
        const uint64_t at = aoff + (uint64_t)i * es;
        alignas(8) uint8_t tmp[16];
        read_elem<P>(r, c.elem, tmp);
        if (!r.ok()) break;
        if (at + es > arena_cap) {
          r.fail(TGPU_ERR_OUTPUT_OVERFLOW, r.pos);
          break;
        }
        copy_bytes(arena + at, tmp, es);
      }
      if (!r.ok()) {
        if (c.ttype == TGPU_T_SET) {
          // deserialize_known_length_set (EncodeHelpers.h:248-259): an element
          // is inserted once read — the set keeps the complete ones
          sp.length = (uint32_t)i;
          if (!i) sp.offset = 0;
          *(tgpu_span*)m = sp;
        } else if (c.elem == TGPU_T_STRING) {
          // non-trivial elements: reserve + emplace_back_default + read
          // (protocol_methods.h:374-386,458-461): the failing element is
          // in the list, empty (readString throws before assigning)
          if (at_ok(aoff, i, es, arena_cap)) zero_bytes(arena + aoff + (uint64_t)i * es, es);
          sp.length = (uint32_t)(i + 1);
          *(tgpu_span*)m = sp;
        } else {
          // leftover elements are value-initialized (protocol_methods.h:441-451)
          for (; i < n; ++i) {
            const uint64_t at = aoff + (uint64_t)i * es;
            if (at + es > arena_cap) break;
            zero_bytes(arena + at, es);
          }
        }
      }
    }
  }
  if (r.ok()) r.ascend();
}

// protocol_methods<map>::read (protocol_methods.h:640-677) of scalar or string
// keys and values: reset to empty, readMapBegin, skip_n on a key/value type
// mismatch of a non-empty map, canReadNElements(n, {k, v}) = n * 2 bytes
// left, then the pairs in wire order, packed {key, value}. A failing pair is
// not inserted (EncodeHelpers.h:188-205): the map keeps the pairs before it.
// Pair i's slot ends within scale x (the end of pair i on the wire), so a
// pair that was read always fits an arena of the documented size.
template <int P>
__device__ void read_map(Reader& r, const CType& c, uint8_t* m, Arena& A) {
  using Pr = Proto<P>;
  tgpu_span sp{0, 0, 0};
  *(tgpu_span*)m = sp;
  uint32_t rk = 0, rv = 0;
  int32_t n = 0;
  Pr::map_begin(r, rk, rv, n);
  if (!r.ok()) return;
  if (n > 0 && (rk != c.elem || rv != c.val)) {
    // skip_n(protocol, n, {k, v}) with depth 0 (Protocol.h:317-344)
    if (0 >= r.max_depth) return r.fail(TGPU_ERR_DEPTH_LIMIT, r.pos);
    const uint32_t fk = Pr::fixed_in_container(rk), fv = Pr::fixed_in_container(rv);
    if (fk && fv) {
      r.skip_bytes((uint64_t)(fk + fv) * (uint32_t)n);
    } else {
      for (int32_t i = 0; i < n && r.ok(); ++i) {
        skip<P>(r, rk, 1);
        if (r.ok()) skip<P>(r, rv, 1);
      }
    }
  } else {
    if ((r.end - r.pos) / 2 < (uint64_t)(uint32_t)n) return r.fail(TGPU_ERR_TRUNCATED, r.pos);
    const uint32_t ks = elem_size(c.elem), ps = ks + elem_size(c.val);
    const bool discard = A.discard();
    if (n > 0 && !A.base && !discard) return r.fail(TGPU_ERR_OUTPUT_OVERFLOW, r.pos);
    const uint64_t aoff = (n > 0 && !discard) ? A.alloc(r.pos, (uint64_t)(uint32_t)n * ps) : 0;
    int32_t i = 0;
    for (; i < n; ++i) {
      alignas(8) uint8_t pr[32];
      read_elem<P>(r, c.elem, pr);
      if (!r.ok()) break;
      read_elem<P>(r, c.val, pr + ks);
      if (!r.ok()) break;
      if (discard) continue;
      const uint64_t at = aoff + (uint64_t)i * ps;
      if (at + ps > A.cap) {
        r.fail(TGPU_ERR_OUTPUT_OVERFLOW, r.pos);
        break;
      }
      copy_bytes(A.base + at, pr, ps);
    }
    if (i > 0 && !discard) {
      sp.offset = aoff;
      sp.length = (uint32_t)i;
      *(tgpu_span*)m = sp;
    }
  }
  if (r.ok()) r.ascend();
}

// The record reader: the generated readNoXfer (deserialize_struct.whisker:
// 19-160) as an explicit frame machine. Frames: a struct being read field by
// field; a list/set whose elements are structs or containers; a map whose
// keys or values are. Their element semantics are the reference's:
//   list  reserve + emplace_back_default + read (protocol_methods.h:374-386,
//         458-461): the list holds the elements read plus the failing one;
//   set   an element is inserted once read (EncodeHelpers.h:248-259);
//   map   a pair is inserted once key and value are read (:188-205).
// A boxed struct field (cpp.ref / thrift.box) is read into a fresh object in
// the arena and pointed to once its read completed (deserialize_field.
// whisker:21-23,49-51).
enum : uint8_t { RF_STRUCT = 1, RF_LIST = 2, RF_MAP = 3 };
// kphase of a list/map frame: the element / pair at i is
enum : uint8_t { KP_NEXT = 0, KP_KEY_OPEN = 1, KP_VALUE = 2, KP_VALUE_OPEN = 3 };
struct ReadFrame {
  uint8_t kind;
  uint8_t is_set;
  uint8_t etype;   // list: element type; map: value type
  uint8_t ktype;   // map: key type
  uint8_t kphase;  // list/map: KP_*
  uint8_t pad_[3];
  int32_t si;      // struct: its index; list/map: struct of the elements / values
  uint32_t ti;     // list/map: type node of container elements / values
  uint8_t* obj;    // struct: the object; list/map: element array
  // struct
  int32_t prev;      // Compact delta base
  uint32_t fidx;     // field whose struct / container value is open
  uint32_t nread;    // fields read or skipped (a union takes one)
  uint32_t pad2_;
  uint64_t seen;     // fields (index < 64) read by this read (required check)
  // list/map
  uint32_t n, i;     // elements, elements done
  uint32_t es, ks;   // element (pair) stride in the arena, key bytes
  int32_t ksi;       // map: struct of struct keys
  uint32_t kti;      // map: type node of container keys
  uint8_t* span;   // list/map: the member / element span being filled
};

__device__ __forceinline__ void set_span_len(uint8_t* m, uint8_t* arr, uint8_t* base, uint32_t len) {
  tgpu_span sp{len ? (uint64_t)(arr - base) : 0, len, 0};
  *(tgpu_span*)m = sp;
}

__device__ __forceinline__ bool boxed(const tgpu_field_desc& f) {
  return f.qualifier == TGPU_BOXED || f.qualifier == TGPU_OPTIONAL_BOXED;
}

// A list frame holding a boxed struct field's object (is_set value).
constexpr uint8_t kBoxedFrame = 2;

// Child value of frame p is complete (and the reader ok).
__device__ __forceinline__ void child_done(const DevSchema& sc, ReadFrame& p, const Arena& A) {
  if (p.kind == RF_STRUCT) {
    const tgpu_field_desc f = sc.f[p.fidx];
    p.obj[f.isset_offset] = 1;  // __isset.set(idx, true)
    const uint32_t k = p.fidx - sc.s[p.si].first_field;
    if (k < 64) p.seen |= 1ull << k;
  } else if (p.kphase == KP_KEY_OPEN) {
    p.kphase = KP_VALUE;
  } else {
    ++p.i;
    p.kphase = KP_NEXT;
    if (p.kind == RF_MAP || p.is_set) set_span_len(p.span, p.obj, A.base, p.i);
  }
}

// Opens the container value of type c at member / element slot m: simple
// elements are read here (returns true: done), elements, keys or values that
// are structs or containers get a frame (returns false).
template <int P>
__device__ bool open_container(Reader& r, const DevSchema& sc, const CType& c, uint8_t* m,
                               Arena& A, ReadFrame& f) {
  using Pr = Proto<P>;
  const bool is_map = c.ttype == TGPU_T_MAP;
  const uint32_t et = is_map ? c.val : c.elem;
  if (!is_complex(et) && !(is_map && is_complex(c.elem))) {
    if (is_map) read_map<P>(r, c, m, A);
    else read_list<P>(r, c, m, A);
    return true;
  }
  *(tgpu_span*)m = tgpu_span{0, 0, 0};  // reset (deserialize_field.whisker:44-47)
  uint32_t rk = 0, rv = 0;
  int32_t n = 0;
  if (is_map) Pr::map_begin(r, rk, rv, n);
  else Pr::list_begin(r, rv, n);
  if (!r.ok()) return true;
  const bool mismatch = is_map ? (n > 0 && (rk != c.elem || rv != c.val)) : rv != c.elem;
  if (mismatch) {
    if (0 >= r.max_depth) {
      r.fail(TGPU_ERR_DEPTH_LIMIT, r.pos);
      return true;
    }
    for (int32_t i = 0; i < n && r.ok(); ++i) {
      if (is_map) skip<P>(r, rk, 1);
      if (r.ok()) skip<P>(r, rv, 1);
    }
    if (r.ok()) r.ascend();
    return true;
  }
  if ((r.end - r.pos) / (is_map ? 2 : 1) < (uint64_t)(uint32_t)n) {
    r.fail(TGPU_ERR_TRUNCATED, r.pos);
    return true;
  }
  if (n == 0) {
    r.ascend();
    return true;
  }
  int32_t ksi = -1;
  uint32_t kti = 0;
  if (is_map && is_complex(c.elem)) {
    if (c.elem == TGPU_T_STRUCT) ksi = sc.t[c.ki - 1].struct_index;
    else kti = c.ki;
  }
  const uint32_t ks = is_map ? slot_size(sc, c.elem, ksi) : 0;
  const uint32_t es = ks + slot_size(sc, et, c.si);
  uint8_t* arr;
  uint32_t stride = es;
  if (A.discard()) {
    arr = A.nest;  // one slot every level reuses (the measuring reads only write)
    stride = 0;
  } else {
    if (!A.base) {
      r.fail(TGPU_ERR_OUTPUT_OVERFLOW, r.pos);
      return true;
    }
    const uint64_t bytes = (uint64_t)(uint32_t)n * es;
    const uint64_t aoff = A.alloc(r.pos, bytes);
    if (aoff + bytes > A.cap) {
      r.fail(TGPU_ERR_OUTPUT_OVERFLOW, r.pos);
      return true;
    }
    arr = A.base + aoff;
  }
  f.kind = is_map ? RF_MAP : RF_LIST;
  f.is_set = c.ttype == TGPU_T_SET;
  f.etype = (uint8_t)et;
  f.ktype = (uint8_t)c.elem;
  f.kphase = KP_NEXT;
  f.si = c.si;
  f.ti = c.ti;
  f.n = (uint32_t)n;
  f.i = 0;
  f.es = stride;
  f.ks = ks;
  f.ksi = ksi;
  f.kti = kti;
  f.obj = arr;
  f.span = m;
  return false;
}

__device__ __forceinline__ ReadFrame struct_frame(int32_t si, uint8_t* obj) {
  ReadFrame f;
  f.kind = RF_STRUCT;
  f.is_set = 0;
  f.etype = f.ktype = f.kphase = 0;
  f.si = si;
  f.ti = 0;
  f.obj = obj;
  f.prev = 0;
  f.nread = 0;
  f.fidx = 0;
  f.pad2_ = 0;
  f.seen = 0;
  f.n = f.i = f.es = f.ks = f.kti = 0;
  f.ksi = -1;
  f.span = nullptr;
  return f;
}

// The frames a reader keeps: kPrivFrames in the lane's private array, or (a
// deep-pass lane, r.deep set) all of them in its HBM slab after its skip
// frames. Running out of private frames is kErrDeep (the record is redone by
// the deep pass), out of slab frames TGPU_ERR_UNSUPPORTED.
__device__ __forceinline__ ReadFrame* slab_read_frames(const Reader& r) {
  return (ReadFrame*)(r.deep + slab_skip_bytes(r.deep_cap));
}

// Reads one record into rec (zeroed by the caller). A.bump: the record's
// region start when A.regions. The open frame `fr` lives in registers; the
// frames below it are saved in `st` (sp of them) only while a child is open
// (a per-iteration reload of the whole frame from scratch was the general
// reader's main cost).
// kDeep: the reader has an HBM slab (r.deep): every frame there (a
// compile-time choice, so the bulk kernels keep theirs in scratch).
template <int P, bool kDeep = false>
__device__ void read_record(Reader& r, const DevSchema& sc, uint8_t* rec, Arena& A) {
  using Pr = Proto<P>;
  ReadFrame priv[kDeep ? 1 : kPrivFrames];
  ReadFrame* const st = kDeep ? slab_read_frames(r) : priv;
  const uint32_t cap = kDeep ? (uint32_t)r.deep_cap : (uint32_t)kPrivFrames;
  const int32_t full = kDeep && !r.deep_more ? TGPU_ERR_UNSUPPORTED : kErrDeep;
  uint32_t sp = 0;  // frames saved below fr
  ReadFrame fr = struct_frame(0, rec);
  while (r.ok()) {
    if (fr.kind != RF_STRUCT) {
      uint8_t* val;
      if (fr.kphase == KP_NEXT) {
        if (fr.i == fr.n) {  // readListEnd / readMapEnd
          if (fr.is_set != kBoxedFrame) r.ascend();
          if (sp == 0) return;
          fr = st[--sp];
          child_done(sc, fr, A);
          continue;
        }
        const uint32_t esz = fr.es ? fr.es : (fr.ks + slot_size(sc, fr.etype, fr.si));
        uint8_t* el = fr.obj + (uint64_t)fr.i * fr.es;
        zero_bytes(el, esz);  // a default-constructed element / pair
        val = el;
        if (fr.kind == RF_MAP) {
          if (!is_complex(fr.ktype)) {
            read_elem<P>(r, fr.ktype, el);
            if (!r.ok()) break;
          } else {  // a struct / container key: its own frame, the value after it
            if (sp >= cap) return r.fail(full, r.pos);
            fr.kphase = KP_KEY_OPEN;
            if (fr.ktype == TGPU_T_STRUCT) {
              st[sp++] = fr;
              fr = struct_frame(fr.ksi, el);
            } else {
              ReadFrame nf;
              if (open_container<P>(r, sc, ctype_node(sc, fr.kti), el, A, nf)) {
                if (r.ok()) child_done(sc, fr, A);
              } else {
                st[sp++] = fr;
                fr = nf;
              }
            }
            continue;
          }
          val = el + fr.ks;
        } else if (!fr.is_set) {
          set_span_len(fr.span, fr.obj, A.base, fr.i + 1);  // emplace_back_default
        }
      } else {  // KP_VALUE: the key of pair i is read
        val = fr.obj + (uint64_t)fr.i * fr.es + fr.ks;
      }
      if (!is_complex(fr.etype)) {  // (a map with a struct / container key)
        read_elem<P>(r, fr.etype, val);
        if (!r.ok()) break;
        fr.kphase = KP_VALUE_OPEN;
        child_done(sc, fr, A);
        continue;
      }
      if (sp >= cap) return r.fail(full, r.pos);
      fr.kphase = KP_VALUE_OPEN;
      if (fr.etype == TGPU_T_STRUCT) {
        st[sp++] = fr;
        fr = struct_frame(fr.si, val);
      } else {
        ReadFrame nf;
        if (open_container<P>(r, sc, ctype_node(sc, fr.ti), val, A, nf)) {
          if (r.ok()) child_done(sc, fr, A);
        } else {
          st[sp++] = fr;
          fr = nf;
        }
      }
      continue;
    }
    const tgpu_struct_desc sd = sc.s[fr.si];
    const bool un = sd.flags & TGPU_STRUCT_UNION;
    uint32_t wt = 0;
    int32_t id = 0;
    if (!Pr::field_header(r, fr.prev, wt, id)) {
      if (!r.ok()) return;
      // a union with no field is cleared (deserialize_union.whisker:26-28)
      if (un && fr.nread == 0) zero_bytes(fr.obj, sd.size);
      // deprecated_enforce_required: every required field read by this
      // read, checked after readStructEnd (deserialize_struct.whisker:116-124)
      if (sd.flags & TGPU_STRUCT_ENFORCE_REQUIRED) {
        for (uint32_t k = 0; k < sd.num_fields && k < 64; ++k)
          if (sc.f[sd.first_field + k].qualifier == TGPU_REQUIRED && !((fr.seen >> k) & 1))
            return r.fail(TGPU_ERR_MISSING_REQUIRED_FIELD, r.pos);
      }
      // STOP: struct done
      if (sp == 0) return;
      fr = st[--sp];
      child_done(sc, fr, A);
      continue;
    }
    // a union's one field must be followed by STOP (throwUnionMissingStop)
    if (un && fr.nread) return r.fail(TGPU_ERR_UNION_MISSING_STOP, r.pos);
    ++fr.nread;
    fr.prev = id;
    // the expected field first (fields in declaration order: the generated
    // reader's fast path), then a scan
    int32_t hit = -1;
    {
      const uint32_t guess = fr.fidx ? fr.fidx + 1 - sd.first_field : 0;
      if (guess < sd.num_fields && sc.f[sd.first_field + guess].id == id) {
        hit = (int32_t)(sd.first_field + guess);
      } else {
        for (uint32_t k = 0; k < sd.num_fields; ++k) {
          if (sc.f[sd.first_field + k].id == id) {
            hit = (int32_t)(sd.first_field + k);
            break;
          }
        }
      }
    }
    if (hit < 0 || sc.f[hit].ttype != wt) {
      skip<P>(r, wt, 0);
      continue;
    }
    const tgpu_field_desc f = sc.f[hit];
    uint8_t* m = fr.obj + f.member_offset;
    fr.fidx = (uint32_t)hit;
    if (un) {  // field_ref().emplace(): a fresh member becomes active
      zero_bytes(fr.obj, sd.size);
      fr.obj[f.isset_offset] = 1;
    }
    if (is_scalar(f.ttype)) {
      Pr::read_scalar(r, f.ttype, m);
    } else if (f.ttype == TGPU_T_STRING) {
      uint64_t v = 0;
      uint32_t l = 0;
      Pr::read_string(r, v, l);
      if (r.ok()) *(tgpu_span*)m = tgpu_span{l ? v : 0, l, 0};
    } else if (f.ttype == TGPU_T_STRUCT) {
      if (sp >= cap) return r.fail(full, r.pos);
      st[sp++] = fr;
      if (boxed(f)) {
        // make_mutable_smart_ptr: a fresh object in the arena, read as the
        // one element of a frame that points the member to it once read (a
        // set's insert-after-read; no list header, so no height)
        const uint32_t size = sc.s[f.struct_index].size;
        uint8_t* obj;
        if (A.discard()) {
          obj = A.nest;
        } else {
          if (!A.base) return r.fail(TGPU_ERR_OUTPUT_OVERFLOW, r.pos);
          const uint64_t aoff = A.alloc(r.pos, size);
          if (aoff + size > A.cap) return r.fail(TGPU_ERR_OUTPUT_OVERFLOW, r.pos);
          obj = A.base + aoff;
        }
#ifdef TGPU_BOXED_DIRECT  // diagnosis only: the round-3 direct form
        if (!A.discard()) {
          zero_bytes(obj, size);
          *(tgpu_span*)m = tgpu_span{(uint64_t)(obj - A.base), 1, 0};
        }
        fr = struct_frame(f.struct_index, obj);
        continue;
#endif
        fr.kind = RF_LIST;
        fr.is_set = kBoxedFrame;
        fr.etype = TGPU_T_STRUCT;
        fr.ktype = 0;
        fr.kphase = KP_NEXT;
        fr.si = f.struct_index;
        fr.ti = 0;
        fr.obj = obj;
        fr.n = 1;
        fr.i = 0;
        fr.es = A.discard() ? 0 : size;
        fr.ks = 0;
        fr.ksi = -1;
        fr.kti = 0;
        fr.span = m;
        continue;
      }
      fr = struct_frame(f.struct_index, m);
      continue;  // isset set when the nested STOP is reached
    } else {
      if (sp >= cap) return r.fail(full, r.pos);
      ReadFrame nf;
      if (!open_container<P>(r, sc, ctype_of(f), m, A, nf)) {
        st[sp++] = fr;
        fr = nf;
        continue;
      }
    }
    if (r.ok()) {
      fr.obj[f.isset_offset] = 1;
      const uint32_t k = (uint32_t)hit - sd.first_field;
      if (k < 64) fr.seen |= 1ull << k;
    }
  }
}

// The schema tables in LDS: the general reader and writer look a struct /
// field / type descriptor up on every field, element and header — dependent
// loads on each lane's critical path, cheaper from LDS than from the caches.
// Copies by the whole workgroup (the caller barriers before use); returns sc
// itself when the tables do not fit `cap` bytes.
__device__ __forceinline__ uint32_t schema_lds_bytes(const DevSchema& sc) {
  return sc.ns * (uint32_t)sizeof(tgpu_struct_desc) + sc.nf * (uint32_t)sizeof(tgpu_field_desc) +
         sc.nt * (uint32_t)sizeof(tgpu_type_desc);
}
__device__ __forceinline__ DevSchema stage_schema(const DevSchema& sc, uint32_t* lds, uint32_t cap) {
  const uint32_t bs = sc.ns * (uint32_t)sizeof(tgpu_struct_desc);
  const uint32_t bf = sc.nf * (uint32_t)sizeof(tgpu_field_desc);
  const uint32_t bt = sc.nt * (uint32_t)sizeof(tgpu_type_desc);
  if (bs + bf + bt > cap) return sc;
  const uint32_t* src[3] = {(const uint32_t*)sc.s, (const uint32_t*)sc.f, (const uint32_t*)sc.t};
  const uint32_t words[3] = {bs / 4, bf / 4, bt / 4};
  uint32_t at = 0;
  for (int k = 0; k < 3; ++k) {
    for (uint32_t w = threadIdx.x; w < words[k]; w += blockDim.x) lds[at + w] = src[k][w];
    at += words[k];
  }
  DevSchema d = sc;
  d.s = (const tgpu_struct_desc*)lds;
  d.f = (const tgpu_field_desc*)(lds + bs / 4);
  d.t = (const tgpu_type_desc*)(lds + (bs + bf) / 4);
  return d;
}

// read_record with the reader's frames: its slab when it has one.
template <int P>
__device__ __forceinline__ void read_record_any(Reader& r, const DevSchema& sc, uint8_t* rec,
                                                Arena& A) {
  if (r.deep) read_record<P, true>(r, sc, rec, A);
  else read_record<P, false>(r, sc, rec, A);
}

// The arena of one record read: the position rule, or the record's region
// (scale x its start) for nested schemas; `nest` = per-level element slots
// when measuring only.
template <int P>
__device__ __forceinline__ Arena record_arena(const DevSchema& sc, uint8_t* base, uint64_t cap,
                                             uint64_t start, uint8_t* nest) {
  Arena A;
  A.base = base;
  A.cap = cap;
  A.regions = sc.bump_scale != 0;
  A.scale = A.regions ? sc.bump_scale : arena_scale<P>(sc);
  A.bump = A.regions ? sc.bump_scale * start : 0;
  A.nest = nest;
  A.nest_slot = sc.nest_slot;
  return A;
}

// ---------------------------------------------------------- deep passes ----
// Lane `lane`'s HBM skip frames (DeepArgs), attached to a reader.
__device__ __forceinline__ void attach_slab(Reader& r, const DeepArgs& d, uint32_t lane) {
  if (!d.slabs) return;
  r.deep = d.slabs + (uint64_t)lane * slab_lane_bytes(d.slab_frames);
  r.deep_cap = d.slab_frames;
  r.deep_more = d.more != 0;
}

// A lane whose reader failed: a value nested past its private skip frames
// defers item i to the deep pass; any other error is a real one.
__device__ __forceinline__ void defer_or_fail(const Reader& r, const DeepArgs& d,
                                              unsigned long long* first_fail, uint64_t i) {
  if (r.err == kErrDeep) d.list[atomicAdd(d.count, 1ull)] = i;
  else atomicMin(first_fail, (unsigned long long)i);
}

// Record i of an indexed stream, zeroed and then read (one readNoXfer into a
// default-constructed T); the reader comes back with any error latched.
// lane >= 0: the deep-pass lane whose HBM frames the skip may use.
// (start: the record's position; kIndexed: a.offs[i], checked as below)
constexpr uint64_t kIndexed = ~0ull;
// src (optional): an LDS copy of stream bytes [base, end) to read from.
template <int P>
__device__ Reader decode_record(const DecodeArgs& a, uint64_t i, int lane,
                                uint64_t at = kIndexed, const uint8_t* src = nullptr,
                                uint64_t base = 0, uint64_t end = 0) {
  uint8_t* rec = a.recs + i * a.rec_size;
  if ((a.rec_size & 7) == 0) {
    for (uint32_t b = 0; b < a.rec_size; b += 8) *(uint64_t*)(rec + b) = 0;
  } else {
    for (uint32_t b = 0; b < a.rec_size; ++b) rec[b] = 0;
  }
  const bool indexed = at == kIndexed;
  const uint64_t start = indexed ? a.offs[i] : at;
  Reader r = make_reader(src ? src : a.in, start, src ? end : a.in_len, a.string_limit,
                         a.container_limit, a.max_depth, a.height);
  if (src) {
    r.base = base;
    if (start < base || start > end) {  // not inside the copy: the caller reads HBM
      r.fail(TGPU_ERR_UNDERFLOW, start);
      return r;
    }
  }
  if (lane >= 0) attach_slab(r, a.deep, (uint32_t)lane);
  // (one read_record call site: each inlined copy carries its own frames)
  if (start > a.in_len || (indexed && a.check_index && a.offs[i + 1] < start)) {
    r.fail(indexed ? TGPU_ERR_INDEX_MISMATCH : TGPU_ERR_UNDERFLOW, start);
    return r;
  }
  Arena A = record_arena<P>(a.sc, a.arena, a.arena_cap, start, nullptr);
  if (lane >= 0 && r.deep) read_record<P, true>(r, a.sc, rec, A);
  else read_record<P, false>(r, a.sc, rec, A);
  if (indexed && r.ok() && a.check_index && r.pos != a.offs[i + 1])
    r.fail(TGPU_ERR_INDEX_MISMATCH, r.pos);
  return r;
}

// ------------------------------------------------------------------ writer --
struct Writer {
  uint8_t* out;  // nullptr: size only
  uint64_t pos, cap;
  int32_t err;
  uint64_t err_off;
  // record frames past the private kPrivFrames (nullptr: kErrDeep instead):
  // a deep-pass lane's HBM slab (the reader's layout)
  uint8_t* deep = nullptr;
  uint64_t deep_cap = 0;
  bool deep_more = false;  // the wide tier's slab: full is kErrDeep
  __device__ __forceinline__ bool ok() const { return err == 0; }
  __device__ __forceinline__ void fail(int32_t code, uint64_t off) {
    if (!err) {
      err = code;
      err_off = off;
    }
  }
  __device__ __forceinline__ void put(uint32_t b) {
    if (err) return;  // never write past the byte that failed validation
    if (out) out[pos] = (uint8_t)b;
    ++pos;
  }
  __device__ __forceinline__ void put_be(uint64_t v, uint32_t n) {
    for (int i = (int)n - 1; i >= 0; --i) put((uint32_t)(v >> (8 * i)));
  }
  __device__ __forceinline__ void varint(uint64_t v) {
    while (v & ~0x7full) {
      put((uint32_t)((v & 0x7f) | 0x80));
      v >>= 7;
    }
    put((uint32_t)v);
  }
  __device__ __forceinline__ void bytes(const uint8_t* src, uint32_t n) {
    if (out) for (uint32_t i = 0; i < n; ++i) out[pos + i] = src[i];
    pos += n;
  }
};

__device__ __forceinline__ uint32_t load_bool(Writer& w, const uint8_t* p) {
  const uint32_t b = *p;
  if (b > 1) w.fail(TGPU_ERR_INVALID_BOOL_WRITE, w.pos);  // validate_bool
  return b;
}

template <int P>
__device__ __forceinline__ void write_scalar(Writer& w, uint32_t t, const uint8_t* p) {
  if (P == TGPU_PROTOCOL_BINARY) {
    switch (t) {
      case TGPU_T_BOOL: w.put(load_bool(w, p)); break;
      case TGPU_T_BYTE: w.put(*p); break;
      case TGPU_T_I16: w.put_be(*(const uint16_t*)p, 2); break;
      case TGPU_T_I32: case TGPU_T_FLOAT: w.put_be(*(const uint32_t*)p, 4); break;
      default: w.put_be(*(const uint64_t*)p, 8); break;
    }
  } else {
    switch (t) {
      case TGPU_T_BOOL: w.put(load_bool(w, p) ? 1 : 2); break;
      case TGPU_T_BYTE: w.put(*p); break;
      case TGPU_T_I16: w.varint(i32_to_zz(*(const int16_t*)p)); break;
      case TGPU_T_I32: w.varint(i32_to_zz(*(const int32_t*)p)); break;
      case TGPU_T_I64: w.varint(i64_to_zz(*(const int64_t*)p)); break;
      case TGPU_T_FLOAT: w.put_be(*(const uint32_t*)p, 4); break;
      default:  // double: BE, CompactV1 LE (CompactV1Protocol-inl.h:36-41)
        if (P == TGPU_PROTOCOL_COMPACT_V1) w.put_be(__builtin_bswap64(*(const uint64_t*)p), 8);
        else w.put_be(*(const uint64_t*)p, 8);
        break;
    }
  }
}

// One container element: a scalar, or a string span into string_base.
template <int P>
__device__ __forceinline__ void write_elem(Writer& w, uint32_t t, const uint8_t* p,
                                           const uint8_t* sbase) {
  if (t != TGPU_T_STRING) return write_scalar<P>(w, t, p);
  tgpu_span e;
  if (((uintptr_t)p & 7) == 0) {
    e = *(const tgpu_span*)p;
  } else {
    uint8_t* b = (uint8_t*)&e;
    for (uint32_t k = 0; k < 16; ++k) b[k] = p[k];
  }
  if (e.length > 0x7fffffffu) return w.fail(TGPU_ERR_WRITE_SIZE_LIMIT, w.pos);  // checkBinarySize
  if (P == TGPU_PROTOCOL_BINARY) w.put_be(e.length, 4);
  else w.varint(e.length);
  w.bytes(sbase + e.offset, e.length);
}

// op::isEmpty of a terse member (Clear.h:98-127): scalars by identity with
// the intrinsic default (all bits zero), strings/containers by length,
// structs by thrift::empty (below).
__device__ __forceinline__ bool terse_leaf_empty(const tgpu_field_desc& f, const uint8_t* m) {
  if (is_scalar(f.ttype)) {
    uint32_t any = 0;
    for (uint32_t b = 0; b < scalar_size(f.ttype); ++b) any |= m[b];
    return any == 0;
  }
  return ((const tgpu_span*)m)->length == 0;
}

// thrift::empty of struct si at obj — the generated __fbthrift_is_empty
// (module_types_cpp/declare_members.whisker:83-113): never empty with an
// unqualified, required or boxed-unqualified field; otherwise empty when no
// optional field is set and every terse field is empty (terse structs
// recursively); a union (union_declare_members.whisker:43-45) when no member
// is active. The walk keeps one (struct, object, next field) per terse
// struct level (schemas nest those at most kMaxTerseDepth deep).
constexpr int kMaxTerseDepth = 16;
__device__ bool struct_empty(const DevSchema& sc, uint32_t si, const uint8_t* obj) {
  struct Lvl {
    uint32_t si, k;
    const uint8_t* obj;
  } st[kMaxTerseDepth + 1];
  int sp = 0;
  st[0] = Lvl{si, 0, obj};
  for (;;) {
    Lvl& L = st[sp];
    const tgpu_struct_desc sd = sc.s[L.si];
    if (L.k >= sd.num_fields) {  // this level is empty
      if (sp == 0) return true;
      --sp;
      continue;
    }
    const tgpu_field_desc f = sc.f[sd.first_field + L.k++];
    if (sd.flags & TGPU_STRUCT_UNION) {
      if (L.obj[f.isset_offset]) return false;
      continue;
    }
    if (f.qualifier == TGPU_UNQUALIFIED || f.qualifier == TGPU_REQUIRED ||
        f.qualifier == TGPU_BOXED)
      return false;
    if (f.qualifier == TGPU_OPTIONAL || f.qualifier == TGPU_OPTIONAL_BOXED) {
      if (L.obj[f.isset_offset]) return false;
      continue;
    }
    const uint8_t* m = L.obj + f.member_offset;  // terse
    if (f.ttype == TGPU_T_STRUCT) {
      if (sp >= kMaxTerseDepth) return false;  // (validated: never reached)
      st[++sp] = Lvl{(uint32_t)f.struct_index, 0, m};
      continue;
    }
    if (!terse_leaf_empty(f, m)) return false;
  }
}

__device__ __forceinline__ bool terse_empty(const DevSchema& sc, const tgpu_field_desc& f,
                                            const uint8_t* m) {
  return f.ttype == TGPU_T_STRUCT ? struct_empty(sc, (uint32_t)f.struct_index, m)
                                  : terse_leaf_empty(f, m);
}

// The record writer: the generated write (serialize_struct.whisker:40-67,
// serialize_field.whisker:17-71) as an explicit frame machine — a struct's
// fields in declaration order, and lists/sets/maps whose elements, keys or
// values are structs or containers element by element.
enum : uint8_t { WF_STRUCT = 1, WF_LIST = 2, WF_MAP = 3 };
struct WriteFrame {
  uint8_t kind;
  uint8_t etype;   // list: element type; map: value type
  uint8_t ktype;   // map: key type
  uint8_t kphase;  // list/map: 0 = element k next, 1 = its value next (key written)
  uint32_t si;     // struct: its index; list/map: struct of the elements / values
  uint32_t ti;     // list/map: type node of container elements / values
  uint32_t k;      // struct: next field index; list/map: next element
  int32_t last;    // struct: Compact lastFieldId_
  uint32_t end;    // struct: one past the last field to write; list/map: elements
  uint32_t es, ks;
  int32_t ksi;     // map: struct of struct keys
  uint32_t kti;    // map: type node of container keys
  const uint8_t* obj;
};

// The fields a struct writes: all of them, or for a union its active member
// only (serialize_union.whisker:52-66): the first whose isset byte is set.
__device__ __forceinline__ WriteFrame write_frame(const DevSchema& sc, uint32_t si,
                                                  const uint8_t* obj) {
  const tgpu_struct_desc sd = sc.s[si];
  WriteFrame w{};
  w.kind = WF_STRUCT;
  w.si = si;
  w.obj = obj;
  w.end = sd.num_fields;
  if (sd.flags & TGPU_STRUCT_UNION) {
    w.k = sd.num_fields;
    for (uint32_t k = 0; k < sd.num_fields; ++k) {
      if (obj[sc.f[sd.first_field + k].isset_offset]) {
        w.k = k;
        w.end = k + 1;
        break;
      }
    }
  }
  return w;
}

// writeListBegin / writeSetBegin / writeMapBegin (BinaryProtocol-inl.h:69-96,
// CompactProtocol-inl.h:182-246) of a container value with `n` elements.
template <int P>
__device__ __forceinline__ void container_header(Writer& w, const CType& c, uint32_t n) {
  if (c.ttype == TGPU_T_MAP) {
    if (P == TGPU_PROTOCOL_BINARY) {
      w.put(c.elem);
      w.put(c.val);
      w.put_be(n, 4);
    } else if (n == 0) {
      w.put(0);
    } else {
      w.varint(n);
      w.put((ttype_to_ctype(c.elem) << 4) | ttype_to_ctype(c.val));
    }
  } else if (P == TGPU_PROTOCOL_BINARY) {
    w.put(c.elem);
    w.put_be(n, 4);
  } else {
    const uint32_t ct = ttype_to_ctype(c.elem);
    if (n <= 14) {
      w.put((n << 4) | ct);
    } else {
      w.put(0xf0 | ct);
      w.varint(n);
    }
  }
}

// Writes the container value of type c held in span member m: simple
// elements here (returns true), a container whose elements, keys or values
// are structs / containers gets a frame (returns false).
template <int P>
__device__ __forceinline__ bool write_container(Writer& w, const DevSchema& sc, const CType& c,
                                const uint8_t* m, const uint8_t* sbase, const uint8_t* lbase,
                                WriteFrame* st, uint32_t& sp, uint32_t cap, int32_t full) {
  const tgpu_span sp_ = *(const tgpu_span*)m;
  // checked_container_size: > INT32_MAX -> SIZE_LIMIT
  if (sp_.length > 0x7fffffffu) {
    w.fail(TGPU_ERR_WRITE_SIZE_LIMIT, w.pos);
    return true;
  }
  container_header<P>(w, c, sp_.length);
  const bool is_map = c.ttype == TGPU_T_MAP;
  const uint32_t et = is_map ? c.val : c.elem;
  const uint8_t* e = lbase + sp_.offset;
  if (!is_complex(et) && !(is_map && is_complex(c.elem))) {
    const uint32_t ks = is_map ? elem_size(c.elem) : 0;
    const uint32_t ps = ks + elem_size(et);
    for (uint32_t i = 0; i < sp_.length && w.ok(); ++i) {
      if (is_map) write_elem<P>(w, c.elem, e + (uint64_t)i * ps, sbase);
      if (w.ok()) write_elem<P>(w, et, e + (uint64_t)i * ps + ks, sbase);
    }
    return true;
  }
  if (sp_.length == 0) return true;
  if (sp >= cap) {
    w.fail(full, w.pos);
    return true;
  }
  int32_t ksi = -1;
  uint32_t kti = 0;
  if (is_map && is_complex(c.elem)) {
    if (c.elem == TGPU_T_STRUCT) ksi = sc.t[c.ki - 1].struct_index;
    else kti = c.ki;
  }
  WriteFrame& f = st[sp++];
  f = WriteFrame{};
  f.kind = is_map ? WF_MAP : WF_LIST;
  f.etype = (uint8_t)et;
  f.ktype = (uint8_t)c.elem;
  f.si = (uint32_t)c.si;
  f.ti = c.ti;
  f.k = 0;
  f.end = sp_.length;
  f.ks = is_map ? slot_size(sc, c.elem, ksi) : 0;
  f.es = f.ks + slot_size(sc, et, c.si);
  f.ksi = ksi;
  f.kti = kti;
  f.obj = e;
  return false;
}

// A struct / container value of type t at p (struct si, node ti): a frame
// (or, for a container of simple elements, written here).
template <int P>
__device__ __forceinline__ void write_complex(Writer& w, const DevSchema& sc, uint32_t t,
                                              int32_t si, uint32_t ti, const uint8_t* p,
                                              const uint8_t* sbase, const uint8_t* lbase,
                                              WriteFrame* st, uint32_t& sp, uint32_t cap,
                                              int32_t full) {
  if (t == TGPU_T_STRUCT) {
    if (sp >= cap) return w.fail(full, w.pos);
    st[sp++] = write_frame(sc, (uint32_t)si, p);
  } else {
    write_container<P>(w, sc, ctype_node(sc, ti), p, sbase, lbase, st, sp, cap, full);
  }
}

// kDeep: a deep-pass lane (w.deep set): every frame in its HBM slab; else
// the lane's kPrivFrames private frames (a compile-time choice, so the bulk
// kernels keep their frames in scratch / registers).
template <int P, bool kDeep = false>
__device__ __forceinline__ void write_record(Writer& w, const DevSchema& sc, const uint8_t* rec,
                             const uint8_t* sbase, const uint8_t* lbase) {
  WriteFrame priv[kDeep ? 1 : kPrivFrames];
  WriteFrame* const st = kDeep ? (WriteFrame*)(w.deep + slab_skip_bytes(w.deep_cap)) : priv;
  const uint32_t cap = kDeep ? (uint32_t)w.deep_cap : (uint32_t)kPrivFrames;
  const int32_t full = kDeep && !w.deep_more ? TGPU_ERR_UNSUPPORTED : kErrDeep;
  uint32_t sp = 0;
  st[sp++] = write_frame(sc, 0, rec);
  while (sp > 0 && w.ok()) {
    WriteFrame& fr = st[sp - 1];
    if (fr.kind != WF_STRUCT) {
      if (fr.kphase == 0) {
        if (fr.k >= fr.end) {  // lists and maps have no end marker on the wire
          --sp;
          continue;
        }
        fr.kphase = 1;
        if (fr.kind == WF_MAP) {
          const uint8_t* key = fr.obj + (uint64_t)fr.k * fr.es;
          if (!is_complex(fr.ktype)) {
            write_elem<P>(w, fr.ktype, key, sbase);
            if (!w.ok()) break;
          } else {  // the key's frame first; its value when the frame is done
            const uint32_t before = sp;
            write_complex<P>(w, sc, fr.ktype, fr.ksi, fr.kti, key, sbase, lbase, st, sp, cap,
                             full);
            if (sp != before) continue;
          }
        }
      }
      const uint8_t* el = fr.obj + (uint64_t)fr.k++ * fr.es + fr.ks;
      fr.kphase = 0;
      if (!is_complex(fr.etype)) write_elem<P>(w, fr.etype, el, sbase);
      else write_complex<P>(w, sc, fr.etype, (int32_t)fr.si, fr.ti, el, sbase, lbase, st, sp, cap,
                            full);
      continue;
    }
    const tgpu_struct_desc sd = sc.s[fr.si];
    if (fr.k >= fr.end) {
      w.put(0);  // writeFieldStop (T_STOP / CT_STOP are both 0)
      --sp;
      continue;
    }
    const tgpu_field_desc f = sc.f[sd.first_field + fr.k++];
    const uint8_t* obj = fr.obj;
    if ((f.qualifier == TGPU_OPTIONAL || f.qualifier == TGPU_OPTIONAL_BOXED) &&
        !obj[f.isset_offset])
      continue;
    const uint8_t* m = obj + f.member_offset;
    if (f.qualifier == TGPU_TERSE && terse_empty(sc, f, m)) continue;
    if (P == TGPU_PROTOCOL_BINARY) {
      w.put(f.ttype);
      w.put_be((uint16_t)f.id, 2);
    } else {
      uint32_t ct = ttype_to_ctype(f.ttype);
      if (f.ttype == TGPU_T_BOOL) ct = load_bool(w, m) ? 1 : 2;
      const int32_t id = f.id;
      if (id > fr.last && id - fr.last <= 15) {
        w.put((uint32_t)(((id - fr.last) << 4) | ct));
      } else {
        w.put(ct);
        w.varint(i32_to_zz(id));
      }
      fr.last = id;
      if (f.ttype == TGPU_T_BOOL) continue;
    }
    if (is_scalar(f.ttype)) {
      write_scalar<P>(w, f.ttype, m);
    } else if (f.ttype == TGPU_T_STRING) {
      const tgpu_span sp_ = *(const tgpu_span*)m;
      if (sp_.length > 0x7fffffffu) return w.fail(TGPU_ERR_WRITE_SIZE_LIMIT, w.pos);
      if (P == TGPU_PROTOCOL_BINARY) w.put_be(sp_.length, 4);
      else w.varint(sp_.length);
      w.bytes(sbase + sp_.offset, sp_.length);
    } else if (f.ttype == TGPU_T_STRUCT) {
      const uint8_t* p = m;
      if (boxed(f)) {
        const tgpu_span b = *(const tgpu_span*)m;
        if (b.length == 0) {  // a null pointer: an empty struct (serialize_field.whisker:44-49)
          w.put(0);
          continue;
        }
        p = lbase + b.offset;
      }
      if (sp >= cap) return w.fail(full, w.pos);
      st[sp++] = write_frame(sc, (uint32_t)f.struct_index, p);
    } else {
      write_container<P>(w, sc, ctype_of(f), m, sbase, lbase, st, sp, cap, full);
    }
  }
}

}  // namespace dev
}  // namespace tgpu
