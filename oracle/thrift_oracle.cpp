/*
 * thrift_oracle.cpp — TEST INFRASTRUCTURE ONLY. See thrift_oracle.h.
 *
 * CPU restatement of the reference's bulk-record semantics. Each reader/writer
 * method cites the fbthrift source it follows (paths relative to the fbthrift
 * tree; the reference checkout is not needed to build or run this file).
 */
#include "thrift_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------- errors ----
struct OErr {
  int code;
  uint64_t off;
};

[[noreturn]] inline void fail(int code, uint64_t off) { throw OErr{code, off}; }

void classify(int code, int32_t* exc, int32_t* tp) {
  // TProtocolException.h:41-51 types; std::out_of_range for cursor/varint.
  int32_t e = TGPU_EXC_RUNTIME, t = 0;
  switch (code) {
    case TGPU_OK: e = TGPU_EXC_NONE; break;
    case TGPU_ERR_UNDERFLOW:
    case TGPU_ERR_INVALID_VARINT: e = TGPU_EXC_OUT_OF_RANGE; break;
    case TGPU_ERR_BOOL_VALUE:
    case TGPU_ERR_INVALID_SKIP_TYPE:
    case TGPU_ERR_TRUNCATED:
    case TGPU_ERR_UNION_MISSING_STOP: e = TGPU_EXC_PROTOCOL; t = 1; break;  // INVALID_DATA
    case TGPU_ERR_NEGATIVE_SIZE: e = TGPU_EXC_PROTOCOL; t = 2; break;
    case TGPU_ERR_SIZE_LIMIT:
    case TGPU_ERR_WRITE_SIZE_LIMIT: e = TGPU_EXC_PROTOCOL; t = 3; break;
    case TGPU_ERR_DEPTH_LIMIT: e = TGPU_EXC_PROTOCOL; t = 8; break;
    case TGPU_ERR_MISSING_REQUIRED_FIELD: e = TGPU_EXC_PROTOCOL; t = 6; break;
    case TGPU_ERR_BAD_TYPE: e = TGPU_EXC_PROTOCOL; t = 0; break;  // UNKNOWN
    case TGPU_ERR_INVALID_BOOL_WRITE: e = TGPU_EXC_ABORT; break;
    default: break;
  }
  if (exc) *exc = e;
  if (tp) *tp = t;
}

void set_status(tgpu_status* st, int code, uint64_t rec, uint64_t off) {
  if (!st) return;
  std::memset(st, 0, sizeof(*st));
  st->code = code;
  classify(code, &st->exc_class, &st->tproto_type);
  st->record = rec;
  st->byte_offset = off;
}

// ---------------------------------------------------------------- cursor ----
// folly::io::Cursor over one contiguous buffer: every read is bounds checked
// and underflow raises std::out_of_range (BinaryProtocol-inl.h:503-533 use
// in_.read / in_.readBE).
struct Cursor {
  const uint8_t* p;
  uint64_t pos, end;
  uint64_t avail() const { return end - pos; }
  bool canAdvance(uint64_t n) const { return avail() >= n; }
  uint8_t read8() {
    if (pos >= end) fail(TGPU_ERR_UNDERFLOW, pos);
    return p[pos++];
  }
  template <class T>
  T readBE() {
    if (avail() < sizeof(T)) fail(TGPU_ERR_UNDERFLOW, pos);
    uint64_t v = 0;
    for (size_t i = 0; i < sizeof(T); ++i) v = (v << 8) | p[pos + i];
    pos += sizeof(T);
    return (T)v;
  }
  void skip(uint64_t n) {
    if (avail() < n) fail(TGPU_ERR_UNDERFLOW, pos);
    pos += n;
  }
};

// -------------------------------------------------------------- varints ----
// VarintUtils-inl.h:85-87 kVarintMaxBytes = ceil(bits/7); :94-107 readVarintSlow
// and :109-134 the unrolled x86 decoder: stop at the first byte without 0x80,
// more continuation bytes than max -> std::out_of_range("invalid varint read")
// (VarintUtils.cpp:125-127); bits beyond the type width are dropped; overlong
// zeros are accepted. Underflow in the middle of a varint -> out_of_range too.
template <int BITS>
uint64_t readVarint(Cursor& c) {
  constexpr int kMax = (BITS + 6) / 7;
  const uint64_t start = c.pos;
  uint64_t result = 0;
  for (int i = 0; i < kMax; ++i) {
    if (c.pos >= c.end) fail(TGPU_ERR_UNDERFLOW, c.pos);
    const uint64_t b = c.p[c.pos++];
    result |= (b & 0x7f) << (7 * i);
    if (!(b & 0x80)) {
      if constexpr (BITS < 64) result &= (1ull << BITS) - 1;  // cast to T
      return result;
    }
  }
  fail(TGPU_ERR_INVALID_VARINT, start);
}

// VarintUtils-inl.h:72-83 zigzag.
inline int32_t zigzagToI32(uint32_t n) { return (n & 1) ? (int32_t)~(n >> 1) : (int32_t)(n >> 1); }
inline int64_t zigzagToI64(uint64_t n) { return (n & 1) ? (int64_t)~(n >> 1) : (int64_t)(n >> 1); }
inline uint32_t i32ToZigzag(int32_t n) { return ((uint32_t)n << 1) ^ (uint32_t)(n >> 31); }
inline uint64_t i64ToZigzag(int64_t n) { return ((uint64_t)n << 1) ^ (uint64_t)(n >> 63); }

// ------------------------------------------------------------- schema view --
struct Schema {
  const tgpu_struct_desc* s;
  uint32_t ns;
  const tgpu_field_desc* f;
  uint32_t nf;
  const tgpu_type_desc* t = nullptr;  // nested container types (type_index k -> t[k-1])
  uint32_t nt = 0;
};

// A container's element (list/set) or key/value (map) types, from a field or
// a nested type (TableBasedForwardTypes.h:37-93 ListFieldExt / MapFieldExt).
struct CT {
  uint8_t ttype, elem, val;
  int32_t si;   // struct of T_STRUCT elements / values
  uint32_t ti;  // 1 + nested type of container elements / values
  uint32_t ki;  // map: 1 + type node of a struct / container key
};
CT ct_of(const tgpu_field_desc& f) {
  return CT{f.ttype, f.elem_ttype, f.val_ttype, f.struct_index, f.type_index, f.key_index};
}
CT ct_node(const Schema& sc, uint32_t ti) {
  const tgpu_type_desc& t = sc.t[ti - 1];
  return CT{t.ttype, t.elem_ttype, t.val_ttype, t.struct_index, t.type_index, t.key_index};
}
// A map key's struct (a T_STRUCT key node) and container node.
int32_t key_si(const Schema& sc, const CT& c) {
  return c.elem == TGPU_T_STRUCT ? sc.t[c.ki - 1].struct_index : -1;
}
uint32_t key_ti(const CT& c) { return c.elem == TGPU_T_STRUCT ? 0 : c.ki; }
// cpp.ref / thrift.box struct fields (thrift_gpu.h TGPU_BOXED)
bool is_boxed(const tgpu_field_desc& f) {
  return f.qualifier == TGPU_BOXED || f.qualifier == TGPU_OPTIONAL_BOXED;
}
bool is_container_t(uint8_t t) {
  return t == TGPU_T_LIST || t == TGPU_T_SET || t == TGPU_T_MAP;
}

bool is_scalar(uint8_t t) {
  switch (t) {
    case TGPU_T_BOOL: case TGPU_T_BYTE: case TGPU_T_I16: case TGPU_T_I32:
    case TGPU_T_I64: case TGPU_T_DOUBLE: case TGPU_T_FLOAT:
      return true;
    default:
      return false;
  }
}
uint32_t scalar_size(uint8_t t) {
  switch (t) {
    case TGPU_T_BOOL: case TGPU_T_BYTE: return 1;
    case TGPU_T_I16: return 2;
    case TGPU_T_I32: case TGPU_T_FLOAT: return 4;
    default: return 8;
  }
}

// op::isEmpty (thrift/lib/cpp2/op/detail/Clear.h:98-127) of a terse member:
// scalars compare identical (bitwise) to the intrinsic default, so -0.0 is
// not empty; strings and containers are empty when they have no elements.
bool terse_leaf_empty(const tgpu_field_desc& f, const uint8_t* m) {
  if (is_scalar(f.ttype)) {
    for (uint32_t b = 0; b < scalar_size(f.ttype); ++b)
      if (m[b]) return false;
    return true;
  }
  uint32_t len;
  std::memcpy(&len, m + 8, 4);  // tgpu_span.length
  return len == 0;
}

// thrift::empty of a struct: the generated __fbthrift_is_empty
// (compiler/generate/templates/cpp2/module_types_cpp/declare_members.whisker:
// 83-113) — false with any unqualified (or required) field; else no optional
// field set and every terse field empty (terse structs recursively). Unions:
// no active member (union_declare_members.whisker:43-45).
bool struct_empty(const Schema& sc, uint32_t si, const uint8_t* obj) {
  const tgpu_struct_desc& sd = sc.s[si];
  for (uint32_t k = 0; k < sd.num_fields; ++k) {
    const tgpu_field_desc& f = sc.f[sd.first_field + k];
    if (sd.flags & TGPU_STRUCT_UNION) {
      if (obj[f.isset_offset]) return false;
      continue;
    }
    if (f.qualifier == TGPU_UNQUALIFIED || f.qualifier == TGPU_REQUIRED ||
        f.qualifier == TGPU_BOXED)
      return false;
    if (f.qualifier == TGPU_OPTIONAL || f.qualifier == TGPU_OPTIONAL_BOXED) {
      if (obj[f.isset_offset]) return false;
      continue;
    }
    const uint8_t* m = obj + f.member_offset;
    if (f.ttype == TGPU_T_STRUCT ? !struct_empty(sc, (uint32_t)f.struct_index, m)
                                 : !terse_leaf_empty(f, m))
      return false;
  }
  return true;
}

bool terse_empty(const Schema& sc, const tgpu_field_desc& f, const uint8_t* m) {
  return f.ttype == TGPU_T_STRUCT ? struct_empty(sc, (uint32_t)f.struct_index, m)
                                  : terse_leaf_empty(f, m);
}

// ================================================================ readers ===
struct Limits {
  int32_t string_limit = 0, container_limit = 0, max_depth = 12000, height = 0;
  int64_t initial_height() const { return (int64_t)(height ? height : max_depth) + 1; }
};

// ProtocolBase::descend/ascend (Protocol.h:59-78, height = max_depth + 1).
struct Height {
  int64_t h;
  void descend(uint64_t off) {
    if (!--h) fail(TGPU_ERR_DEPTH_LIMIT, off);
  }
  void ascend() { ++h; }
};

// ---- Binary (BinaryProtocol-inl.h:384-661, BinaryProtocol.cpp:140-225) ----
struct BinaryReader {
  Cursor c;
  Limits lim;
  Height height;

  void checkStringSize(int32_t size, uint64_t off) {  // -inl.h:535-543
    if (size < 0) fail(TGPU_ERR_NEGATIVE_SIZE, off);
    if (lim.string_limit > 0 && size > lim.string_limit) fail(TGPU_ERR_SIZE_LIMIT, off);
  }
  void checkContainerSize(int32_t size, uint64_t off) {  // -inl.h:545-551
    if (size < 0) fail(TGPU_ERR_NEGATIVE_SIZE, off);
    if (lim.container_limit && size > lim.container_limit) fail(TGPU_ERR_SIZE_LIMIT, off);
  }
  // readFieldBeginWithState (-inl.h:623-632): type byte, STOP has no id.
  // advanceToNextField's 3-byte fast path (:586-621) yields the same result.
  bool readFieldHeader(int16_t /*prev*/, uint8_t& type, int16_t& id) {
    type = c.read8();
    if (type == TGPU_T_STOP) return false;
    id = c.readBE<int16_t>();
    return true;
  }
  bool readBool() {  // -inl.h:489-495
    const uint64_t off = c.pos;
    const uint8_t b = c.read8();
    if (b >= 2) fail(TGPU_ERR_BOOL_VALUE, off);
    return b != 0;
  }
  void readListBegin(uint8_t& elem, int32_t& size) {  // -inl.h:457-467
    const uint64_t off = c.pos;
    height.descend(off);
    elem = c.read8();
    const uint64_t soff = c.pos;
    size = c.readBE<int32_t>();
    checkContainerSize(size, soff);
  }
  void readMapBegin(uint8_t& k, uint8_t& v, int32_t& size) {  // -inl.h:439-451
    height.descend(c.pos);
    k = c.read8();
    v = c.read8();
    const uint64_t soff = c.pos;
    size = c.readBE<int32_t>();
    checkContainerSize(size, soff);
  }
  // readString -> readStringBody -> checkStringSize + detail::readStringBody
  // (Protocol.h:435-449: canAdvance before allocation -> throwTruncatedData).
  void readString(uint64_t& view, uint32_t& len) {
    const uint64_t off = c.pos;
    const int32_t size = c.readBE<int32_t>();
    checkStringSize(size, off);
    if (!c.canAdvance((uint64_t)size)) fail(TGPU_ERR_TRUNCATED, c.pos);
    view = c.pos;
    len = (uint32_t)size;
    c.pos += (uint64_t)size;
  }
  static uint32_t fixedSizeInContainer(uint8_t t) {  // -inl.h:634-661
    switch (t) {
      case TGPU_T_BOOL: case TGPU_T_BYTE: return 1;
      case TGPU_T_I16: return 2;
      case TGPU_T_I32: case TGPU_T_FLOAT: return 4;
      case TGPU_T_I64: case TGPU_T_DOUBLE: return 8;
      default: return 0;
    }
  }
  // Protocol.h:297-344 skip_n.
  void skip_n(uint32_t n, const uint8_t* types, int nt, int depth) {
    if (depth >= lim.max_depth) fail(TGPU_ERR_DEPTH_LIMIT, c.pos);
    uint64_t sum = 0;
    bool allFixed = true;
    for (int i = 0; i < nt; ++i) {
      const uint32_t s = fixedSizeInContainer(types[i]);
      sum += s;
      allFixed = allFixed && s;
    }
    if (allFixed) {
      c.skip(sum * n);
      return;
    }
    for (uint32_t i = 0; i < n; ++i)
      for (int j = 0; j < nt; ++j) skip(types[j], depth + 1);
  }
  // BinaryProtocolReader::skip (BinaryProtocol.cpp:140-225).
  void skip(uint8_t type, int depth) {
    if (depth >= lim.max_depth) fail(TGPU_ERR_DEPTH_LIMIT, c.pos);
    uint64_t bytes = 0;
    switch (type) {
      case TGPU_T_BYTE: case TGPU_T_BOOL: bytes = 1; break;
      case TGPU_T_I16: bytes = 2; break;
      case TGPU_T_FLOAT: case TGPU_T_I32: bytes = 4; break;
      case TGPU_T_DOUBLE: case TGPU_T_U64: case TGPU_T_I64: bytes = 8; break;
      case TGPU_T_UTF8: case TGPU_T_UTF16: case TGPU_T_STRING: {
        // canAdvance(size) is checked from the cursor copy taken BEFORE the
        // length was read, with size cast through int32 -> size_t.
        const uint64_t before = c.pos;
        const int32_t size = c.readBE<int32_t>();
        const uint64_t want = (uint64_t)(int64_t)size;  // negative -> huge
        if (c.end - before < want) fail(TGPU_ERR_TRUNCATED, c.pos);
        bytes = (uint64_t)(uint32_t)size;
        break;
      }
      case TGPU_T_STRUCT: {
        height.descend(c.pos);  // readStructBegin
        while (true) {
          const uint8_t ft = c.read8();
          if (ft == TGPU_T_STOP) {
            height.ascend();
            return;
          }
          c.skip(2);
          skip(ft, depth + 1);
        }
      }
      case TGPU_T_MAP: {
        uint8_t kv[2];
        int32_t size;
        readMapBegin(kv[0], kv[1], size);
        skip_n((uint32_t)size, kv, 2, depth + 1);
        height.ascend();
        return;
      }
      case TGPU_T_SET:
      case TGPU_T_LIST: {
        uint8_t e;
        int32_t size;
        readListBegin(e, size);
        skip_n((uint32_t)size, &e, 1, depth + 1);
        height.ascend();
        return;
      }
      default:
        fail(TGPU_ERR_INVALID_SKIP_TYPE, c.pos);
    }
    c.skip(bytes);
  }
  // Scalar value reads (-inl.h:503-533).
  void readScalar(uint8_t t, uint8_t* dst) {
    switch (t) {
      case TGPU_T_BOOL: *dst = readBool() ? 1 : 0; break;
      case TGPU_T_BYTE: *dst = c.read8(); break;
      case TGPU_T_I16: { int16_t v = c.readBE<int16_t>(); std::memcpy(dst, &v, 2); break; }
      case TGPU_T_I32:
      case TGPU_T_FLOAT: { int32_t v = c.readBE<int32_t>(); std::memcpy(dst, &v, 4); break; }
      default: { int64_t v = c.readBE<int64_t>(); std::memcpy(dst, &v, 8); break; }
    }
  }
  uint8_t listElemWire(uint8_t elem) const { return elem; }
  static constexpr uint64_t kArenaScale = 1;
};

// ---- Compact (CompactProtocol-inl.h:531-938, CompactProtocol.cpp:48-54) ----
// CTypeToTType (-inl.h:70-85); index >= 14 -> throwBadType.
const uint8_t kCTypeToTType[14] = {
    TGPU_T_STOP, TGPU_T_BOOL, TGPU_T_BOOL, TGPU_T_BYTE, TGPU_T_I16,
    TGPU_T_I32, TGPU_T_I64, TGPU_T_DOUBLE, TGPU_T_STRING, TGPU_T_LIST,
    TGPU_T_SET, TGPU_T_MAP, TGPU_T_STRUCT, TGPU_T_FLOAT};
// TTypeToCType (-inl.h:48-69).
uint8_t ttypeToCType(uint8_t t) {
  switch (t) {
    case TGPU_T_STOP: return 0;
    case TGPU_T_BOOL: return 1;
    case TGPU_T_BYTE: return 3;
    case TGPU_T_DOUBLE: return 7;
    case TGPU_T_I16: return 4;
    case TGPU_T_I32: return 5;
    case TGPU_T_I64: return 6;
    case TGPU_T_STRING: return 8;
    case TGPU_T_STRUCT: return 12;
    case TGPU_T_MAP: return 11;
    case TGPU_T_SET: return 10;
    case TGPU_T_LIST: return 9;
    case TGPU_T_FLOAT: return 13;
    default: return 0;
  }
}

struct CompactReader {
  Cursor c;
  Limits lim;
  Height height;
  bool hasBool = false, boolVal = false;  // boolValue_ latch

  uint8_t getType(uint8_t ct, uint64_t off) {  // -inl.h:783-791
    if (ct >= 14) fail(TGPU_ERR_BAD_TYPE, off);
    return kCTypeToTType[ct];
  }
  void checkStringSize(int32_t size, uint64_t off) {  // -inl.h:742-749
    if (size < 0) fail(TGPU_ERR_NEGATIVE_SIZE, off);
    if (lim.string_limit > 0 && size > lim.string_limit) fail(TGPU_ERR_SIZE_LIMIT, off);
  }
  // readFieldBeginWithStateImpl (-inl.h:884-910). Any byte with a zero low
  // nibble ends the struct after consuming 1 byte (0x00 directly; 0xN0 via
  // getType(0) == T_STOP).
  bool readFieldHeader(int16_t prev, uint8_t& type, int16_t& id) {
    const uint64_t off = c.pos;
    const uint8_t b = c.read8();
    if ((b & 0x0f) == 0) return false;
    const int16_t modifier = (int16_t)(b >> 4);
    if (modifier != 0) {
      id = (int16_t)(prev + modifier);
    } else {
      id = (int16_t)zigzagToI32((uint32_t)readVarint<32>(c));  // readI16 via i32
    }
    const uint8_t ct = b & 0x0f;
    type = getType(ct, off);
    if (ct == 1 || ct == 2) {
      hasBool = true;
      boolVal = (ct == 1);
    }
    return true;
  }
  bool readBool() {  // -inl.h:692-701
    if (hasBool) {
      hasBool = false;
      return boolVal;
    }
    return c.read8() == 1;
  }
  void readListBegin(uint8_t& elem, int32_t& size) {  // -inl.h:615-640
    const uint64_t off = c.pos;
    height.descend(off);
    const uint8_t b = c.read8();
    int32_t lsize = (b >> 4) & 0x0f;
    if (lsize == 15) lsize = (int32_t)(uint32_t)readVarint<32>(c);
    if (lsize < 0) fail(TGPU_ERR_NEGATIVE_SIZE, off);
    if (lim.container_limit && lsize > lim.container_limit) fail(TGPU_ERR_SIZE_LIMIT, off);
    elem = getType(b & 0x0f, off);
    size = lsize;
  }
  void readMapBegin(uint8_t& k, uint8_t& v, int32_t& size) {  // -inl.h:578-610
    const uint64_t off = c.pos;
    height.descend(off);
    uint8_t kv = 0;
    const int32_t msize = (int32_t)(uint32_t)readVarint<32>(c);
    if (msize != 0) kv = c.read8();
    if (msize < 0) fail(TGPU_ERR_NEGATIVE_SIZE, off);
    if (lim.container_limit && msize > lim.container_limit) fail(TGPU_ERR_SIZE_LIMIT, off);
    k = getType(kv >> 4, off);
    v = getType(kv & 0xf, off);
    size = msize;
  }
  void readString(uint64_t& view, uint32_t& len) {  // -inl.h:751-781
    const uint64_t off = c.pos;
    const int32_t size = (int32_t)(uint32_t)readVarint<32>(c);
    checkStringSize(size, off);
    if (size == 0) {
      view = 0;
      len = 0;
      return;
    }
    if (!c.canAdvance((uint64_t)size)) fail(TGPU_ERR_TRUNCATED, c.pos);
    view = c.pos;
    len = (uint32_t)size;
    c.pos += (uint64_t)size;
  }
  static uint32_t fixedSizeInContainer(uint8_t t) {  // -inl.h:912-938
    switch (t) {
      case TGPU_T_BOOL: case TGPU_T_BYTE: return 1;
      case TGPU_T_FLOAT: return 4;
      case TGPU_T_DOUBLE: return 8;
      default: return 0;
    }
  }
  void skip_n(uint32_t n, const uint8_t* types, int nt, int depth) {  // Protocol.h:317-344
    if (depth >= lim.max_depth) fail(TGPU_ERR_DEPTH_LIMIT, c.pos);
    uint64_t sum = 0;
    bool allFixed = true;
    for (int i = 0; i < nt; ++i) {
      const uint32_t s = fixedSizeInContainer(types[i]);
      sum += s;
      allFixed = allFixed && s;
    }
    if (allFixed) {
      c.skip(sum * n);
      return;
    }
    for (uint32_t i = 0; i < n; ++i)
      for (int j = 0; j < nt; ++j) skip(types[j], depth + 1);
  }
  // apache::thrift::skip (Protocol.h:187-283) instantiated for Compact.
  void skip(uint8_t type, int depth) {
    if (depth >= lim.max_depth) fail(TGPU_ERR_DEPTH_LIMIT, c.pos);
    switch (type) {
      case TGPU_T_BOOL: readBool(); return;
      case TGPU_T_BYTE: c.read8(); return;
      case TGPU_T_I16:
      case TGPU_T_I32: readVarint<32>(c); return;
      case TGPU_T_U64:
      case TGPU_T_I64: readVarint<64>(c); return;
      case TGPU_T_DOUBLE: c.readBE<int64_t>(); return;
      case TGPU_T_FLOAT: c.readBE<int32_t>(); return;
      case TGPU_T_UTF8: case TGPU_T_UTF16: case TGPU_T_STRING: {
        uint64_t v;
        uint32_t l;
        readString(v, l);
        return;
      }
      case TGPU_T_STRUCT: {
        height.descend(c.pos);  // readStructBegin: push lastFieldId_, = 0
        int16_t last = 0;
        while (true) {
          uint8_t ft;
          int16_t fid;
          if (!readFieldHeader(last, ft, fid)) break;
          last = fid;
          skip(ft, depth + 1);
        }
        height.ascend();
        return;
      }
      case TGPU_T_MAP: {
        uint8_t kv[2];
        int32_t size;
        readMapBegin(kv[0], kv[1], size);
        skip_n((uint32_t)size, kv, 2, depth + 1);
        height.ascend();
        return;
      }
      case TGPU_T_SET:
      case TGPU_T_LIST: {
        uint8_t e;
        int32_t size;
        readListBegin(e, size);
        skip_n((uint32_t)size, &e, 1, depth + 1);
        height.ascend();
        return;
      }
      default:
        fail(TGPU_ERR_INVALID_SKIP_TYPE, c.pos);
    }
  }
  void readScalar(uint8_t t, uint8_t* dst) {  // -inl.h:703-740
    switch (t) {
      case TGPU_T_BOOL: *dst = readBool() ? 1 : 0; break;
      case TGPU_T_BYTE: *dst = c.read8(); break;
      case TGPU_T_I16: { int16_t v = (int16_t)zigzagToI32((uint32_t)readVarint<32>(c)); std::memcpy(dst, &v, 2); break; }
      case TGPU_T_I32: { int32_t v = zigzagToI32((uint32_t)readVarint<32>(c)); std::memcpy(dst, &v, 4); break; }
      case TGPU_T_I64: { int64_t v = zigzagToI64(readVarint<64>(c)); std::memcpy(dst, &v, 8); break; }
      case TGPU_T_FLOAT: { int32_t v = c.readBE<int32_t>(); std::memcpy(dst, &v, 4); break; }
      default: { int64_t v = c.readBE<int64_t>(); std::memcpy(dst, &v, 8); break; }  // double
    }
  }
  static constexpr uint64_t kArenaScale = 8;
};

// ---- CompactV1 (CompactV1Protocol.h): readDouble is readLE (-inl.h:73-79) --
struct CompactV1Reader : CompactReader {
  void readScalar(uint8_t t, uint8_t* dst) {
    if (t == TGPU_T_DOUBLE) {
      const uint64_t v = __builtin_bswap64((uint64_t)c.readBE<int64_t>());
      std::memcpy(dst, &v, 8);
      return;
    }
    CompactReader::readScalar(t, dst);
  }
};

// ---- generated readNoXfer restated, table-driven (TableBasedSerializerImpl.h
// :695-767 has the same contract; deserialize_struct.whisker:19-160) --------
struct DecodeCtx {
  const Schema* sc;
  uint8_t* arena;
  uint64_t arena_cap;
  uint64_t scale;  // arena bytes per wire byte: 1/8, or 4/16 with string elements
  // nested schemas: each record's containers are allocated in wire order
  // from scale x its start, 8-byte aligned (thrift_gpu.h
  // tgpu_schema_arena_scale); otherwise scale x the first element's position
  bool regions = false;
  uint64_t bump = 0;
  uint64_t alloc(uint64_t first_elem_pos, uint64_t bytes) {
    if (!regions) return scale * first_elem_pos;
    const uint64_t o = bump;
    bump = (bump + bytes + 7) & ~7ull;
    return o;
  }
};

bool has_string_elems(const Schema& sc) {
  auto se = [](uint8_t t, uint8_t e, uint8_t v) {
    return is_container_t(t) && (e == TGPU_T_STRING || (t == TGPU_T_MAP && v == TGPU_T_STRING));
  };
  for (uint32_t k = 0; k < sc.nf; ++k)
    if (se(sc.f[k].ttype, sc.f[k].elem_ttype, sc.f[k].val_ttype)) return true;
  for (uint32_t k = 0; k < sc.nt; ++k)
    if (se(sc.t[k].ttype, sc.t[k].elem_ttype, sc.t[k].val_ttype)) return true;
  return false;
}

// Scalars in native layout; strings and containers as 16-byte spans.
uint32_t elem_size(uint8_t t) {
  return (t == TGPU_T_STRING || is_container_t(t)) ? 16 : scalar_size(t);
}
uint32_t slot_size(const Schema& sc, uint8_t t, int32_t si) {
  return t == TGPU_T_STRUCT ? sc.s[si].size : elem_size(t);
}
bool is_complex_t(uint8_t t) { return t == TGPU_T_STRUCT || is_container_t(t); }

// ---- arena regions of nested schemas -----------------------------------------
// Every arena byte of a record is charged to wire bytes of its own: an
// element's slot to the element's own bytes (a struct element can be one
// STOP byte), a container's alignment padding (<= 7) to its header. The scale
// is the largest bytes-per-wire-byte ratio of the schema's element kinds,
// at least 8, rounded up to a multiple of 8.
uint32_t min_wire(uint8_t t, bool compact) {
  switch (t) {
    case TGPU_T_BOOL: case TGPU_T_BYTE: return 1;
    case TGPU_T_I16: return compact ? 1 : 2;
    case TGPU_T_I32: return compact ? 1 : 4;
    case TGPU_T_I64: return compact ? 1 : 8;
    case TGPU_T_FLOAT: return 4;
    case TGPU_T_DOUBLE: return 8;
    case TGPU_T_STRING: return compact ? 1 : 4;
    case TGPU_T_LIST: case TGPU_T_SET: return compact ? 1 : 5;
    case TGPU_T_MAP: return compact ? 1 : 6;
    default: return 1;
  }
}
bool nested_schema(const Schema& sc) {
  auto nested = [](uint8_t t, uint8_t e, uint8_t v) {
    return is_container_t(t) && (is_complex_t(t == TGPU_T_MAP ? v : e) ||
                                 (t == TGPU_T_MAP && is_complex_t(e)));
  };
  for (uint32_t k = 0; k < sc.nf; ++k)
    if (nested(sc.f[k].ttype, sc.f[k].elem_ttype, sc.f[k].val_ttype) || is_boxed(sc.f[k]))
      return true;
  return false;
}
// Every container description (fields and type nodes) and every boxed field
// once: recursive schemas are covered without recursion.
void ratio_of(const Schema& sc, const CT& c, bool compact, double& ratio) {
  if (!is_container_t(c.ttype)) return;
  const bool is_map = c.ttype == TGPU_T_MAP;
  const uint8_t v = is_map ? c.val : c.elem;
  const double kb = is_map ? slot_size(sc, c.elem, key_si(sc, c)) : 0;
  const double kw = is_map ? min_wire(c.elem, compact) : 0;
  const double pad = (is_container_t(v) ? 7 : 0) + (is_map && is_container_t(c.elem) ? 7 : 0);
  const double vb = slot_size(sc, v, c.si);
  ratio = std::max(ratio, (kb + vb + pad) / (kw + min_wire(v, compact)));
  ratio = std::max(ratio, 7.0 / min_wire(c.ttype, compact));
}
uint32_t region_scale(const Schema& sc, bool compact) {
  double ratio = 8.0;
  for (uint32_t k = 0; k < sc.nf; ++k) {
    ratio_of(sc, ct_of(sc.f[k]), compact, ratio);
    if (sc.f[k].ttype == TGPU_T_STRUCT && is_boxed(sc.f[k]))  // field header + STOP
      ratio = std::max(ratio, (sc.s[sc.f[k].struct_index].size + 7.0) / (compact ? 2.0 : 4.0));
  }
  for (uint32_t k = 0; k < sc.nt; ++k) ratio_of(sc, ct_node(sc, k + 1), compact, ratio);
  return ((uint32_t)std::ceil(ratio) + 7) & ~7u;
}

// A container element: a scalar, or a string as a span into the stream.
template <class R>
void readElem(R& r, uint8_t t, uint8_t* dst) {
  if (t != TGPU_T_STRING) return r.readScalar(t, dst);
  tgpu_span sp{0, 0, 0};
  r.readString(sp.offset, sp.length);
  if (sp.length == 0) sp.offset = 0;
  std::memcpy(dst, &sp, sizeof(sp));
}

template <class R>
void readStruct(R& r, uint32_t si, uint8_t* obj, DecodeCtx& dc);
template <class R>
void readContainer(R& r, const CT& c, uint8_t* member, DecodeCtx& dc);

inline void put_span(uint8_t* m, uint64_t off, uint32_t len) {
  const tgpu_span sp{len ? off : 0, len, 0};
  std::memcpy(m, &sp, sizeof(sp));
}

// A list/set element or map value of type t (struct si / nested type ti)
// read into its slot.
template <class R>
void readValue(R& r, uint8_t t, int32_t si, uint32_t ti, uint8_t* dst, DecodeCtx& dc) {
  if (t == TGPU_T_STRUCT) readStruct(r, (uint32_t)si, dst, dc);
  else if (is_container_t(t)) readContainer(r, ct_node(*dc.sc, ti), dst, dc);
  else readElem(r, t, dst);
}

template <class R>
void readList(R& r, const CT& f, uint8_t* member, DecodeCtx& dc) {
  // protocol_methods<list>::read (protocol_methods.h:389-467). The member is
  // reset to empty first (deserialize_field.whisker:44-47).
  tgpu_span span{0, 0, 0};
  std::memcpy(member, &span, sizeof(span));
  uint8_t reported;
  int32_t n;
  r.readListBegin(reported, n);
  if (reported != f.elem) {
    r.skip_n((uint32_t)n, &reported, 1, 0);
  } else if (is_complex_t(f.elem)) {
    // structs / containers as elements: reserve + emplace_back_default +
    // read per element (:374-386,458-461) — the list holds the elements
    // read plus the failing one; a set inserts an element once it is read
    // (EncodeHelpers.h:248-259)
    if (!r.c.canAdvance((uint64_t)(uint32_t)n)) fail(TGPU_ERR_TRUNCATED, r.c.pos);
    const uint32_t es = slot_size(*dc.sc, f.elem, f.si);
    if (n > 0) {
      if (!dc.arena) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
      const uint64_t bytes = (uint64_t)(uint32_t)n * es;
      const uint64_t aoff = dc.alloc(r.c.pos, bytes);
      if (aoff + bytes > dc.arena_cap) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
      const bool is_set = f.ttype == TGPU_T_SET;
      for (int32_t i = 0; i < n; ++i) {
        uint8_t* el = dc.arena + aoff + (uint64_t)i * es;
        std::memset(el, 0, es);
        if (!is_set) put_span(member, aoff, (uint32_t)(i + 1));
        readValue(r, f.elem, f.si, f.ti, el, dc);
        if (is_set) put_span(member, aoff, (uint32_t)(i + 1));
      }
    }
  } else {
    if (!r.c.canAdvance((uint64_t)(uint32_t)n)) fail(TGPU_ERR_TRUNCATED, r.c.pos);  // canReadNElements
    const uint32_t es = elem_size(f.elem);
    const uint64_t aoff = n > 0 ? dc.alloc(r.c.pos, (uint64_t)(uint32_t)n * es) : 0;
    if (n > 0) {
      if (!dc.arena) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
      // resizeWithoutInitialization(out, n) happens before the element reads
      span.offset = aoff;
      span.length = (uint32_t)n;
      std::memcpy(member, &span, sizeof(span));
    }
    int32_t i = 0;
    try {
      for (; i < n; ++i) {
        // read first: truncation fails as the reader does (the arena always
        // holds an element that was read when sized as documented)
        const uint64_t at = aoff + (uint64_t)i * es;
        uint8_t tmp[16];
        readElem(r, f.elem, tmp);
        if (at + es > dc.arena_cap) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
        std::memcpy(dc.arena + at, tmp, es);
      }
    } catch (const OErr&) {
      if (f.ttype == TGPU_T_SET) {
        // deserialize_known_length_set (EncodeHelpers.h:248-259, std::set):
        // an element is inserted once read — the complete ones remain
        span.length = (uint32_t)i;
        if (!i) span.offset = 0;
        std::memcpy(member, &span, sizeof(span));
      } else if (f.elem == TGPU_T_STRING) {
        // non-trivial elements: reserve + emplace_back_default + read
        // (protocol_methods.h:374-386,458-461): the failing element is in
        // the list, empty
        if (aoff + ((uint64_t)i + 1) * es <= dc.arena_cap)
          std::memset(dc.arena + aoff + (uint64_t)i * es, 0, es);
        span.length = (uint32_t)(i + 1);
        std::memcpy(member, &span, sizeof(span));
      } else {
        // protocol_methods.h:441-451: leftover elements are value-initialized
        for (; i < n; ++i) {
          const uint64_t at = aoff + (uint64_t)i * es;
          if (at + es > dc.arena_cap) break;
          std::memset(dc.arena + at, 0, es);
        }
      }
      throw;
    }
  }
  r.height.ascend();  // readListEnd
}

template <class R>
void readMap(R& r, const CT& f, uint8_t* member, DecodeCtx& dc) {
  // protocol_methods<map>::read (protocol_methods.h:640-677); the member is
  // reset first (deserialize_field.whisker:44-47). Pairs in wire order, packed
  // {key, value}. deserialize_known_length_map (EncodeHelpers.h:188-205)
  // inserts a pair only once both reads succeeded: a failing map keeps the
  // complete pairs before the failure.
  tgpu_span span{0, 0, 0};
  std::memcpy(member, &span, sizeof(span));
  uint8_t kv[2];
  int32_t n;
  r.readMapBegin(kv[0], kv[1], n);
  if (n > 0 && (kv[0] != f.elem || kv[1] != f.val)) {
    r.skip_n((uint32_t)n, kv, 2, 0);
  } else if (is_complex_t(f.val) || is_complex_t(f.elem)) {
    // structs / containers as keys or values: the key's and the value's
    // reads, then the pair is inserted
    if (!r.c.canAdvance((uint64_t)(uint32_t)n * 2)) fail(TGPU_ERR_TRUNCATED, r.c.pos);
    const int32_t ksi = key_si(*dc.sc, f);
    const uint32_t ks = slot_size(*dc.sc, f.elem, ksi), ps = ks + slot_size(*dc.sc, f.val, f.si);
    if (n > 0) {
      if (!dc.arena) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
      const uint64_t bytes = (uint64_t)(uint32_t)n * ps;
      const uint64_t aoff = dc.alloc(r.c.pos, bytes);
      if (aoff + bytes > dc.arena_cap) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
      for (int32_t i = 0; i < n; ++i) {
        uint8_t* pr = dc.arena + aoff + (uint64_t)i * ps;
        std::memset(pr, 0, ps);
        readValue(r, f.elem, ksi, key_ti(f), pr, dc);
        readValue(r, f.val, f.si, f.ti, pr + ks, dc);
        put_span(member, aoff, (uint32_t)(i + 1));
      }
    }
  } else {
    if (!r.c.canAdvance((uint64_t)(uint32_t)n * 2)) fail(TGPU_ERR_TRUNCATED, r.c.pos);
    const uint32_t ks = elem_size(f.elem), ps = ks + elem_size(f.val);
    const uint64_t aoff = n > 0 ? dc.alloc(r.c.pos, (uint64_t)(uint32_t)n * ps) : 0;
    if (n > 0 && !dc.arena) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
    int32_t i = 0;
    try {
      for (; i < n; ++i) {
        uint8_t pr[32];
        readElem(r, f.elem, pr);
        readElem(r, f.val, pr + ks);
        const uint64_t at = aoff + (uint64_t)i * ps;
        if (at + ps > dc.arena_cap) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
        std::memcpy(dc.arena + at, pr, ps);
      }
    } catch (const OErr&) {
      if (i > 0) {
        span = tgpu_span{aoff, (uint32_t)i, 0};
        std::memcpy(member, &span, sizeof(span));
      }
      throw;
    }
    if (n > 0) {
      span = tgpu_span{aoff, (uint32_t)n, 0};
      std::memcpy(member, &span, sizeof(span));
    }
  }
  r.height.ascend();  // readMapEnd
}

template <class R>
void readContainer(R& r, const CT& c, uint8_t* member, DecodeCtx& dc) {
  if (c.ttype == TGPU_T_MAP) readMap(r, c, member, dc);
  else readList(r, c, member, dc);
}

template <class R>
void readStruct(R& r, uint32_t si, uint8_t* obj, DecodeCtx& dc) {
  const tgpu_struct_desc& sd = dc.sc->s[si];
  // A union (deserialize_union.whisker:19-60): an immediate STOP clears it,
  // one field (read or skipped), then the STOP is required.
  const bool un = sd.flags & TGPU_STRUCT_UNION;
  int16_t prev = 0;
  bool first = true;
  uint64_t seen = 0;  // the generated reader's local isset_<field> flags
  while (true) {
    uint8_t wt;
    int16_t id;
    if (!r.readFieldHeader(prev, wt, id)) {
      if (un && first) std::memset(obj, 0, sd.size);  // apache::thrift::clear
      break;
    }
    if (un && !first) fail(TGPU_ERR_UNION_MISSING_STOP, r.c.pos);  // throwUnionMissingStop
    first = false;
    prev = id;
    const tgpu_field_desc* f = nullptr;
    for (uint32_t k = 0; k < sd.num_fields; ++k) {
      const tgpu_field_desc& c = dc.sc->f[sd.first_field + k];
      if (c.id == id) {
        f = &c;
        break;
      }
    }
    // isCompatibleWithType: fieldType == expected (BinaryProtocol.h:353-356,
    // CompactProtocol.h:433-437); else skip (deserialize_struct.whisker:140-157).
    if (!f || f->ttype != wt) {
      r.skip(wt, 0);
      continue;
    }
    uint8_t* m = obj + f->member_offset;
    if (un) {  // field_ref().emplace(): the union now holds a fresh member
      std::memset(obj, 0, sd.size);
      obj[f->isset_offset] = 1;
    }
    if (is_scalar(f->ttype)) {
      r.readScalar(f->ttype, m);
    } else if (f->ttype == TGPU_T_STRING) {
      tgpu_span sp{0, 0, 0};
      r.readString(sp.offset, sp.length);
      if (sp.length == 0) sp.offset = 0;
      std::memcpy(m, &sp, sizeof(sp));
    } else if (f->ttype == TGPU_T_STRUCT && is_boxed(*f)) {
      // cpp.ref / thrift.box: make_mutable_smart_ptr, read, then the member
      // points to the fresh object (deserialize_field.whisker:21-23,49-51)
      const uint32_t size = dc.sc->s[f->struct_index].size;
      if (!dc.arena) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
      const uint64_t aoff = dc.alloc(r.c.pos, size);
      if (aoff + size > dc.arena_cap) fail(TGPU_ERR_OUTPUT_OVERFLOW, r.c.pos);
      std::memset(dc.arena + aoff, 0, size);
      readStruct(r, (uint32_t)f->struct_index, dc.arena + aoff, dc);
      put_span(m, aoff, 1);
    } else if (f->ttype == TGPU_T_STRUCT) {
      readStruct(r, (uint32_t)f->struct_index, m, dc);  // merges into member
    } else if (is_container_t(f->ttype)) {
      readContainer(r, ct_of(*f), m, dc);
    }
    obj[f->isset_offset] = 1;  // __isset.set(idx, true)
    const uint32_t k = (uint32_t)(f - (dc.sc->f + sd.first_field));
    if (k < 64) seen |= 1ull << k;
  }
  // deprecated_enforce_required (deserialize_struct.whisker:116-124): after
  // readStructEnd, a required field this read did not see throws
  // MISSING_REQUIRED_FIELD
  if (sd.flags & TGPU_STRUCT_ENFORCE_REQUIRED)
    for (uint32_t k = 0; k < sd.num_fields && k < 64; ++k)
      if (dc.sc->f[sd.first_field + k].qualifier == TGPU_REQUIRED && !((seen >> k) & 1))
        fail(TGPU_ERR_MISSING_REQUIRED_FIELD, r.c.pos);
}

void init_record(const Schema& sc, uint8_t* rec) {
  std::memset(rec, 0, sc.s[0].size);  // default-constructed T (zero defaults)
}

// ---- block rule (round 6): list / set elements of flat-list schemas --------
// A schema whose containers are all lists / sets of scalars (no maps, no
// strings or structs or containers as elements, nothing boxed: not a nested
// schema), at most kPackSlots of them counting those inside by-value struct
// members, keeps no per-record arena regions: records are grouped by index
// in blocks of kArenaBlock, and block b's element arrays are allocated in
// read order (records in order, a record's arrays in wire order), each
// 8-byte aligned, from align8(scale x the wire start of the block's first
// record). Every array then is the dense std::vector the reference's
// readArithmeticVector fills (protocol_methods.h:390-441), and a block's
// arrays fit the bytes its wire took (an array's 8 header bytes hold its
// padding). Restated here as a pass over the position-rule arena (each array
// moves down: its packed start is never above its wire position x scale).
constexpr uint32_t kArenaBlock = 64;
constexpr uint32_t kPackSlots = 8;
struct PackSlot {
  uint32_t member, es;
};
bool pack_slots_of(const Schema& sc, uint32_t si, uint32_t base, std::vector<PackSlot>& out,
                   int depth) {
  if (depth > 64) return false;
  const tgpu_struct_desc& sd = sc.s[si];
  for (uint32_t k = 0; k < sd.num_fields; ++k) {
    const tgpu_field_desc& f = sc.f[sd.first_field + k];
    if (is_boxed(f)) return false;
    if (f.ttype == TGPU_T_STRUCT) {
      if (!pack_slots_of(sc, (uint32_t)f.struct_index, base + f.member_offset, out, depth + 1))
        return false;
    } else if (f.ttype == TGPU_T_MAP) {
      return false;
    } else if (is_container_t(f.ttype)) {
      if (!is_scalar(f.elem_ttype)) return false;
      out.push_back(PackSlot{base + f.member_offset, scalar_size(f.elem_ttype)});
    }
  }
  return true;
}
// The slots of a block-packed schema (empty: the position rule applies).
std::vector<PackSlot> block_pack_slots(const Schema& sc) {
  std::vector<PackSlot> v;
  if (nested_schema(sc) || has_string_elems(sc) || !pack_slots_of(sc, 0, 0, v, 0) ||
      v.size() > kPackSlots)
    v.clear();
  return v;
}
// Records [0, m) (the failing record included) from the position rule to the
// block rule: bytes moved in place in increasing order (a byte's destination
// never lies above its source, nor above a later byte's source); a source
// byte past the arena's end (a failing record's list resized past it) reads
// as zero, a destination past it is not written.
void pack_blocks(const Schema& sc, const std::vector<PackSlot>& slots, const uint64_t* starts,
                 uint64_t m, uint8_t* recs, uint8_t* arena, uint64_t cap, uint64_t scale) {
  const uint32_t rs = sc.s[0].size;
  for (uint64_t b0 = 0; b0 < m; b0 += kArenaBlock) {
    uint64_t cur = (scale * starts[b0] + 7) & ~7ull;
    const uint64_t b1 = std::min<uint64_t>(m, b0 + kArenaBlock);
    for (uint64_t i = b0; i < b1; ++i) {
      uint8_t* rec = recs + i * rs;
      std::vector<std::pair<uint64_t, uint32_t>> order;  // (source, slot) of the non-empty arrays
      for (uint32_t k = 0; k < slots.size(); ++k) {
        tgpu_span sp;
        std::memcpy(&sp, rec + slots[k].member, sizeof(sp));
        if (sp.length) order.emplace_back(sp.offset, k);
      }
      std::sort(order.begin(), order.end());
      for (const auto& o : order) {
        tgpu_span sp;
        std::memcpy(&sp, rec + slots[o.second].member, sizeof(sp));
        const uint64_t bytes = (uint64_t)sp.length * slots[o.second].es;
        cur = (cur + 7) & ~7ull;
        if (arena)
          for (uint64_t t = 0; t < bytes; ++t) {
            const uint64_t d = cur + t, src = sp.offset + t;
            if (d < cap) arena[d] = src < cap ? arena[src] : 0;
          }
        sp.offset = cur;
        std::memcpy(rec + slots[o.second].member, &sp, sizeof(sp));
        cur += bytes;
      }
    }
  }
}

template <class R>
int decode_impl(const Schema& sc, const uint8_t* in, uint64_t in_len,
                const uint64_t* offsets, uint64_t n, uint8_t* recs,
                uint8_t* arena, uint64_t arena_cap, const Limits& lim,
                tgpu_status* st, uint64_t* n_dec, uint64_t* consumed) {
  DecodeCtx dc{&sc, arena, arena_cap,
               has_string_elems(sc) ? (R::kArenaScale == 1 ? 4u : 16u) : R::kArenaScale};
  if (nested_schema(sc)) {
    dc.regions = true;
    dc.scale = region_scale(sc, R::kArenaScale != 1);
  }
  uint64_t pos = offsets ? offsets[0] : 0;
  const uint32_t rs = sc.s[0].size;
  const std::vector<PackSlot> slots = dc.regions ? std::vector<PackSlot>() : block_pack_slots(sc);
  std::vector<uint64_t> starts;
  auto pack = [&](uint64_t m) {
    if (!slots.empty() && m) pack_blocks(sc, slots, starts.data(), m, recs, arena, arena_cap, dc.scale);
  };
  for (uint64_t i = 0; i < n; ++i) {
    uint8_t* rec = recs + i * rs;
    init_record(sc, rec);
    const uint64_t start = offsets ? offsets[i] : pos;
    if (!slots.empty()) starts.push_back(start);
    R r;
    r.c = Cursor{in, start, in_len};
    r.lim = lim;
    r.height.h = lim.initial_height();
    dc.bump = dc.scale * start;  // the record's region (nested schemas)
    try {
      readStruct(r, 0, rec, dc);
    } catch (const OErr& e) {
      pack(i + 1);
      set_status(st, e.code, i, e.off);
      if (n_dec) *n_dec = i;
      if (consumed) *consumed = start - (offsets ? offsets[0] : 0);
      return e.code;
    }
    if (offsets && r.c.pos != offsets[i + 1]) {
      pack(i + 1);
      set_status(st, TGPU_ERR_INDEX_MISMATCH, i, r.c.pos);
      if (n_dec) *n_dec = i;
      if (consumed) *consumed = start - offsets[0];
      return TGPU_ERR_INDEX_MISMATCH;
    }
    pos = r.c.pos;
  }
  pack(n);
  set_status(st, TGPU_OK, n, 0);
  if (n_dec) *n_dec = n;
  if (consumed) *consumed = pos - (offsets ? offsets[0] : 0);
  return TGPU_OK;
}

// ================================================================ writers ===
struct Sink {
  uint8_t* out;  // may be null (size only)
  uint64_t pos, cap;
  void put(uint8_t b) {
    if (out) {
      if (pos >= cap) fail(TGPU_ERR_OUTPUT_OVERFLOW, pos);
      out[pos] = b;
    }
    ++pos;
  }
  void putBE(uint64_t v, int nbytes) {
    for (int i = nbytes - 1; i >= 0; --i) put((uint8_t)(v >> (8 * i)));
  }
  void putBytes(const uint8_t* p, uint64_t n) {
    if (out) {
      if (pos + n > cap) fail(TGPU_ERR_OUTPUT_OVERFLOW, pos);
      std::memcpy(out + pos, p, n);
    }
    pos += n;
  }
  // writeVarintSlow / writeVarintUnrolled (VarintUtils-inl.h:413-447); the
  // BMI2 branch-free encoder (:545-595) produces the same bytes.
  void varint(uint64_t v) {
    while (v & ~0x7full) {
      put((uint8_t)((v & 0x7f) | 0x80));
      v >>= 7;
    }
    put((uint8_t)v);
  }
};

struct EncodeCtx {
  const Schema* sc;
  const uint8_t* sbase;
  const uint8_t* lbase;
};

tgpu_span ld_span(const uint8_t* p) {
  tgpu_span v;
  std::memcpy(&v, p, sizeof(v));
  return v;
}

// A union writes its active member only (serialize_union.whisker:52-66,
// switch (getType())): the first member whose isset byte is set, or none.
void union_range(const EncodeCtx& ec, const tgpu_struct_desc& sd, const uint8_t* obj,
                 uint32_t& k0, uint32_t& k1) {
  if (!(sd.flags & TGPU_STRUCT_UNION)) return;
  k0 = k1 = sd.num_fields;
  for (uint32_t k = 0; k < sd.num_fields; ++k) {
    if (obj[ec.sc->f[sd.first_field + k].isset_offset]) {
      k0 = k;
      k1 = k + 1;
      return;
    }
  }
}

// The object a struct member holds: the member itself, or for a boxed member
// the object its pointer (span into list_base) names; nullptr for a null
// pointer, which serialize_field.whisker:44-49 writes as an empty struct
// (writeStructBegin, writeFieldStop, writeStructEnd).
const uint8_t* boxed_object(const EncodeCtx& ec, const tgpu_field_desc& f, const uint8_t* m) {
  if (!is_boxed(f)) return m;
  const tgpu_span sp = ld_span(m);
  return sp.length ? ec.lbase + sp.offset : nullptr;
}

uint8_t load_bool_checked(const uint8_t* p, uint64_t off) {
  // validate_bool (Protocol.h:126-163): LOG(FATAL) on a byte not in {0,1}.
  if (*p > 1) fail(TGPU_ERR_INVALID_BOOL_WRITE, off);
  return *p;
}

template <class T>
T ld(const uint8_t* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

// BinaryProtocolWriter (BinaryProtocol-inl.h:41-222) + generated write
// (serialize_struct.whisker:40-67; gen/module_types_tcc.h:106-121).
struct BinaryWriter {
  Sink s;
  void stringLen(uint32_t n) { s.putBE(n, 4); }
  void scalar(uint8_t t, const uint8_t* p) {
    switch (t) {
      case TGPU_T_BOOL: s.put(load_bool_checked(p, s.pos)); break;
      case TGPU_T_BYTE: s.put(*p); break;
      case TGPU_T_I16: s.putBE((uint16_t)ld<int16_t>(p), 2); break;
      case TGPU_T_I32: case TGPU_T_FLOAT: s.putBE(ld<uint32_t>(p), 4); break;
      default: s.putBE(ld<uint64_t>(p), 8); break;
    }
  }
  // writeMapBegin / writeListBegin (BinaryProtocol-inl.h:69-96)
  void header(const CT& c, uint32_t n) {
    if (c.ttype == TGPU_T_MAP) {
      s.put(c.elem);
      s.put(c.val);
    } else {
      s.put(c.elem);
    }
    s.putBE(n, 4);
  }
  // a list/set element or map value: a struct (the generated write), a
  // container, or a scalar / string
  void value(const EncodeCtx& ec, uint8_t t, int32_t si, uint32_t ti, const uint8_t* p) {
    if (t == TGPU_T_STRUCT) structure(ec, (uint32_t)si, p);
    else if (is_container_t(t)) container(ec, ct_node(*ec.sc, ti), p);
    else elem(ec, t, p);
  }
  // protocol_methods<list/set/map>::write (protocol_methods.h:469-489,
  // 693-701): header, then the elements (key then value per pair) in the
  // given order
  void container(const EncodeCtx& ec, const CT& c, const uint8_t* m) {
    const tgpu_span sp = ld<tgpu_span>(m);
    if (sp.length > 0x7fffffffu) fail(TGPU_ERR_WRITE_SIZE_LIMIT, s.pos);  // checked_container_size
    header(c, sp.length);
    const bool is_map = c.ttype == TGPU_T_MAP;
    const uint8_t v = is_map ? c.val : c.elem;
    const int32_t ksi = is_map ? key_si(*ec.sc, c) : -1;
    const uint32_t ks = is_map ? slot_size(*ec.sc, c.elem, ksi) : 0;
    const uint32_t ps = ks + slot_size(*ec.sc, v, c.si);
    const uint8_t* e = ec.lbase + sp.offset;
    for (uint32_t i = 0; i < sp.length; ++i) {
      if (is_map) value(ec, c.elem, ksi, key_ti(c), e + (uint64_t)i * ps);
      value(ec, v, c.si, c.ti, e + (uint64_t)i * ps + ks);
    }
  }
  // a container element: scalar, or a string span into string_base
  // (writeBinary: checkBinarySize then the length and bytes)
  void elem(const EncodeCtx& ec, uint8_t t, const uint8_t* p) {
    if (t != TGPU_T_STRING) return scalar(t, p);
    const tgpu_span sp = ld<tgpu_span>(p);
    if (sp.length > 0x7fffffffu) fail(TGPU_ERR_WRITE_SIZE_LIMIT, s.pos);
    stringLen(sp.length);
    s.putBytes(ec.sbase + sp.offset, sp.length);
  }
  void structure(const EncodeCtx& ec, uint32_t si, const uint8_t* obj) {
    const tgpu_struct_desc& sd = ec.sc->s[si];
    uint32_t k0 = 0, k1 = sd.num_fields;
    union_range(ec, sd, obj, k0, k1);
    for (uint32_t k = k0; k < k1; ++k) {
      const tgpu_field_desc& f = ec.sc->f[sd.first_field + k];
      if ((f.qualifier == TGPU_OPTIONAL || f.qualifier == TGPU_OPTIONAL_BOXED) &&
          !obj[f.isset_offset])
        continue;
      const uint8_t* m = obj + f.member_offset;
      if (f.qualifier == TGPU_TERSE && terse_empty(*ec.sc, f, m)) continue;  // fields.whisker:84
      s.put(f.ttype);  // writeFieldBegin: byte type + BE i16 id
      s.putBE((uint16_t)f.id, 2);
      if (is_scalar(f.ttype)) {
        scalar(f.ttype, m);
      } else if (f.ttype == TGPU_T_STRING) {
        const tgpu_span sp = ld<tgpu_span>(m);
        if (sp.length > 0x7fffffffu) fail(TGPU_ERR_WRITE_SIZE_LIMIT, s.pos);  // checkBinarySize
        s.putBE(sp.length, 4);
        s.putBytes(ec.sbase + sp.offset, sp.length);
      } else if (f.ttype == TGPU_T_STRUCT) {
        const uint8_t* o = boxed_object(ec, f, m);
        if (o) structure(ec, (uint32_t)f.struct_index, o);
        else s.put(TGPU_T_STOP);  // a null ref: an empty struct
      } else {  // list / set / map
        container(ec, ct_of(f), m);
      }
    }
    s.put(TGPU_T_STOP);  // writeFieldStop
  }
};

// CompactProtocolWriter (CompactProtocol-inl.h:91-383); kV1: CompactV1
// (CompactV1Protocol-inl.h:36-41, doubles little-endian).
template <bool kV1>
struct CompactWriterT {
  Sink s;
  void stringLen(uint32_t n) { s.varint(n); }
  void fieldHeader(uint8_t ctype, int16_t id, int16_t& last) {  // :133-160
    if (id > last && id - last <= 15) {
      s.put((uint8_t)(((id - last) << 4) | ctype));
    } else {
      s.put(ctype);
      s.varint(i32ToZigzag(id));  // writeI16 -> i32ToZigzag -> writeVarint
    }
    last = id;
  }
  void scalar(uint8_t t, const uint8_t* p) {
    switch (t) {
      case TGPU_T_BOOL: s.put(load_bool_checked(p, s.pos) ? 1 : 2); break;  // :252-273 (container form)
      case TGPU_T_BYTE: s.put(*p); break;
      case TGPU_T_I16: s.varint(i32ToZigzag(ld<int16_t>(p))); break;
      case TGPU_T_I32: s.varint(i32ToZigzag(ld<int32_t>(p))); break;
      case TGPU_T_I64: s.varint(i64ToZigzag(ld<int64_t>(p))); break;
      case TGPU_T_FLOAT: s.putBE(ld<uint32_t>(p), 4); break;
      default:  // double: BE (v2); V1 writes it little-endian
        s.putBE(kV1 ? __builtin_bswap64(ld<uint64_t>(p)) : ld<uint64_t>(p), 8);
        break;
    }
  }
  // writeMapBegin (:182-201) / writeCollectionBegin (:209-224)
  void header(const CT& c, uint32_t n) {
    if (c.ttype == TGPU_T_MAP) {
      if (n == 0) {
        s.put(0);
      } else {
        s.varint(n);
        s.put((uint8_t)((ttypeToCType(c.elem) << 4) | ttypeToCType(c.val)));
      }
      return;
    }
    const uint8_t ct = ttypeToCType(c.elem);
    if (n <= 14) {
      s.put((uint8_t)((n << 4) | ct));
    } else {
      s.put((uint8_t)(0xf0 | ct));
      s.varint(n);
    }
  }
  // a list/set element or map value: a struct (the generated write), a
  // container, or a scalar / string
  void value(const EncodeCtx& ec, uint8_t t, int32_t si, uint32_t ti, const uint8_t* p) {
    if (t == TGPU_T_STRUCT) structure(ec, (uint32_t)si, p);
    else if (is_container_t(t)) container(ec, ct_node(*ec.sc, ti), p);
    else elem(ec, t, p);
  }
  // protocol_methods<list/set/map>::write (protocol_methods.h:469-489,
  // 693-701): header, then the elements (key then value per pair) in the
  // given order
  void container(const EncodeCtx& ec, const CT& c, const uint8_t* m) {
    const tgpu_span sp = ld<tgpu_span>(m);
    if (sp.length > 0x7fffffffu) fail(TGPU_ERR_WRITE_SIZE_LIMIT, s.pos);  // checked_container_size
    header(c, sp.length);
    const bool is_map = c.ttype == TGPU_T_MAP;
    const uint8_t v = is_map ? c.val : c.elem;
    const int32_t ksi = is_map ? key_si(*ec.sc, c) : -1;
    const uint32_t ks = is_map ? slot_size(*ec.sc, c.elem, ksi) : 0;
    const uint32_t ps = ks + slot_size(*ec.sc, v, c.si);
    const uint8_t* e = ec.lbase + sp.offset;
    for (uint32_t i = 0; i < sp.length; ++i) {
      if (is_map) value(ec, c.elem, ksi, key_ti(c), e + (uint64_t)i * ps);
      value(ec, v, c.si, c.ti, e + (uint64_t)i * ps + ks);
    }
  }
  // a container element: scalar, or a string span into string_base
  // (writeBinary: checkBinarySize then the length and bytes)
  void elem(const EncodeCtx& ec, uint8_t t, const uint8_t* p) {
    if (t != TGPU_T_STRING) return scalar(t, p);
    const tgpu_span sp = ld<tgpu_span>(p);
    if (sp.length > 0x7fffffffu) fail(TGPU_ERR_WRITE_SIZE_LIMIT, s.pos);
    stringLen(sp.length);
    s.putBytes(ec.sbase + sp.offset, sp.length);
  }
  void structure(const EncodeCtx& ec, uint32_t si, const uint8_t* obj) {
    const tgpu_struct_desc& sd = ec.sc->s[si];
    int16_t last = 0;  // writeStructBegin pushes lastFieldId_ and resets it
    uint32_t k0 = 0, k1 = sd.num_fields;
    union_range(ec, sd, obj, k0, k1);
    for (uint32_t k = k0; k < k1; ++k) {
      const tgpu_field_desc& f = ec.sc->f[sd.first_field + k];
      if ((f.qualifier == TGPU_OPTIONAL || f.qualifier == TGPU_OPTIONAL_BOXED) &&
          !obj[f.isset_offset])
        continue;
      const uint8_t* m = obj + f.member_offset;
      if (f.qualifier == TGPU_TERSE && terse_empty(*ec.sc, f, m)) continue;  // fields.whisker:84
      if (f.ttype == TGPU_T_BOOL) {  // bool value rides in the header
        const uint8_t b = load_bool_checked(m, s.pos);
        fieldHeader(b ? 1 : 2, f.id, last);
        continue;
      }
      fieldHeader(ttypeToCType(f.ttype), f.id, last);
      if (is_scalar(f.ttype)) {
        scalar(f.ttype, m);
      } else if (f.ttype == TGPU_T_STRING) {
        const tgpu_span sp = ld<tgpu_span>(m);
        if (sp.length > 0x7fffffffu) fail(TGPU_ERR_WRITE_SIZE_LIMIT, s.pos);
        s.varint(sp.length);  // writeVarint(out_, (int32_t)size)
        s.putBytes(ec.sbase + sp.offset, sp.length);
      } else if (f.ttype == TGPU_T_STRUCT) {
        const uint8_t* o = boxed_object(ec, f, m);
        if (o) structure(ec, (uint32_t)f.struct_index, o);
        else s.put(0);  // a null ref: an empty struct (writeFieldStop only)
      } else {  // list / set / map
        container(ec, ct_of(f), m);
      }
    }
    s.put(0);  // writeFieldStop
  }
};

using CompactWriter = CompactWriterT<false>;
using CompactV1Writer = CompactWriterT<true>;

template <class W>
int encode_impl(const Schema& sc, const uint8_t* recs, uint64_t n,
                const uint8_t* sbase, const uint8_t* lbase, uint8_t* out,
                uint64_t cap, uint64_t* offs, tgpu_status* st,
                uint64_t* out_size) {
  EncodeCtx ec{&sc, sbase, lbase};
  W w;
  w.s = Sink{out, 0, cap};
  const uint32_t rs = sc.s[0].size;
  for (uint64_t i = 0; i < n; ++i) {
    if (offs) offs[i] = w.s.pos;
    const uint64_t start = w.s.pos;
    try {
      w.structure(ec, 0, recs + i * rs);
    } catch (const OErr& e) {
      set_status(st, e.code, i, e.off);
      if (out_size) *out_size = start;
      return e.code;
    }
  }
  if (offs) offs[n] = w.s.pos;
  set_status(st, TGPU_OK, n, 0);
  if (out_size) *out_size = w.s.pos;
  return TGPU_OK;
}

Limits to_limits(const tgpu_limits* l) {
  Limits r;
  if (l) {
    r.string_limit = l->string_limit;
    r.container_limit = l->container_limit;
    r.max_depth = l->max_depth;
    r.height = l->height;
  }
  return r;
}

template <class F>
void parallel_for(uint64_t n, int threads, F&& fn) {
  if (threads <= 1 || n < 1024) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> ts;
  const uint64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const uint64_t b = std::min(n, chunk * t), e = std::min(n, chunk * (t + 1));
    if (b < e) ts.emplace_back([&fn, b, e] { fn(b, e); });
  }
  for (auto& t : ts) t.join();
}

inline uint64_t load_be64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}

}  // namespace

// ================================================================ C entry ===
extern "C" {

int oracle_encode_batch_ex(const tgpu_struct_desc* structs, uint32_t n_structs,
                        const tgpu_field_desc* fields, uint32_t n_fields,
                        const tgpu_type_desc* types, uint32_t n_types,
                        int protocol, const void* records, uint64_t n_records,
                        const void* string_base, const void* list_base,
                        void* out, uint64_t out_capacity, uint64_t* out_offsets,
                        tgpu_status* st, uint64_t* out_size) {
  Schema sc{structs, n_structs, fields, n_fields, types, n_types};
  auto rec = (const uint8_t*)records;
  auto sb = (const uint8_t*)string_base;
  auto lb = (const uint8_t*)list_base;
  if (protocol == TGPU_PROTOCOL_BINARY)
    return encode_impl<BinaryWriter>(sc, rec, n_records, sb, lb, (uint8_t*)out,
                                     out_capacity, out_offsets, st, out_size);
  if (protocol == TGPU_PROTOCOL_COMPACT)
    return encode_impl<CompactWriter>(sc, rec, n_records, sb, lb, (uint8_t*)out,
                                      out_capacity, out_offsets, st, out_size);
  if (protocol == TGPU_PROTOCOL_COMPACT_V1)
    return encode_impl<CompactV1Writer>(sc, rec, n_records, sb, lb, (uint8_t*)out,
                                        out_capacity, out_offsets, st, out_size);
  set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
  return TGPU_ERR_INVALID_ARGUMENT;
}

int oracle_encode_batch(const tgpu_struct_desc* structs, uint32_t n_structs,
                        const tgpu_field_desc* fields, uint32_t n_fields,
                        int protocol, const void* records, uint64_t n_records,
                        const void* string_base, const void* list_base,
                        void* out, uint64_t out_capacity, uint64_t* out_offsets,
                        tgpu_status* st, uint64_t* out_size) {
  return oracle_encode_batch_ex(structs, n_structs, fields, n_fields, nullptr, 0, protocol,
                                records, n_records, string_base, list_base, out, out_capacity,
                                out_offsets, st, out_size);
}

int oracle_decode_batch_ex(const tgpu_struct_desc* structs, uint32_t n_structs,
                        const tgpu_field_desc* fields, uint32_t n_fields,
                        const tgpu_type_desc* types, uint32_t n_types,
                        int protocol, const void* in, uint64_t in_len,
                        const uint64_t* offsets, uint64_t n_records,
                        void* records, void* list_arena,
                        uint64_t list_arena_capacity, const tgpu_limits* limits,
                        tgpu_status* st, uint64_t* n_decoded,
                        uint64_t* consumed) {
  Schema sc{structs, n_structs, fields, n_fields, types, n_types};
  const Limits lim = to_limits(limits);
  auto p = (const uint8_t*)in;
  if (protocol == TGPU_PROTOCOL_BINARY)
    return decode_impl<BinaryReader>(sc, p, in_len, offsets, n_records,
                                     (uint8_t*)records, (uint8_t*)list_arena,
                                     list_arena_capacity, lim, st, n_decoded,
                                     consumed);
  if (protocol == TGPU_PROTOCOL_COMPACT)
    return decode_impl<CompactReader>(sc, p, in_len, offsets, n_records,
                                      (uint8_t*)records, (uint8_t*)list_arena,
                                      list_arena_capacity, lim, st, n_decoded,
                                      consumed);
  if (protocol == TGPU_PROTOCOL_COMPACT_V1)
    return decode_impl<CompactV1Reader>(sc, p, in_len, offsets, n_records,
                                        (uint8_t*)records, (uint8_t*)list_arena,
                                        list_arena_capacity, lim, st, n_decoded,
                                        consumed);
  set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
  return TGPU_ERR_INVALID_ARGUMENT;
}

int oracle_decode_batch(const tgpu_struct_desc* structs, uint32_t n_structs,
                        const tgpu_field_desc* fields, uint32_t n_fields,
                        int protocol, const void* in, uint64_t in_len,
                        const uint64_t* offsets, uint64_t n_records,
                        void* records, void* list_arena,
                        uint64_t list_arena_capacity, const tgpu_limits* limits,
                        tgpu_status* st, uint64_t* n_decoded,
                        uint64_t* consumed) {
  return oracle_decode_batch_ex(structs, n_structs, fields, n_fields, nullptr, 0, protocol, in,
                                in_len, offsets, n_records, records, list_arena,
                                list_arena_capacity, limits, st, n_decoded, consumed);
}

// Arena bytes per input byte a decode of this schema needs (the library's
// tgpu_schema_arena_scale, restated).
uint32_t oracle_arena_scale(const tgpu_struct_desc* structs, uint32_t n_structs,
                            const tgpu_field_desc* fields, uint32_t n_fields,
                            const tgpu_type_desc* types, uint32_t n_types, int protocol) {
  Schema sc{structs, n_structs, fields, n_fields, types, n_types};
  const bool bin = protocol == TGPU_PROTOCOL_BINARY;
  bool lists = false;
  for (uint32_t k = 0; k < n_fields; ++k)
    lists |= is_container_t(fields[k].ttype) || is_boxed(fields[k]);  // boxed objects: the arena
  if (!lists) return 0;
  if (nested_schema(sc)) return region_scale(sc, !bin);
  return has_string_elems(sc) ? (bin ? 4 : 16) : (bin ? 1 : 8);
}

int64_t oracle_record_length(int protocol, const void* in, uint64_t in_len,
                             uint64_t pos, int32_t max_depth, int32_t height) {
  Limits lim;
  lim.max_depth = max_depth;
  lim.height = height;
  try {
    if (protocol == TGPU_PROTOCOL_BINARY) {
      BinaryReader r;
      r.c = Cursor{(const uint8_t*)in, pos, in_len};
      r.lim = lim;
      r.height.h = lim.initial_height();
      r.skip(TGPU_T_STRUCT, 0);
      return (int64_t)(r.c.pos - pos);
    }
    CompactReader r;
    r.c = Cursor{(const uint8_t*)in, pos, in_len};
    r.lim = lim;
    r.height.h = lim.initial_height();
    r.skip(TGPU_T_STRUCT, 0);
    return (int64_t)(r.c.pos - pos);
  } catch (const OErr& e) {
    return -(int64_t)e.code;
  }
}

int64_t oracle_skip_value(int protocol, const void* in, uint64_t in_len, uint64_t pos,
                          int ttype, int32_t max_depth, int32_t height) {
  Limits lim;
  lim.max_depth = max_depth;
  lim.height = height;
  try {
    if (protocol == TGPU_PROTOCOL_BINARY) {
      BinaryReader r;
      r.c = Cursor{(const uint8_t*)in, pos, in_len};
      r.lim = lim;
      r.height.h = lim.initial_height();
      r.skip((uint8_t)ttype, 0);
      return (int64_t)(r.c.pos - pos);
    }
    CompactReader r;
    r.c = Cursor{(const uint8_t*)in, pos, in_len};
    r.lim = lim;
    r.height.h = lim.initial_height();
    r.skip((uint8_t)ttype, 0);
    return (int64_t)(r.c.pos - pos);
  } catch (const OErr& e) {
    return -(int64_t)e.code;
  }
}

// Schemaless skim: the field loop of protocol::parseObject
// (protocol/detail/Object.h:416-432) keeping each value as the bytes
// apache::thrift::skip passes over (setMaskedDataFull,
// protocol/detail/FieldMaskUtil.h:373-388); bools are read
// (FieldMaskUtil.h:441-450). Sequential, record by record; stops at the
// first record the reader rejects or whose end disagrees with offsets[i+1].
// One struct level of it: every field's entry in pre-order; a struct-valued
// field below max_nest recurses as parseValue -> parseObjectInplace does,
// after the checks skip(T_STRUCT, level) makes (max_depth, readStructBegin's
// descend, Protocol.h:187-283); any other value is passed over by skip at
// this level's depth.
extern "C++" template <class R>
void skim_level(R& r, uint32_t level, uint32_t max_nest, uint64_t i, uint64_t n,
                tgpu_skim_field* fields, uint32_t max_fields, uint32_t& count) {
  int16_t prev = 0;
  while (true) {
    uint8_t wt;
    int16_t id;
    if (!r.readFieldHeader(prev, wt, id)) return;
    prev = id;
    const uint64_t off = r.c.pos;
    const uint32_t slot = count++;
    uint8_t flags = (uint8_t)(level << TGPU_SKIM_LEVEL_SHIFT);
    if (wt == TGPU_T_STRUCT && level < max_nest) {
      if ((int64_t)level >= r.lim.max_depth) fail(TGPU_ERR_DEPTH_LIMIT, off);
      r.height.descend(off);  // readStructBegin
      skim_level(r, level + 1, max_nest, i, n, fields, max_fields, count);
      r.height.ascend();      // readStructEnd
    } else if (wt == TGPU_T_BOOL) {
      flags |= TGPU_SKIM_BOOL | (r.readBool() ? TGPU_SKIM_TRUE : 0);
    } else {
      r.skip(wt, (int)level);
    }
    // an entry's length is 32 bits: a longer value is not representable
    if (r.c.pos - off > 0xffffffffull) fail(TGPU_ERR_UNSUPPORTED, off);
    if (slot < max_fields) {
      tgpu_skim_field& f = fields[(uint64_t)slot * n + i];
      f.id = id;
      f.ttype = wt;
      f.flags = flags;
      f.length = (uint32_t)(r.c.pos - off);
      f.offset = off;
    }
  }
}

extern "C++" template <class R>
int skim_impl(const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
              tgpu_skim_field* fields, uint32_t max_fields, uint32_t* counts, uint32_t max_nest,
              const Limits& lim, tgpu_status* st, uint64_t* n_done) {
  for (uint64_t i = 0; i < n; ++i) {
    R r;
    r.c = Cursor{in, offsets[i], in_len};
    r.lim = lim;
    r.height.h = lim.initial_height();
    uint32_t count = 0;
    try {
      if (offsets[i] > in_len || offsets[i + 1] < offsets[i])
        fail(TGPU_ERR_INDEX_MISMATCH, offsets[i]);
      skim_level(r, 0, max_nest, i, n, fields, max_fields, count);
      counts[i] = count;
      if (r.c.pos != offsets[i + 1]) fail(TGPU_ERR_INDEX_MISMATCH, r.c.pos);
    } catch (const OErr& e) {
      set_status(st, e.code, i, e.off);
      if (n_done) *n_done = i;
      return e.code;
    }
  }
  set_status(st, TGPU_OK, n, 0);
  if (n_done) *n_done = n;
  return TGPU_OK;
}

int oracle_skim_batch_ex(int protocol, const void* in, uint64_t in_len, const uint64_t* offsets,
                         uint64_t n_records, tgpu_skim_field* fields, uint32_t max_fields,
                         uint32_t* field_counts, uint32_t max_nest, const tgpu_limits* limits,
                         tgpu_status* st, uint64_t* n_done) {
  const Limits lim = to_limits(limits);
  auto p = (const uint8_t*)in;
  if (max_nest > TGPU_SKIM_MAX_NEST) {
    set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  if (protocol == TGPU_PROTOCOL_BINARY)
    return skim_impl<BinaryReader>(p, in_len, offsets, n_records, fields, max_fields,
                                   field_counts, max_nest, lim, st, n_done);
  if (protocol == TGPU_PROTOCOL_COMPACT)
    return skim_impl<CompactReader>(p, in_len, offsets, n_records, fields, max_fields,
                                    field_counts, max_nest, lim, st, n_done);
  if (protocol == TGPU_PROTOCOL_COMPACT_V1)
    return skim_impl<CompactV1Reader>(p, in_len, offsets, n_records, fields, max_fields,
                                      field_counts, max_nest, lim, st, n_done);
  set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
  return TGPU_ERR_INVALID_ARGUMENT;
}

int oracle_skim_batch(int protocol, const void* in, uint64_t in_len, const uint64_t* offsets,
                      uint64_t n_records, tgpu_skim_field* fields, uint32_t max_fields,
                      uint32_t* field_counts, const tgpu_limits* limits, tgpu_status* st,
                      uint64_t* n_done) {
  return oracle_skim_batch_ex(protocol, in, in_len, offsets, n_records, fields, max_fields,
                              field_counts, 0, limits, st, n_done);
}

int oracle_read_varint(const void* in, uint64_t len, int bits, uint64_t* value,
                       uint64_t* consumed) {
  Cursor c{(const uint8_t*)in, 0, len};
  try {
    uint64_t v = 0;
    if (bits == 64) v = readVarint<64>(c);
    else if (bits == 32) v = readVarint<32>(c);
    else if (bits == 16) v = (uint16_t)readVarint<32>(c);  // i16 reads via i32
    else return TGPU_ERR_INVALID_ARGUMENT;
    *value = v;
    *consumed = c.pos;
    return TGPU_OK;
  } catch (const OErr& e) {
    *consumed = c.pos;
    return e.code;
  }
}

int oracle_write_varint(uint64_t value, void* out) {
  Sink s{(uint8_t*)out, 0, 16};
  s.varint(value);
  return (int)s.pos;
}

// ---- codegen-equivalent flat {1..8: i64}, Binary ---------------------------
// Generated readNoXfer (deserialize_struct.whisker:19-160) with
// BinaryProtocolReader::advanceToNextField's fast path (BinaryProtocol-inl.h
// :586-621): >= 3 bytes, type byte == T_I64, BE id == expected -> readBE<i64>.
// Baseline timing runs on canonical streams only: a miss (the generated
// _loop / switch / skip path) is reported as TGPU_ERR_UNSUPPORTED and the
// caller uses oracle_decode_batch for irregular streams.
int oracle_flat8_binary_decode(const void* in, uint64_t n, void* records,
                               int n_threads) {
  const uint8_t* p = (const uint8_t*)in;
  uint8_t* out = (uint8_t*)records;
  int rc = TGPU_OK;
  parallel_for(n, n_threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      const uint8_t* r = p + i * 89;
      uint8_t* o = out + i * 72;
      bool ok = true;
      for (int k = 0; k < 8 && ok; ++k) {
        const uint8_t* f = r + 11 * k;
        ok = f[0] == TGPU_T_I64 && f[1] == 0 && f[2] == (uint8_t)(k + 1);
        if (ok) {
          const uint64_t v = load_be64(f + 3);
          std::memcpy(o + 8 * k, &v, 8);
          o[64 + k] = 1;
        }
      }
      if (!ok || r[88] != TGPU_T_STOP) rc = TGPU_ERR_UNSUPPORTED;  // irregular
    }
  });
  return rc;
}

int oracle_flat8_binary_encode(const void* records, uint64_t n, void* out,
                               int n_threads) {
  const uint8_t* rp = (const uint8_t*)records;
  uint8_t* o = (uint8_t*)out;
  parallel_for(n, n_threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      const uint8_t* r = rp + i * 72;
      uint8_t* w = o + i * 89;
      for (int k = 0; k < 8; ++k) {
        w[11 * k] = TGPU_T_I64;
        w[11 * k + 1] = 0;
        w[11 * k + 2] = (uint8_t)(k + 1);
        uint64_t v;
        std::memcpy(&v, r + 8 * k, 8);
        v = __builtin_bswap64(v);
        std::memcpy(w + 11 * k + 3, &v, 8);
      }
      w[88] = TGPU_T_STOP;
    }
  });
  return TGPU_OK;
}

// ---- codegen-equivalent {1..4: i32, 5..6: string}, Compact -----------------
// Device layout: i32 @0,4,8,12; span @16,32; isset[6] @48; size 56.
int oracle_mixed_compact_decode(const void* in, const uint64_t* offsets,
                                uint64_t n, void* records, int n_threads) {
  const uint8_t* p = (const uint8_t*)in;
  uint8_t* out = (uint8_t*)records;
  int rc = TGPU_OK;
  parallel_for(n, n_threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      uint8_t* o = out + i * 56;
      std::memset(o, 0, 56);
      CompactReader r;
      r.c = Cursor{p, offsets[i], offsets[n]};
      r.height.h = 12001;
      try {
        // advanceToNextField(prev, next, T_I32): 1-byte header (Δ=1 | CT_I32)
        for (int k = 0; k < 4; ++k) {
          if (r.c.avail() && r.c.p[r.c.pos] == 0x15) {
            r.c.pos++;
            const int32_t v = zigzagToI32((uint32_t)readVarint<32>(r.c));
            std::memcpy(o + 4 * k, &v, 4);
            o[48 + k] = 1;
          } else {
            throw OErr{TGPU_ERR_UNSUPPORTED, r.c.pos};
          }
        }
        for (int k = 0; k < 2; ++k) {
          if (r.c.avail() && r.c.p[r.c.pos] == 0x18) {
            r.c.pos++;
            tgpu_span sp{0, 0, 0};
            r.readString(sp.offset, sp.length);
            std::memcpy(o + 16 + 16 * k, &sp, 16);
            o[52 + k] = 1;
          } else {
            throw OErr{TGPU_ERR_UNSUPPORTED, r.c.pos};
          }
        }
        if (!(r.c.avail() && r.c.p[r.c.pos] == 0)) throw OErr{TGPU_ERR_UNSUPPORTED, r.c.pos};
      } catch (const OErr& err) {
        rc = err.code;
      }
    }
  });
  return rc;
}

int oracle_mixed_compact_encode(const void* records, uint64_t n,
                                const void* string_base, void* out,
                                const uint64_t* offsets, int n_threads) {
  const uint8_t* rp = (const uint8_t*)records;
  const uint8_t* sb = (const uint8_t*)string_base;
  uint8_t* o = (uint8_t*)out;
  parallel_for(n, n_threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      const uint8_t* r = rp + i * 56;
      Sink s{o, offsets[i], offsets[n]};
      for (int k = 0; k < 4; ++k) {
        s.put(0x15);
        s.varint(i32ToZigzag(ld<int32_t>(r + 4 * k)));
      }
      for (int k = 0; k < 2; ++k) {
        const tgpu_span sp = ld<tgpu_span>(r + 16 + 16 * k);
        s.put(0x18);
        s.varint(sp.length);
        s.putBytes(sb + sp.offset, sp.length);
      }
      s.put(0);
    }
  });
  return TGPU_OK;
}

// serializedSize of the codegen-equivalent mixed record (exact, the size
// pass a contiguous multi-threaded encode needs): sizes[i], then the
// exclusive prefix is the caller's (out_offsets = sizes scanned).
int oracle_mixed_compact_size(const void* records, uint64_t n, uint64_t* sizes,
                              int n_threads) {
  const uint8_t* rp = (const uint8_t*)records;
  parallel_for(n, n_threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      const uint8_t* r = rp + i * 56;
      Sink s{nullptr, 0, 0};
      for (int k = 0; k < 4; ++k) {
        s.put(0x15);
        s.varint(i32ToZigzag(ld<int32_t>(r + 4 * k)));
      }
      for (int k = 0; k < 2; ++k) {
        const tgpu_span sp = ld<tgpu_span>(r + 16 + 16 * k);
        s.put(0x18);
        s.varint(sp.length);
        s.pos += sp.length;
      }
      s.put(0);
      sizes[i] = s.pos;
    }
  });
  return TGPU_OK;
}

// ---- codegen-equivalent nested {1: i64, 2: list<i32>, 3: Inner{1..3: double}},
// Binary (BASELINE config 4) -------------------------------------------------
// Device layout: i64 @0; span @8; Inner @24 (f64 @24,32,40, isset @48..50);
// isset @56..58; size 64. The generated write (serialize_struct.whisker:40-67)
// / readNoXfer fast path (advanceToNextField, BinaryProtocol-inl.h:586-621;
// readListBegin + readArithmeticVector, BinaryProtocol.cpp:49-72; nested
// struct via beforeSubobject/afterSubobject) restated for this one schema.
// List elements decode natively little-endian into the arena under the
// device's block rule (scale 1 Binary): blocks of kArenaBlock records, each
// block's lists back to back (8-byte aligned) from align8(its first wire
// byte) — each block read by one thread in record order, the arrays written
// where they belong (no move).
namespace {
inline void nested_write(Sink& s, const uint8_t* r, const uint8_t* lb) {
  s.put(TGPU_T_I64); s.putBE(1, 2); s.putBE(ld<uint64_t>(r), 8);
  const tgpu_span sp = ld<tgpu_span>(r + 8);
  s.put(TGPU_T_LIST); s.putBE(2, 2); s.put(TGPU_T_I32); s.putBE(sp.length, 4);
  if (s.out) {
    if (s.pos + 4ull * sp.length > s.cap) fail(TGPU_ERR_OUTPUT_OVERFLOW, s.pos);
    const uint8_t* e = lb + sp.offset;
    uint8_t* o = s.out + s.pos;
    for (uint32_t k = 0; k < sp.length; ++k) {
      const uint32_t v = __builtin_bswap32(ld<uint32_t>(e + 4 * k));
      std::memcpy(o + 4 * k, &v, 4);
    }
  }
  s.pos += 4ull * sp.length;
  s.put(TGPU_T_STRUCT); s.putBE(3, 2);
  for (int k = 0; k < 3; ++k) {
    s.put(TGPU_T_DOUBLE); s.putBE((uint64_t)(k + 1), 2); s.putBE(ld<uint64_t>(r + 24 + 8 * k), 8);
  }
  s.put(0);
  s.put(0);
}
}  // namespace

int oracle_nested_binary_size(const void* records, uint64_t n, uint64_t* sizes, int n_threads) {
  const uint8_t* rp = (const uint8_t*)records;
  parallel_for(n, n_threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i)
      sizes[i] = 57 + 4ull * ld<tgpu_span>(rp + i * 64 + 8).length;
  });
  return TGPU_OK;
}

int oracle_nested_binary_encode(const void* records, uint64_t n, const void* list_base,
                                void* out, const uint64_t* offsets, int n_threads) {
  const uint8_t* rp = (const uint8_t*)records;
  parallel_for(n, n_threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      Sink s{(uint8_t*)out, offsets[i], offsets[n]};
      nested_write(s, rp + i * 64, (const uint8_t*)list_base);
    }
  });
  return TGPU_OK;
}

int oracle_nested_binary_decode(const void* in, const uint64_t* offsets, uint64_t n,
                                void* records, void* arena, int n_threads) {
  const uint8_t* p = (const uint8_t*)in;
  uint8_t* out = (uint8_t*)records;
  uint8_t* ar = (uint8_t*)arena;
  int rc = TGPU_OK;
  auto hdr = [](const uint8_t* q, uint8_t t, int id) {
    return q[0] == t && q[1] == 0 && q[2] == (uint8_t)id;
  };
  const uint64_t nb = (n + kArenaBlock - 1) / kArenaBlock;
  parallel_for(nb, n_threads, [&](uint64_t bb, uint64_t be) {
    for (uint64_t i = bb * kArenaBlock, cur = 0; i < std::min(n, be * kArenaBlock); ++i) {
      if (i % kArenaBlock == 0) cur = (offsets[i] + 7) & ~7ull;  // the block's arrays
      uint8_t* o = out + i * 64;
      std::memset(o, 0, 64);
      uint64_t pos = offsets[i];
      const uint64_t end = offsets[n];
      // the canonical form only (a miss is the generated _loop path: the
      // caller uses oracle_decode_batch for irregular streams)
      if (end - pos < 57 || !hdr(p + pos, TGPU_T_I64, 1)) { rc = TGPU_ERR_UNSUPPORTED; continue; }
      const uint64_t v = load_be64(p + pos + 3);
      std::memcpy(o, &v, 8);
      o[56] = 1;
      pos += 11;
      if (!hdr(p + pos, TGPU_T_LIST, 2) || p[pos + 3] != TGPU_T_I32) { rc = TGPU_ERR_UNSUPPORTED; continue; }
      uint32_t cnt;
      std::memcpy(&cnt, p + pos + 4, 4);
      cnt = __builtin_bswap32(cnt);
      pos += 8;
      if ((int32_t)cnt < 0 || end - pos < 4ull * cnt + 37) { rc = TGPU_ERR_UNSUPPORTED; continue; }
      for (uint32_t k = 0; k < cnt; ++k) {
        uint32_t x;
        std::memcpy(&x, p + pos + 4 * k, 4);
        x = __builtin_bswap32(x);
        std::memcpy(ar + cur + 4 * k, &x, 4);
      }
      const tgpu_span sp{cnt ? cur : 0, cnt, 0};
      std::memcpy(o + 8, &sp, 16);
      if (cnt) cur = (cur + 4ull * cnt + 7) & ~7ull;
      o[57] = 1;
      pos += 4ull * cnt;
      if (!hdr(p + pos, TGPU_T_STRUCT, 3)) { rc = TGPU_ERR_UNSUPPORTED; continue; }
      pos += 3;
      bool ok = true;
      for (int k = 0; k < 3 && ok; ++k) {
        ok = hdr(p + pos, TGPU_T_DOUBLE, k + 1);
        const uint64_t d = load_be64(p + pos + 3);
        std::memcpy(o + 24 + 8 * k, &d, 8);
        o[48 + k] = 1;
        pos += 11;
      }
      if (!ok || p[pos] != 0 || p[pos + 1] != 0) { rc = TGPU_ERR_UNSUPPORTED; continue; }
      o[58] = 1;
    }
  });
  return rc;
}

// A file of records read the reference's way: one cursor, record after
// record (while (!cursor.isAtEnd()) deserialize<T>(cursor), Serializer.h:97-100),
// through the codegen-equivalent mixed reader. Writes the record starts
// (n + 1) and returns the number of records (the stream must hold exactly
// canonical records; 0 otherwise).
uint64_t oracle_mixed_compact_read_file(const void* in, uint64_t in_len, uint64_t max_records,
                                        void* records, uint64_t* offsets) {
  const uint8_t* p = (const uint8_t*)in;
  uint8_t* out = (uint8_t*)records;
  uint64_t pos = 0, i = 0;
  while (pos < in_len && i < max_records) {
    uint8_t* o = out + i * 56;
    std::memset(o, 0, 56);
    CompactReader r;
    r.c = Cursor{p, pos, in_len};
    r.height.h = 12001;
    offsets[i] = pos;
    try {
      for (int k = 0; k < 4; ++k) {
        if (!(r.c.avail() && r.c.p[r.c.pos] == 0x15)) return 0;
        r.c.pos++;
        const int32_t v = zigzagToI32((uint32_t)readVarint<32>(r.c));
        std::memcpy(o + 4 * k, &v, 4);
        o[48 + k] = 1;
      }
      for (int k = 0; k < 2; ++k) {
        if (!(r.c.avail() && r.c.p[r.c.pos] == 0x18)) return 0;
        r.c.pos++;
        tgpu_span sp{0, 0, 0};
        r.readString(sp.offset, sp.length);
        std::memcpy(o + 16 + 16 * k, &sp, 16);
        o[52 + k] = 1;
      }
      if (!(r.c.avail() && r.c.p[r.c.pos] == 0)) return 0;
      r.c.pos++;
    } catch (const OErr&) {
      return 0;
    }
    pos = r.c.pos;
    ++i;
  }
  offsets[i] = pos;
  return i;
}

// ---- generators ------------------------------------------------------------
// Counter-based splitmix64 (Steele/Lea/Flood; the survey's PRNG, seed 0x1729 =
// VarintUtilsTestUtil.h:59): z = seed + (index+1)*golden, then the finalizer.
uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t index) {
  uint64_t z = seed + (index + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Config 1/2: value(i, k) = splitmix64_at(seed, 8*i + k); records with
// i % 997 < 5 carry edge values {0, -1, 1, INT64_MIN, INT64_MAX} rotated.
void oracle_gen_flat8(uint64_t seed, uint64_t first, uint64_t n, void* records) {
  static const int64_t edges[5] = {0, -1, 1, INT64_MIN, INT64_MAX};
  uint8_t* o = (uint8_t*)records;
  for (uint64_t j = 0; j < n; ++j) {
    const uint64_t i = first + j;
    uint8_t* r = o + j * 72;
    for (int k = 0; k < 8; ++k) {
      int64_t v = (int64_t)oracle_splitmix64_at(seed, 8 * i + k);
      if (i % 997 < 5) v = edges[(i % 997 + k) % 5];
      std::memcpy(r + 8 * k, &v, 8);
      r[64 + k] = 1;
    }
  }
}

}  // extern "C"
