/*
 * HostBinding.h — host materialization of decoded records into the
 * reference's owning C++ types (std::string, std::vector, std::set,
 * std::map, nested structs) and back into the device form for encoding.
 *
 * The device form of a record (thrift_gpu.h) holds strings and containers as
 * 16-byte spans: into the decoded input (strings) and into the list arena
 * (container elements). A codegen'd T holds them in std::string /
 * std::vector members instead, filled with the reader's default COPY
 * semantics (ExternalBufferSharing::COPY_EXTERNAL_BUFFER, readStringBody,
 * thrift/lib/cpp2/protocol/Protocol.h:406-454). A HostStruct binds each
 * schema field to a member of T by offset and kind — the role of the
 * table-based serializer's FieldInfo::memberOffset and TypeInfo::set / get
 * function pointers (thrift/lib/cpp2/protocol/TableBasedSerializer.h:90-118,
 * 205-302), which thrift1 generates per type; here the bindings are built
 * with the templates below (scalarType, stringType, structType, listType,
 * setType, mapType).
 */
#ifndef THRIFT_GPU_HOST_BINDING_H_
#define THRIFT_GPU_HOST_BINDING_H_

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../thrift_gpu.h"

namespace apache::thrift::gpu {

struct HostStruct;

/* How one value (a field's, an element's, a key's) lives on the host. */
struct HostType {
  enum Kind : uint8_t { Scalar, String, Struct, Container, Boxed };
  using Fill = void (*)(void* ctx, void* elem_or_key, void* val);
  using Visit = void (*)(void* ctx, const void* elem_or_key, const void* val);
  Kind kind = Scalar;
  uint32_t size = 0;              /* Scalar: bytes */
  const HostStruct* st = nullptr; /* Struct */
  /* Container: element (list/set) or key / value (map) types. */
  const HostType* elem = nullptr;
  const HostType* val = nullptr;
  void (*clear)(void* c) = nullptr;
  /* Adds one element: `fill` reads it into a default-constructed element
     (list: appended first, so a failing read leaves it in the list like the
     reader's emplace_back_default; set / map: inserted after the read,
     deserialize_known_length_set / _map, EncodeHelpers.h:188-260). */
  void (*add)(void* c, void* ctx, Fill fill) = nullptr;
  /* Every element in container order (encode). */
  void (*each)(const void* c, void* ctx, Visit fn) = nullptr;
  /* Boxed (a cpp.ref / thrift.box member, e.g. std::unique_ptr<T>; `st` is
     T's binding): a fresh default-constructed T the member now owns, and
     the object the member points to (nullptr: null). */
  void* (*make)(void* member) = nullptr;
  const void* (*get)(const void* member) = nullptr;
};

/* One schema field of a struct, in the schema's declaration order. */
struct HostField {
  const HostType* type = nullptr; /* nullptr: field not materialized */
  uint32_t offset = 0;            /* member offset in the host object */
  int32_t isset = -1;             /* host isset byte offset (-1: none) */
};

struct HostStruct {
  std::vector<HostField> fields;
};

// ---- bindings for common C++ types -----------------------------------------
template <class S>
const HostType* scalarType() {
  static const HostType t{HostType::Scalar, (uint32_t)sizeof(S)};
  return &t;
}
inline const HostType* stringType() {
  static const HostType t{HostType::String};
  return &t;
}
inline HostType structType(const HostStruct* st) {
  HostType t;
  t.kind = HostType::Struct;
  t.st = st;
  return t;
}
/* std::unique_ptr<T> (or another owning pointer with reset / get) for a
   boxed struct field. */
template <class Ptr>
HostType boxType(const HostStruct* st) {
  HostType t;
  t.kind = HostType::Boxed;
  t.st = st;
  t.make = [](void* m) -> void* {
    auto* p = static_cast<Ptr*>(m);
    p->reset(new typename Ptr::element_type());
    return p->get();
  };
  t.get = [](const void* m) -> const void* { return static_cast<const Ptr*>(m)->get(); };
  return t;
}
/* std::vector<E> for list<...>. */
template <class V>
HostType listType(const HostType* elem) {
  HostType t;
  t.kind = HostType::Container;
  t.elem = elem;
  t.clear = [](void* c) { static_cast<V*>(c)->clear(); };
  t.add = [](void* c, void* ctx, HostType::Fill fill) {
    fill(ctx, &static_cast<V*>(c)->emplace_back(), nullptr);
  };
  t.each = [](const void* c, void* ctx, HostType::Visit fn) {
    for (const auto& e : *static_cast<const V*>(c)) fn(ctx, &e, nullptr);
  };
  return t;
}
/* std::set<E> (or any insert-able set) for set<...>. */
template <class C>
HostType setType(const HostType* elem) {
  HostType t;
  t.kind = HostType::Container;
  t.elem = elem;
  t.clear = [](void* c) { static_cast<C*>(c)->clear(); };
  t.add = [](void* c, void* ctx, HostType::Fill fill) {
    typename C::value_type e{};
    fill(ctx, &e, nullptr);
    static_cast<C*>(c)->insert(std::move(e));
  };
  t.each = [](const void* c, void* ctx, HostType::Visit fn) {
    for (const auto& e : *static_cast<const C*>(c)) fn(ctx, &e, nullptr);
  };
  return t;
}
/* std::map<K, V> for map<...>: the first of equal keys wins (emplace). */
template <class C>
HostType mapType(const HostType* key, const HostType* val) {
  HostType t;
  t.kind = HostType::Container;
  t.elem = key;
  t.val = val;
  t.clear = [](void* c) { static_cast<C*>(c)->clear(); };
  t.add = [](void* c, void* ctx, HostType::Fill fill) {
    typename C::key_type k{};
    typename C::mapped_type v{};
    fill(ctx, &k, &v);
    static_cast<C*>(c)->emplace(std::move(k), std::move(v));
  };
  t.each = [](const void* c, void* ctx, HostType::Visit fn) {
    for (const auto& kv : *static_cast<const C*>(c)) fn(ctx, &kv.first, &kv.second);
  };
  return t;
}

/* The schema tables a binding walks (the library's; GpuSchema holds them). */
struct SchemaTables {
  const tgpu_struct_desc* s;
  const tgpu_field_desc* f;
  const tgpu_type_desc* t;
};

namespace detail {

inline uint32_t scalarBytes(uint32_t t) {
  switch (t) {
    case TGPU_T_BOOL: case TGPU_T_BYTE: return 1;
    case TGPU_T_I16: return 2;
    case TGPU_T_I32: case TGPU_T_FLOAT: return 4;
    default: return 8;
  }
}
inline bool isContainer(uint32_t t) {
  return t == TGPU_T_LIST || t == TGPU_T_SET || t == TGPU_T_MAP;
}
inline uint32_t slotBytes(const SchemaTables& sc, uint32_t t, int32_t si) {
  if (t == TGPU_T_STRUCT) return sc.s[si].size;
  if (t == TGPU_T_STRING || isContainer(t)) return 16;
  return scalarBytes(t);
}
/* A container's element / key / value types (from a field or a node). */
struct CType {
  uint32_t ttype, elem, val;
  int32_t si;
  uint32_t ti;
  uint32_t ki;  /* map: 1 + type node of a struct / container key */
};
inline CType ctypeOf(const tgpu_field_desc& f) {
  return CType{f.ttype, f.elem_ttype, f.val_ttype, f.struct_index, f.type_index, f.key_index};
}
inline CType ctypeNode(const SchemaTables& sc, uint32_t ti) {
  const tgpu_type_desc& t = sc.t[ti - 1];
  return CType{t.ttype, t.elem_ttype, t.val_ttype, t.struct_index, t.type_index, t.key_index};
}
/* A map key's struct (a T_STRUCT key node), and its container node. */
inline int32_t keyStruct(const SchemaTables& sc, const CType& c) {
  return (c.elem == TGPU_T_STRUCT && c.ki) ? sc.t[c.ki - 1].struct_index : -1;
}
inline uint32_t keyNode(const CType& c) { return c.elem == TGPU_T_STRUCT ? 0 : c.ki; }
inline bool isBoxed(const tgpu_field_desc& f) {
  return f.qualifier == TGPU_BOXED || f.qualifier == TGPU_OPTIONAL_BOXED;
}
inline tgpu_span loadSpan(const uint8_t* p) {
  tgpu_span s;
  std::memcpy(&s, p, sizeof(s));
  return s;
}
inline void storeSpan(uint8_t* p, uint64_t off, uint64_t len) {
  const tgpu_span s{len ? off : 0, (uint32_t)len, 0};
  std::memcpy(p, &s, sizeof(s));
}

// ---- device form -> host objects (decode) ------------------------------------
struct Sources {
  const uint8_t* strings; /* decode: the input bytes */
  const uint8_t* arena;   /* list arena */
};

void readStruct(const SchemaTables&, uint32_t si, const uint8_t* dev, const Sources&,
                const HostStruct&, uint8_t* host);
void readContainer(const SchemaTables&, const CType&, const uint8_t* dev, const Sources&,
                   const HostType&, void* host);

/* A value of wire type t (struct si / container node ti) at dev. */
inline void readValue(const SchemaTables& sc, uint32_t t, int32_t si, uint32_t ti,
                      const uint8_t* dev, const Sources& src, const HostType& ht, void* host) {
  if (t == TGPU_T_STRING) {
    const tgpu_span s = loadSpan(dev);
    static_cast<std::string*>(host)->assign((const char*)src.strings + s.offset, s.length);
  } else if (t == TGPU_T_STRUCT) {
    readStruct(sc, (uint32_t)si, dev, src, *ht.st, (uint8_t*)host);
  } else if (isContainer(t)) {
    readContainer(sc, ctypeNode(sc, ti), dev, src, ht, host);
  } else {
    std::memcpy(host, dev, scalarBytes(t));
  }
}

struct ElemCtx {
  const SchemaTables* sc;
  const CType* c;
  const Sources* src;
  const HostType* ht;
  const uint8_t* e;  /* device element / pair */
  uint32_t ks;       /* key bytes (map) */
};

inline void readContainer(const SchemaTables& sc, const CType& c, const uint8_t* dev,
                          const Sources& src, const HostType& ht, void* host) {
  const tgpu_span s = loadSpan(dev);
  ht.clear(host);
  const bool is_map = c.ttype == TGPU_T_MAP;
  const uint32_t v = is_map ? c.val : c.elem;
  const uint32_t ks = is_map ? slotBytes(sc, c.elem, keyStruct(sc, c)) : 0;
  const uint32_t es = ks + slotBytes(sc, v, c.si);
  for (uint32_t i = 0; i < s.length; ++i) {
    ElemCtx ctx{&sc, &c, &src, &ht, src.arena + s.offset + (uint64_t)i * es, ks};
    ht.add(host, &ctx, [](void* p, void* ek, void* hv) {
      const ElemCtx& x = *static_cast<const ElemCtx*>(p);
      const bool m = x.c->ttype == TGPU_T_MAP;
      if (m) {
        readValue(*x.sc, x.c->elem, keyStruct(*x.sc, *x.c), keyNode(*x.c), x.e, *x.src,
                  *x.ht->elem, ek);
        readValue(*x.sc, x.c->val, x.c->si, x.c->ti, x.e + x.ks, *x.src, *x.ht->val, hv);
      } else {
        readValue(*x.sc, x.c->elem, x.c->si, x.c->ti, x.e, *x.src, *x.ht->elem, ek);
      }
    });
  }
}

inline void readStruct(const SchemaTables& sc, uint32_t si, const uint8_t* dev,
                       const Sources& src, const HostStruct& hs, uint8_t* host) {
  const tgpu_struct_desc& sd = sc.s[si];
  for (uint32_t k = 0; k < sd.num_fields && k < hs.fields.size(); ++k) {
    const tgpu_field_desc& f = sc.f[sd.first_field + k];
    const HostField& hf = hs.fields[k];
    if (!hf.type) continue;
    const uint8_t set = dev[f.isset_offset];
    if (hf.isset >= 0) host[hf.isset] = set;
    if (!set) continue;  // absent on the wire: the member keeps its value
    const uint8_t* m = dev + f.member_offset;
    void* h = host + hf.offset;
    if (isBoxed(f)) {  // the object the device member points to, in the arena
      const tgpu_span b = loadSpan(m);
      if (b.length)
        readStruct(sc, (uint32_t)f.struct_index, src.arena + b.offset, src, *hf.type->st,
                   (uint8_t*)hf.type->make(h));
    } else if (isContainer(f.ttype)) {
      readContainer(sc, ctypeOf(f), m, src, *hf.type, h);
    } else {
      readValue(sc, f.ttype, f.struct_index, 0, m, src, *hf.type, h);
    }
  }
}

// ---- host objects -> device form (encode input) ------------------------------
/* The encode-side buffers: records, then the string base and list base the
   records' spans are relative to (list arrays 8-byte aligned). */
struct DeviceForm {
  std::vector<uint8_t> records, strings, lists;
  uint64_t alloc(uint64_t bytes) {
    const uint64_t o = (lists.size() + 7) & ~7ull;
    lists.resize(o + bytes);
    return o;
  }
};

void writeStruct(const SchemaTables&, uint32_t si, const uint8_t* host, const HostStruct&,
                 DeviceForm&, uint64_t dev_off, std::vector<uint8_t>* buf);

/* Writes the value at host into buf[off..] (buf: records or lists; resized
   by nested allocations, so addressed by offset). */
inline void writeValue(const SchemaTables& sc, uint32_t t, int32_t si, uint32_t ti,
                       const void* host, const HostType& ht, DeviceForm& out,
                       std::vector<uint8_t>* buf, uint64_t off);

struct WriteCtx {
  const SchemaTables* sc;
  const CType* c;
  const HostType* ht;
  DeviceForm* out;
  uint64_t arr;  /* element array offset in out->lists */
  uint32_t es, ks;
  uint64_t i;
};

inline void writeContainer(const SchemaTables& sc, const CType& c, const void* host,
                           const HostType& ht, DeviceForm& out, std::vector<uint8_t>* buf,
                           uint64_t off) {
  uint64_t n = 0;
  ht.each(host, &n, [](void* p, const void*, const void*) { ++*static_cast<uint64_t*>(p); });
  const bool is_map = c.ttype == TGPU_T_MAP;
  const uint32_t v = is_map ? c.val : c.elem;
  const uint32_t ks = is_map ? slotBytes(sc, c.elem, keyStruct(sc, c)) : 0;
  const uint32_t es = ks + slotBytes(sc, v, c.si);
  const uint64_t arr = n ? out.alloc(n * es) : 0;
  storeSpan(buf->data() + off, arr, n);
  WriteCtx ctx{&sc, &c, &ht, &out, arr, es, ks, 0};
  ht.each(host, &ctx, [](void* p, const void* ek, const void* hv) {
    WriteCtx& x = *static_cast<WriteCtx*>(p);
    const uint64_t at = x.arr + x.i++ * x.es;
    if (x.c->ttype == TGPU_T_MAP) {
      writeValue(*x.sc, x.c->elem, keyStruct(*x.sc, *x.c), keyNode(*x.c), ek, *x.ht->elem,
                 *x.out, &x.out->lists, at);
      writeValue(*x.sc, x.c->val, x.c->si, x.c->ti, hv, *x.ht->val, *x.out, &x.out->lists,
                 at + x.ks);
    } else {
      writeValue(*x.sc, x.c->elem, x.c->si, x.c->ti, ek, *x.ht->elem, *x.out, &x.out->lists,
                 at);
    }
  });
}

inline void writeValue(const SchemaTables& sc, uint32_t t, int32_t si, uint32_t ti,
                       const void* host, const HostType& ht, DeviceForm& out,
                       std::vector<uint8_t>* buf, uint64_t off) {
  if (t == TGPU_T_STRING) {
    const std::string& s = *static_cast<const std::string*>(host);
    storeSpan(buf->data() + off, out.strings.size(), s.size());
    out.strings.insert(out.strings.end(), s.begin(), s.end());
  } else if (t == TGPU_T_STRUCT) {
    writeStruct(sc, (uint32_t)si, (const uint8_t*)host, *ht.st, out, off, buf);
  } else if (isContainer(t)) {
    writeContainer(sc, ctypeNode(sc, ti), host, ht, out, buf, off);
  } else {
    std::memcpy(buf->data() + off, host, scalarBytes(t));
  }
}

inline void writeStruct(const SchemaTables& sc, uint32_t si, const uint8_t* host,
                        const HostStruct& hs, DeviceForm& out, uint64_t dev_off,
                        std::vector<uint8_t>* buf) {
  const tgpu_struct_desc& sd = sc.s[si];
  for (uint32_t k = 0; k < sd.num_fields && k < hs.fields.size(); ++k) {
    const tgpu_field_desc& f = sc.f[sd.first_field + k];
    const HostField& hf = hs.fields[k];
    if (!hf.type) continue;
    const uint8_t set = hf.isset >= 0 ? host[hf.isset] : 1;
    (*buf)[dev_off + f.isset_offset] = set;
    const void* h = host + hf.offset;
    if (isBoxed(f)) {  // the pointee into the list base; null stays {0, 0}
      const void* obj = hf.type->get(h);
      if (obj) {
        const uint64_t o = out.alloc(sc.s[f.struct_index].size);
        storeSpan(buf->data() + dev_off + f.member_offset, o, 1);
        writeStruct(sc, (uint32_t)f.struct_index, (const uint8_t*)obj, *hf.type->st, out, o,
                    &out.lists);
      }
    } else if (isContainer(f.ttype))
      writeContainer(sc, ctypeOf(f), h, *hf.type, out, buf, dev_off + f.member_offset);
    else
      writeValue(sc, f.ttype, f.struct_index, 0, h, *hf.type, out, buf,
                 dev_off + f.member_offset);
  }
}

// ---- spans of one thread's part moved to the merged buffers -------------------
/* Adds sd to every string span and ld to every list / boxed span of a value
   (the thread's records, and its part of the merged list buffer `lists`
   whose contents it reaches through spans already moved by ld). */
void rebaseStruct(const SchemaTables& sc, uint32_t si, uint8_t* obj, uint8_t* lists,
                  uint64_t sd, uint64_t ld);
void rebaseContainer(const SchemaTables& sc, const CType& c, uint8_t* p, uint8_t* lists,
                     uint64_t sd, uint64_t ld);
inline void rebaseSpan(uint8_t* p, uint64_t d) {
  tgpu_span s = loadSpan(p);
  if (s.length) {
    s.offset += d;
    std::memcpy(p, &s, sizeof(s));
  }
}
inline void rebaseValue(const SchemaTables& sc, uint32_t t, int32_t si, uint32_t ti, uint8_t* p,
                        uint8_t* lists, uint64_t sd, uint64_t ld) {
  if (t == TGPU_T_STRING) rebaseSpan(p, sd);
  else if (t == TGPU_T_STRUCT) rebaseStruct(sc, (uint32_t)si, p, lists, sd, ld);
  else if (isContainer(t)) rebaseContainer(sc, ctypeNode(sc, ti), p, lists, sd, ld);
}
inline bool hasSpans(uint32_t t) {
  return t == TGPU_T_STRING || t == TGPU_T_STRUCT || isContainer(t);
}
inline void rebaseContainer(const SchemaTables& sc, const CType& c, uint8_t* p, uint8_t* lists,
                            uint64_t sd, uint64_t ld) {
  rebaseSpan(p, ld);
  const tgpu_span s = loadSpan(p);
  const bool is_map = c.ttype == TGPU_T_MAP;
  const uint32_t v = is_map ? c.val : c.elem;
  if (!hasSpans(v) && !(is_map && hasSpans(c.elem))) return;
  const int32_t ksi = is_map ? keyStruct(sc, c) : -1;
  const uint32_t ks = is_map ? slotBytes(sc, c.elem, ksi) : 0;
  const uint32_t es = ks + slotBytes(sc, v, c.si);
  for (uint32_t i = 0; i < s.length; ++i) {
    uint8_t* e = lists + s.offset + (uint64_t)i * es;
    if (is_map) rebaseValue(sc, c.elem, ksi, keyNode(c), e, lists, sd, ld);
    rebaseValue(sc, v, c.si, c.ti, e + ks, lists, sd, ld);
  }
}
inline void rebaseStruct(const SchemaTables& sc, uint32_t si, uint8_t* obj, uint8_t* lists,
                         uint64_t sd, uint64_t ld) {
  const tgpu_struct_desc& d = sc.s[si];
  for (uint32_t k = 0; k < d.num_fields; ++k) {
    const tgpu_field_desc& f = sc.f[d.first_field + k];
    uint8_t* m = obj + f.member_offset;
    if (isBoxed(f)) {
      rebaseSpan(m, ld);
      const tgpu_span b = loadSpan(m);
      if (b.length) rebaseStruct(sc, (uint32_t)f.struct_index, lists + b.offset, lists, sd, ld);
    } else if (isContainer(f.ttype)) {
      rebaseContainer(sc, ctypeOf(f), m, lists, sd, ld);
    } else {
      rebaseValue(sc, f.ttype, f.struct_index, 0, m, lists, sd, ld);
    }
  }
}

}  // namespace detail

/* Host threads the batch materialization uses: TGPU_HOST_THREADS, else the
   hardware's, at most 16 (the GPU boxes' CPU share per GPU). */
inline unsigned materialize_threads() {
  static const unsigned t = [] {
    const char* e = std::getenv("TGPU_HOST_THREADS");
    const unsigned v = e ? (unsigned)std::atoi(e) : std::thread::hardware_concurrency();
    return std::max(1u, std::min(v ? v : 1u, 16u));
  }();
  return t;
}

namespace detail {
/* fn(t, begin, end) over contiguous parts of [0, n) on up to T threads. */
template <class F>
void parallel_parts(uint64_t n, unsigned T, F&& fn) {
  if (T <= 1 || n < 4096) {
    fn(0u, (uint64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  const uint64_t per = (n + T - 1) / T;
  for (unsigned t = 0; t < T; ++t) {
    const uint64_t b = std::min<uint64_t>(n, t * per), e = std::min<uint64_t>(n, b + per);
    if (b < e) th.emplace_back([&fn, t, b, e] { fn(t, b, e); });
  }
  for (auto& x : th) x.join();
}
}  // namespace detail

/* Decoded device-form records (host copies) -> host objects T (stride
   sizeof(T), default-constructed by the caller); records are independent,
   so contiguous parts go to materialize_threads() threads. */
inline void materialize(const SchemaTables& sc, const uint8_t* records, uint64_t n,
                        uint32_t record_size, const uint8_t* strings, const uint8_t* arena,
                        const HostStruct& hs, void* objects, size_t stride) {
  const detail::Sources src{strings, arena};
  detail::parallel_parts(n, materialize_threads(), [&](unsigned, uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i)
      detail::readStruct(sc, 0, records + i * record_size, src, hs,
                         (uint8_t*)objects + i * stride);
  });
}

/* Host objects T -> the encode input (records + string base + list base).
   Each thread writes its part's records in place and its strings / lists
   into buffers of its own; the parts' buffers are then concatenated and
   their spans moved by the part's base. */
inline detail::DeviceForm dematerialize(const SchemaTables& sc, uint32_t record_size,
                                        const void* objects, uint64_t n, size_t stride,
                                        const HostStruct& hs) {
  detail::DeviceForm out;
  out.records.assign(n * record_size, 0);
  const unsigned T = (n < 4096) ? 1u : materialize_threads();
  std::vector<detail::DeviceForm> part(T);
  std::vector<std::pair<uint64_t, uint64_t>> range(T, {0, 0});
  detail::parallel_parts(n, T, [&](unsigned t, uint64_t b, uint64_t e) {
    range[t] = {b, e};
    detail::DeviceForm& f = T == 1 ? out : part[t];
    for (uint64_t i = b; i < e; ++i)
      detail::writeStruct(sc, 0, (const uint8_t*)objects + i * stride, hs, f, i * record_size,
                          &out.records);
  });
  if (T == 1) return out;
  std::vector<uint64_t> sbase(T), lbase(T);
  uint64_t S = 0, L = 0;
  for (unsigned t = 0; t < T; ++t) {
    sbase[t] = S;
    lbase[t] = L;
    S += part[t].strings.size();
    L = (L + part[t].lists.size() + 7) & ~7ull;
  }
  out.strings.resize(S);
  out.lists.resize(L);
  // each part's thread copies its buffers into place and moves its spans
  // (the part boundaries are the same as in the write above)
  detail::parallel_parts(n, T, [&](unsigned t, uint64_t b, uint64_t e) {
    if (!part[t].strings.empty())
      std::memcpy(out.strings.data() + sbase[t], part[t].strings.data(), part[t].strings.size());
    if (!part[t].lists.empty())
      std::memcpy(out.lists.data() + lbase[t], part[t].lists.data(), part[t].lists.size());
    for (uint64_t i = b; i < e; ++i)
      detail::rebaseStruct(sc, 0, out.records.data() + i * record_size, out.lists.data(),
                           sbase[t], lbase[t]);
  });
  return out;
}

}  // namespace apache::thrift::gpu

#endif  // THRIFT_GPU_HOST_BINDING_H_
