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
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <type_traits>
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
  /* Container: element count (encode sizes the element array with it). */
  uint64_t (*count)(const void* c) = nullptr;
  /* Contiguous containers of arithmetic elements (std::vector<int32_t>, ...):
     the whole element array at once — `assign` replaces the contents with n
     elements (decode: the reader's resize + readArithmeticVector,
     protocol_methods.h:413-441, BinaryProtocol.cpp:49-72), `data` returns
     them (encode: writeArithmeticVector, BinaryProtocol.cpp:95-117). The
     device element slots of a scalar list are the elements themselves. */
  void (*assign)(void* c, const void* data, uint64_t n) = nullptr;
  const void* (*data)(const void* c) = nullptr;
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
  using E = typename V::value_type;
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
  t.count = [](const void* c) -> uint64_t { return static_cast<const V*>(c)->size(); };
  if constexpr (std::is_arithmetic_v<E> && !std::is_same_v<E, bool> &&
                std::is_same_v<V, std::vector<E>>) {
    if (elem && elem->kind == HostType::Scalar && elem->size == sizeof(E)) {
      t.assign = [](void* c, const void* d, uint64_t n) {
        static_cast<V*>(c)->assign(static_cast<const E*>(d), static_cast<const E*>(d) + n);
      };
      t.data = [](const void* c) -> const void* { return static_cast<const V*>(c)->data(); };
    }
  }
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
  t.count = [](const void* c) -> uint64_t { return static_cast<const C*>(c)->size(); };
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
  t.count = [](const void* c) -> uint64_t { return static_cast<const C*>(c)->size(); };
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
    const uint32_t w = scalarBytes(t);
    // never more bytes than the bound C++ scalar holds (a list<i64> bound to
    // std::vector<int32_t> keeps the low 4 bytes; a binding of unknown size
    // takes the schema width)
    const uint32_t hw = ht.kind == HostType::Scalar && ht.size ? ht.size : w;
    std::memcpy(host, dev, w < hw ? w : hw);
    // an integer bound to a wider C++ integer: sign-extended (a list<i16>
    // bound to std::vector<int32_t> reads -3 as -3, not 65533)
    if (hw > w && w < 8 &&
        (t == TGPU_T_BYTE || t == TGPU_T_I16 || t == TGPU_T_I32) && (dev[w - 1] & 0x80))
      std::memset(static_cast<uint8_t*>(host) + w, 0xff, hw - w);
  }
}

/* Whether a list's element array can move in one copy: scalar elements
   whose schema width is the bound C++ element's (a list<i16> bound to
   std::vector<int32_t> takes the per-element path, as before the fast path). */
inline bool fastElems(const CType& c, const HostType& ht) {
  return !isContainer(c.elem) && c.elem != TGPU_T_STRING && c.elem != TGPU_T_STRUCT && ht.elem &&
         scalarBytes(c.elem) == ht.elem->size;
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
  if (ht.assign && c.ttype == TGPU_T_LIST && fastElems(c, ht)) {  // the element array, whole
    ht.assign(host, src.arena + s.offset, s.length);
    return;
  }
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
/* Where one part of a chunk's device form goes: string bytes at
   strings + spos.., list arrays (8-byte aligned) at lists + lpos... Positions
   are relative to the chunk's string / list base, and a part starts at its
   own base, so every span it stores is final. Count mode (the sizing pass
   that places the parts) only advances the positions. */
struct Sink {
  uint8_t* strings = nullptr;
  uint8_t* lists = nullptr;
  uint64_t spos = 0, lpos = 0;
  uint64_t alloc(uint64_t bytes) {
    const uint64_t o = (lpos + 7) & ~7ull;
    lpos = o + bytes;
    return o;
  }
};

template <bool Count>
void writeStruct(const SchemaTables&, uint32_t si, const uint8_t* host, const HostStruct&, Sink&,
                 uint8_t* dev);
template <bool Count>
void writeValue(const SchemaTables& sc, uint32_t t, int32_t si, uint32_t ti, const void* host,
                const HostType& ht, Sink& out, uint8_t* dev);

template <bool Count>
struct WriteCtx {
  const SchemaTables* sc;
  const CType* c;
  const HostType* ht;
  Sink* out;
  uint64_t arr; /* element array position in the list base */
  uint32_t es, ks;
  uint64_t i;
};

inline bool hasSpans(uint32_t t) {
  return t == TGPU_T_STRING || t == TGPU_T_STRUCT || isContainer(t);
}

/* A container's span at dev and its element array in the list base. */
template <bool Count>
void writeContainer(const SchemaTables& sc, const CType& c, const void* host, const HostType& ht,
                    Sink& out, uint8_t* dev) {
  uint64_t n = 0;
  if (ht.count) n = ht.count(host);
  else ht.each(host, &n, [](void* p, const void*, const void*) { ++*static_cast<uint64_t*>(p); });
  const bool is_map = c.ttype == TGPU_T_MAP;
  const uint32_t v = is_map ? c.val : c.elem;
  const uint32_t ks = is_map ? slotBytes(sc, c.elem, keyStruct(sc, c)) : 0;
  const uint32_t es = ks + slotBytes(sc, v, c.si);
  const uint64_t arr = n ? out.alloc(n * es) : 0;
  if (!Count) storeSpan(dev, arr, n);
  if (!n) return;
  if (ht.data && c.ttype == TGPU_T_LIST && fastElems(c, ht)) {  // arithmetic elements: one copy
    if (!Count) std::memcpy(out.lists + arr, ht.data(host), n * es);
    return;
  }
  // scalar elements place nothing else (count mode is done)
  if (Count && !hasSpans(v) && !(is_map && hasSpans(c.elem))) return;
  // struct slots: fields the binding skips read as zero (unset)
  if (!Count && (v == TGPU_T_STRUCT || (is_map && c.elem == TGPU_T_STRUCT)))
    std::memset(out.lists + arr, 0, n * es);
  WriteCtx<Count> ctx{&sc, &c, &ht, &out, arr, es, ks, 0};
  ht.each(host, &ctx, [](void* p, const void* ek, const void* hv) {
    WriteCtx<Count>& x = *static_cast<WriteCtx<Count>*>(p);
    const uint64_t at = x.arr + x.i++ * x.es;
    uint8_t* e = Count ? nullptr : x.out->lists + at;
    if (x.c->ttype == TGPU_T_MAP) {
      writeValue<Count>(*x.sc, x.c->elem, keyStruct(*x.sc, *x.c), keyNode(*x.c), ek, *x.ht->elem,
                        *x.out, e);
      writeValue<Count>(*x.sc, x.c->val, x.c->si, x.c->ti, hv, *x.ht->val, *x.out,
                        Count ? nullptr : e + x.ks);
    } else {
      writeValue<Count>(*x.sc, x.c->elem, x.c->si, x.c->ti, ek, *x.ht->elem, *x.out, e);
    }
  });
}

/* The value at host into its device slot dev (nullptr in count mode). */
template <bool Count>
void writeValue(const SchemaTables& sc, uint32_t t, int32_t si, uint32_t ti, const void* host,
                const HostType& ht, Sink& out, uint8_t* dev) {
  if (t == TGPU_T_STRING) {
    const std::string& s = *static_cast<const std::string*>(host);
    if (!Count) {
      storeSpan(dev, out.spos, s.size());
      std::memcpy(out.strings + out.spos, s.data(), s.size());
    }
    out.spos += s.size();
  } else if (t == TGPU_T_STRUCT) {
    writeStruct<Count>(sc, (uint32_t)si, (const uint8_t*)host, *ht.st, out, dev);
  } else if (isContainer(t)) {
    writeContainer<Count>(sc, ctypeNode(sc, ti), host, ht, out, dev);
  } else if (!Count) {
    // a C++ scalar narrower than the schema type fills the slot's low bytes
    // and is sign-extended (std::vector<int32_t> bound to list<i64>); never
    // read past the host object
    const uint32_t w = scalarBytes(t);
    const uint32_t hw = ht.kind == HostType::Scalar && ht.size ? ht.size : w;
    if (hw >= w) {
      std::memcpy(dev, host, w);
    } else {
      std::memcpy(dev, host, hw);
      const bool neg = t != TGPU_T_BOOL && t != TGPU_T_DOUBLE && t != TGPU_T_FLOAT &&
                       (static_cast<const uint8_t*>(host)[hw - 1] & 0x80);
      std::memset(dev + hw, neg ? 0xff : 0, w - hw);
    }
  }
}

/* A struct's members and isset bytes into its zero-filled slot dev. */
template <bool Count>
void writeStruct(const SchemaTables& sc, uint32_t si, const uint8_t* host, const HostStruct& hs,
                 Sink& out, uint8_t* dev) {
  const tgpu_struct_desc& sd = sc.s[si];
  for (uint32_t k = 0; k < sd.num_fields && k < hs.fields.size(); ++k) {
    const tgpu_field_desc& f = sc.f[sd.first_field + k];
    const HostField& hf = hs.fields[k];
    if (!hf.type) continue;
    const uint8_t set = hf.isset >= 0 ? host[hf.isset] : 1;
    if (!Count) dev[f.isset_offset] = set;
    const void* h = host + hf.offset;
    uint8_t* m = Count ? nullptr : dev + f.member_offset;
    if (isBoxed(f)) {  // the pointee into the list base; null stays {0, 0}
      const void* obj = hf.type->get(h);
      if (obj) {
        const uint32_t bs = sc.s[f.struct_index].size;
        const uint64_t o = out.alloc(bs);
        uint8_t* slot = nullptr;
        if (!Count) {
          storeSpan(m, o, 1);
          slot = out.lists + o;
          std::memset(slot, 0, bs);
        }
        writeStruct<Count>(sc, (uint32_t)f.struct_index, (const uint8_t*)obj, *hf.type->st, out,
                           slot);
      }
    } else if (isContainer(f.ttype)) {
      writeContainer<Count>(sc, ctypeOf(f), h, *hf.type, out, m);
    } else {
      writeValue<Count>(sc, f.ttype, f.struct_index, 0, h, *hf.type, out, m);
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

/* A process-wide pool of materialize_threads() workers for the batch
   materialization. Tasks belong to a Group; Group::wait() runs queued tasks
   on the waiting thread as well until the group's last one is done, then
   rethrows the first exception one of them threw (the reference's reader
   throws into the caller, so a binding hook's exception must too). */
class HostPool {
 public:
  class Group {
   public:
    Group() = default;
    Group(const Group&) = delete;
    ~Group() { instance().wait(*this, false); }
    void run(std::function<void()> fn) { instance().submit(this, std::move(fn)); }
    void wait() { instance().wait(*this, true); }

   private:
    friend class HostPool;
    uint64_t pending = 0;  // guarded by the pool's mutex
    std::exception_ptr err;
  };
  static HostPool& instance() {
    static HostPool p(materialize_threads());
    return p;
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  struct Task {
    Group* g;
    std::function<void()> fn;
  };
  explicit HostPool(unsigned n) {
    for (unsigned i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  void submit(Group* g, std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      ++g->pending;
      q_.push_back(Task{g, std::move(fn)});
    }
    cv_.notify_one();
  }
  void execute(Task& t) {
    std::exception_ptr e;
    try {
      t.fn();
    } catch (...) {
      e = std::current_exception();
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (e && !t.g->err) t.g->err = e;
    if (--t.g->pending == 0) done_.notify_all();
  }
  void loop() {
    for (;;) {
      Task t;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        t = std::move(q_.front());
        q_.pop_front();
      }
      execute(t);
    }
  }
  void wait(Group& g, bool rethrow) {
    std::unique_lock<std::mutex> lk(mu_);
    while (g.pending) {
      if (!q_.empty()) {  // help: run a queued task here
        Task t = std::move(q_.front());
        q_.pop_front();
        lk.unlock();
        execute(t);
        lk.lock();
        continue;
      }
      done_.wait(lk);
    }
    if (rethrow && g.err) {
      std::exception_ptr e = g.err;
      g.err = nullptr;
      std::rethrow_exception(e);
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::deque<Task> q_;
  std::vector<std::thread> workers_;
  bool stop_ = false;
};

/* Records per materialization task: small enough that every worker has
   work as soon as a chunk lands, large enough to keep the queue cheap. */
constexpr uint64_t kMaterializeBlock = 8192;

/* Decoded device-form records (host copies) -> host objects T (stride
   sizeof(T), default-constructed by the caller), records [b, e) of the
   batch, on the calling thread. */
inline void materializeRange(const SchemaTables& sc, const uint8_t* records, uint64_t b,
                             uint64_t e, uint32_t record_size, const uint8_t* strings,
                             const uint8_t* arena, const HostStruct& hs, void* objects,
                             size_t stride) {
  const detail::Sources src{strings, arena};
  for (uint64_t i = b; i < e; ++i)
    detail::readStruct(sc, 0, records + i * record_size, src, hs, (uint8_t*)objects + i * stride);
}

/* The same for records [b, e), queued on the pool in blocks of
   kMaterializeBlock records (records are independent). */
inline void materializeAsync(HostPool::Group& g, const SchemaTables& sc, const uint8_t* records,
                             uint64_t b, uint64_t e, uint32_t record_size, const uint8_t* strings,
                             const uint8_t* arena, const HostStruct& hs, void* objects,
                             size_t stride) {
  for (uint64_t x = b; x < e; x += kMaterializeBlock) {
    const uint64_t y = std::min(e, x + kMaterializeBlock);
    g.run([=, &sc, &hs] {
      materializeRange(sc, records, x, y, record_size, strings, arena, hs, objects, stride);
    });
  }
}

/* All n records, in parallel; returns when they are materialized. */
inline void materialize(const SchemaTables& sc, const uint8_t* records, uint64_t n,
                        uint32_t record_size, const uint8_t* strings, const uint8_t* arena,
                        const HostStruct& hs, void* objects, size_t stride) {
  HostPool::Group g;
  materializeAsync(g, sc, records, 0, n, record_size, strings, arena, hs, objects, stride);
  g.wait();
}

/* String and list bytes of host objects [b, e) in the device form (the
   sizing pass: strings packed, list arrays 8-byte aligned, from a base of
   0 — the same bytes from any 8-aligned base). */
inline std::pair<uint64_t, uint64_t> formBytes(const SchemaTables& sc, const void* objects,
                                               uint64_t b, uint64_t e, size_t stride,
                                               const HostStruct& hs) {
  detail::Sink k;
  for (uint64_t i = b; i < e; ++i)
    detail::writeStruct<true>(sc, 0, (const uint8_t*)objects + i * stride, hs, k, nullptr);
  return {k.spos, k.lpos};
}

/* Host objects [b, e) -> their device form: records at records[(i - b) * S]
   (zero-filled here first), strings and list arrays through `sink`, whose
   positions start at the part's base in the chunk's string / list base (from
   formBytes; lpos 8-aligned). */
inline void formWrite(const SchemaTables& sc, uint32_t record_size, const void* objects,
                      uint64_t b, uint64_t e, size_t stride, const HostStruct& hs,
                      uint8_t* records, detail::Sink sink) {
  std::memset(records, 0, (e - b) * record_size);
  for (uint64_t i = b; i < e; ++i)
    detail::writeStruct<false>(sc, 0, (const uint8_t*)objects + i * stride, hs, sink,
                               records + (i - b) * record_size);
}

/* The encode input of n host objects as owned buffers (records + string base
   + list base), built in parallel parts (each part sized, then written at its
   base). */
struct DeviceForm {
  std::vector<uint8_t> records, strings, lists;
};
inline DeviceForm dematerialize(const SchemaTables& sc, uint32_t record_size,
                                const void* objects, uint64_t n, size_t stride,
                                const HostStruct& hs) {
  const uint64_t P = std::max<uint64_t>(1, std::min<uint64_t>(materialize_threads() * 4,
                                                              n / 1024));
  std::vector<std::pair<uint64_t, uint64_t>> sz(P);
  auto part = [&](uint64_t t) { return std::make_pair(n * t / P, n * (t + 1) / P); };
  {
    HostPool::Group g;
    for (uint64_t t = 0; t < P; ++t)
      g.run([&, t] { sz[t] = formBytes(sc, objects, part(t).first, part(t).second, stride, hs); });
    g.wait();
  }
  std::vector<detail::Sink> at(P);
  uint64_t S = 0, L = 0;
  for (uint64_t t = 0; t < P; ++t) {
    at[t].spos = S;
    at[t].lpos = L;
    S += sz[t].first;
    L = (L + sz[t].second + 7) & ~7ull;
  }
  DeviceForm out;
  out.records.resize(n * record_size);
  out.strings.resize(S);
  out.lists.resize(L);
  HostPool::Group g;
  for (uint64_t t = 0; t < P; ++t)
    g.run([&, t] {
      detail::Sink k = at[t];
      k.strings = out.strings.data();
      k.lists = out.lists.data();
      formWrite(sc, record_size, objects, part(t).first, part(t).second, stride, hs,
                out.records.data() + part(t).first * record_size, k);
    });
  g.wait();
  return out;
}

}  // namespace apache::thrift::gpu

#endif  // THRIFT_GPU_HOST_BINDING_H_
