// tgpu_api.cpp — host side of the C-ABI (include/thrift_gpu.h): schema
// validation/upload, the canonical Binary template, context workspaces and
// the stream-ordered launch sequences of encode/decode.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "tgpu_internal.h"

using namespace tgpu;

struct tgpu_schema {
  std::vector<tgpu_struct_desc> structs;
  std::vector<tgpu_field_desc> fields;
  std::vector<tgpu_type_desc> types;  // nested container types
  tgpu_struct_desc* d_structs = nullptr;
  tgpu_field_desc* d_fields = nullptr;
  tgpu_type_desc* d_types = nullptr;
  // containers of structs / containers: per-record arena regions
  bool nested = false;
  uint32_t region_scale[2] = {0, 0};  // Binary, Compact (and CompactV1)
  uint32_t nest_slot = 0;             // measuring reads: element slot bytes
  int device = 0;
  bool has_lists = false;
  bool has_strings = false;
  bool fixed_binary = false;
  FixedTemplate tmpl{};
  FixedTemplate* d_tmpl = nullptr;
  bool has_plan = false;  // word-gather form of tmpl (S % 8 == 0)
  FixedPlan plan{};
  FixedPlan* d_plan = nullptr;
  bool has_prog[3] = {false, false, false};  // compiled programs by protocol id
  bool has_double = false;  // any double member/element (CompactV1 differs there)
  bool str_elems = false;   // strings inside lists/sets/maps (arena scale 4 / 16)
  VProgram prog[3]{};
  VProgram* d_prog[3] = {nullptr, nullptr, nullptr};
  // the same programs taking appended unknown fields at the root STOP
  // (kStopSkipsUnknown): a separate variant, so the canonical kernels keep
  // their register footprint; used where a stream is known to carry them
  VProgram prog_tol[3]{};
  VProgram* d_prog_tol[3] = {nullptr, nullptr, nullptr};
  // nested schemas (lists / sets of structs or of scalar lists): the
  // canonical form with VOP_SEQ loops, compiled only (JIT_NESTED); nprog_depth
  // = the deepest container nesting (the height it needs)
  bool has_nprog[3] = {false, false, false};
  VProgram nprog[3]{};
  VProgram* d_nprog[3] = {nullptr, nullptr, nullptr};  // (the index's AOT repair kernels read it)
  uint32_t nprog_depth[3] = {0, 0, 0};
  // a recursive schema's unrolled program (VOP_DEFER): decode / index only
  bool nprog_defer[3] = {false, false, false};
  // a struct reachable from itself (the deep passes' wide tier)
  bool recursive = false;
  // the wire bytes per record (x16) of the last batch whose size this schema
  // learned (blocking encode / size calls), by protocol id: sizes the
  // compiled write pass's LDS output tile (enc_out_cap)
  std::atomic<uint64_t> mean16[3] = {0, 0, 0};
  // the block rule's slots (n = 0: the position rule; ArenaPack, k_arena.hip)
  ArenaPack pack{};
};

namespace {
// The block rule's slots of struct si's members (by-value structs flattened):
// lists / sets of scalars; false when the schema holds anything else in a
// container (a map, strings or structs as elements), a boxed member, or more
// than kPackSlots lists (thrift_oracle.cpp block_pack_slots restates it).
bool block_pack_slots(const tgpu_schema& s, uint32_t si, uint32_t base, ArenaPack& p, int depth) {
  if (depth > 64) return false;
  const tgpu_struct_desc& sd = s.structs[si];
  for (uint32_t k = 0; k < sd.num_fields; ++k) {
    const tgpu_field_desc& f = s.fields[sd.first_field + k];
    if (f.qualifier == TGPU_BOXED || f.qualifier == TGPU_OPTIONAL_BOXED) return false;
    if (f.ttype == TGPU_T_STRUCT) {
      if (!block_pack_slots(s, (uint32_t)f.struct_index, base + f.member_offset, p, depth + 1))
        return false;
    } else if (f.ttype == TGPU_T_MAP) {
      return false;
    } else if (f.ttype == TGPU_T_LIST || f.ttype == TGPU_T_SET) {
      uint32_t es;
      switch (f.elem_ttype) {
        case TGPU_T_BOOL: case TGPU_T_BYTE: es = 1; break;
        case TGPU_T_I16: es = 2; break;
        case TGPU_T_I32: case TGPU_T_FLOAT: es = 4; break;
        case TGPU_T_I64: case TGPU_T_DOUBLE: es = 8; break;
        default: return false;
      }
      if (p.n == kPackSlots) return false;
      p.member[p.n] = base + f.member_offset;
      p.es[p.n] = es;
      ++p.n;
    }
  }
  return true;
}

int proto_slot(int protocol) { return protocol == TGPU_PROTOCOL_BINARY ? 0 : protocol == TGPU_PROTOCOL_COMPACT ? 1 : 2; }

void learn_mean(const tgpu_schema* s, int protocol, uint64_t bytes, uint64_t n) {
  if (n >= 256 && bytes) const_cast<tgpu_schema*>(s)->mean16[proto_slot(protocol)] = bytes * 16 / n;
}

// LDS output tile of the compiled write pass: 256 records of the schema's
// mean size with 25 % slack (records past it go to HBM directly), between
// 4 and 24 KiB (a smaller tile lets more workgroups share a CU: the write
// pass waits on memory most of the time). 0 = the kernel's default (24 KiB)
// until a size is known. TGPU_ENC_OUTCAP=<bytes> overrides (A/B).
// The nested write pass's LDS output tile: 256 records of the learned mean
// size + 15 % + 1 KiB (48 KiB until a size is known), 4..60 KiB.
// TGPU_NESTED_OUTCAP=<bytes> overrides (0: no staging, A/B).
uint32_t nested_out_cap(const tgpu_schema* s, int protocol) {
  if (const char* v = getenv("TGPU_NESTED_OUTCAP")) {
    const uint32_t f = (uint32_t)strtoul(v, nullptr, 10);
    return f ? std::min<uint32_t>(std::max<uint32_t>(f, 4096), 60 * 1024) & ~15u : 0u;
  }
  const uint64_t m16 = s->mean16[proto_slot(protocol)];
  if (!m16) return 48 * 1024;
  const uint64_t want = (m16 * 256 / 16) * 115 / 100 + 1024;
  return (uint32_t)std::min<uint64_t>(std::max<uint64_t>(want, 4096), 60 * 1024) & ~15u;
}

uint32_t enc_out_cap(const tgpu_schema* s, int protocol) {
  static const uint32_t force = [] {
    const char* v = getenv("TGPU_ENC_OUTCAP");
    return v ? (uint32_t)strtoul(v, nullptr, 10) : 0u;
  }();
  if (force) return std::min<uint32_t>(std::max<uint32_t>(force, 4096), 24 * 1024) & ~15u;
  const uint64_t m16 = s->mean16[proto_slot(protocol)];
  if (!m16) return 0;
  const uint64_t want = (m16 * 256 / 16) * 5 / 4 + 64;
  const uint64_t cap = (want + 1023) & ~1023ull;
  return (uint32_t)std::min<uint64_t>(std::max<uint64_t>(cap, 4096), 24 * 1024);
}
}  // namespace

struct tgpu_context {
  int device = 0;
  DevResult* d_res = nullptr;
  DevResult* h_res = nullptr;  // pinned
  uint64_t* h_words = nullptr;  // pinned, 8 words: the stream index's mid-call reads
  uint64_t* d_offs = nullptr;
  unsigned long long* d_block_sums = nullptr;
  unsigned long long* d_scan_part = nullptr;  // partial sums of the tile scan
  uint64_t* d_irr = nullptr;                  // program decode: irregular record list
  uint64_t* d_deep = nullptr;                 // records deferred to the deep pass
  uint64_t reserved = 0;  // records
  // deep-pass skip frames (DeepArgs): slab_lanes x slab_frames, grow-only
  uint8_t* d_slabs = nullptr;
  uint8_t* d_wslabs = nullptr;  // the deep passes' wide tier (wslab_lanes x kWideFrames)
  uint32_t wslab_lanes = 0;
  uint64_t* d_deep2 = nullptr;  // records the wide tier leaves to the max_depth slabs
  uint64_t slab_frames = 0;
  uint32_t slab_lanes = 0;
  // stream indexer workspace (per chunk)
  uint8_t* d_index = nullptr;
  uint64_t index_bytes = 0;
  // the last two-pass index's counters (tgpu_index_stats): its scal words
  unsigned long long* last_scal = nullptr;
  uint64_t last_chunks = 0;
  int last_op = 0;        // 1 decode, 2 encode
  void* host_pipe = nullptr;  // tgpu_host.cpp: streams + chunk buffers of the host path
  // transcode: decoded records and list arena between the two passes
  uint8_t* d_xrec = nullptr;
  uint64_t xrec_bytes = 0;
  uint8_t* d_xarena = nullptr;
  uint64_t xarena_bytes = 0;
  // transcode without materialized records: output starts when the caller
  // asked for none (the listed records' holes, the finish's failing record)
  uint8_t* d_xoffs = nullptr;
  uint64_t xoffs_bytes = 0;
  // the stream index's exhaustive resolution (k_index.hip), on demand
  uint8_t* d_xtab = nullptr;
  uint64_t xtab_bytes = 0;
  // the single-pass transcoder's look-back status words (tiles + 1)
  uint8_t* d_xstat = nullptr;
  uint64_t xstat_bytes = 0;
  // the block rule: per-block marks of the blocks the decode tiles packed
  // (reserved / kArenaBlock + 1 words), and the last call's epoch
  uint32_t* d_pack_flags = nullptr;
  uint32_t pack_epoch = 0;
};

namespace tgpu {
bool schema_has_lists(const tgpu_schema* s) { return s->has_lists; }
bool schema_block_rule(const tgpu_schema* s) { return s->pack.n > 0; }

bool valid_protocol(int p) {
  return p == TGPU_PROTOCOL_BINARY || p == TGPU_PROTOCOL_COMPACT || p == TGPU_PROTOCOL_COMPACT_V1;
}
// The record program that runs `protocol`: CompactV1 differs from Compact
// only in the byte order of doubles (CompactV1Protocol-inl.h:44-53,84), so
// a schema without doubles runs Compact's program; with doubles, its own
// (slot kV1Slot: Compact's ops with the doubles' ops little-endian,
// kFixedLE).
int prog_protocol(const tgpu_schema* s, int protocol) {
  if (protocol == TGPU_PROTOCOL_COMPACT_V1) return s->has_double ? kV1Slot : TGPU_PROTOCOL_COMPACT;
  return protocol;
}
bool has_prog(const tgpu_schema* s, int protocol) {
  const int q = prog_protocol(s, protocol);
  return q >= 0 && s->has_prog[q];
}
void* context_host_pipe(tgpu_context* c) {
  if (!c->host_pipe) c->host_pipe = host_pipe_create();
  return c->host_pipe;
}
uint32_t packable_lists(const tgpu_schema* s, int protocol, uint32_t* member, uint32_t* width,
                        uint32_t max) {
  const int q = prog_protocol(s, protocol);
  if (q < 0 || !s->has_prog[q] || s->nested || s->str_elems || !s->has_lists) return 0;
  const VProgram& P = s->prog[q];
  uint32_t k = 0;
  for (uint32_t i = 0; i < P.n_ops; ++i) {
    if (P.ops[i].kind != VOP_LIST) continue;
    if (k == max) return 0;
    member[k] = P.ops[i].member;
    width[k] = P.ops[i].width;
    ++k;
  }
  return k;
}
}  // namespace tgpu

namespace {

bool is_scalar(uint32_t t) {
  switch (t) {
    case TGPU_T_BOOL: case TGPU_T_BYTE: case TGPU_T_I16: case TGPU_T_I32:
    case TGPU_T_I64: case TGPU_T_DOUBLE: case TGPU_T_FLOAT:
      return true;
    default:
      return false;
  }
}
uint32_t scalar_size(uint32_t t) {
  switch (t) {
    case TGPU_T_BOOL: case TGPU_T_BYTE: return 1;
    case TGPU_T_I16: return 2;
    case TGPU_T_I32: case TGPU_T_FLOAT: return 4;
    default: return 8;
  }
}
uint32_t align_up(uint32_t x, uint32_t a) { return (x + a - 1) / a * a; }

bool is_container_t(uint32_t t) { return t == TGPU_T_LIST || t == TGPU_T_SET || t == TGPU_T_MAP; }
bool is_complex_t(uint32_t t) { return t == TGPU_T_STRUCT || is_container_t(t); }
bool is_boxed(const tgpu_field_desc& f) {
  return f.qualifier == TGPU_BOXED || f.qualifier == TGPU_OPTIONAL_BOXED;
}

// Layout of struct si (memoized in `done`): declaration-order members at
// natural alignment, then one isset byte per field (Isset.h:243-296). A boxed
// struct member is a 16-byte span (the pointer), so recursion through it (or
// through a container) needs no layout recursion; a struct holding itself
// by value has no layout.
int layout_struct(tgpu_struct_desc* s, uint32_t ns, tgpu_field_desc* f, uint32_t nf,
                  uint32_t si, std::vector<int>& state) {
  if (si >= ns) return TGPU_ERR_INVALID_ARGUMENT;
  if (state[si] == 2) return TGPU_OK;
  if (state[si] == 1) return TGPU_ERR_UNSUPPORTED;  // a struct holding itself by value
  state[si] = 1;
  tgpu_struct_desc& sd = s[si];
  if ((uint64_t)sd.first_field + sd.num_fields > nf) return TGPU_ERR_INVALID_ARGUMENT;
  uint32_t off = 0, align = 1;
  for (uint32_t k = 0; k < sd.num_fields; ++k) {
    tgpu_field_desc& fd = f[sd.first_field + k];
    uint32_t sz, al;
    if (is_scalar(fd.ttype)) {
      sz = al = scalar_size(fd.ttype);
    } else if (fd.ttype == TGPU_T_STRING || is_container_t(fd.ttype) ||
               (fd.ttype == TGPU_T_STRUCT && is_boxed(fd))) {
      sz = 16;
      al = 8;
    } else if (fd.ttype == TGPU_T_STRUCT) {
      if (fd.struct_index < 0) return TGPU_ERR_INVALID_ARGUMENT;
      const int rc = layout_struct(s, ns, f, nf, (uint32_t)fd.struct_index, state);
      if (rc) return rc;
      sz = s[fd.struct_index].size;
      al = s[fd.struct_index].align;
    } else {
      return TGPU_ERR_UNSUPPORTED;
    }
    off = align_up(off, al);
    fd.member_offset = off;
    off += sz;
    align = std::max(align, al);
  }
  for (uint32_t k = 0; k < sd.num_fields; ++k) f[sd.first_field + k].isset_offset = off + k;
  off += sd.num_fields;
  sd.align = align;
  sd.size = align_up(std::max(off, 1u), align);
  state[si] = 2;
  return TGPU_OK;
}

// The schema tables a validation walks (fields' type_index / struct_index /
// key_index into these).
struct Tables {
  const tgpu_struct_desc* s;
  uint32_t ns;
  const tgpu_field_desc* f;
  uint32_t nf;
  const tgpu_type_desc* t;
  uint32_t nt;
};

struct SchemaFacts {
  bool has_lists = false;
  bool nested = false;  // a container holds structs or containers, a complex key, a boxed field
};

// Terse struct members nest at most this deep (the device's emptiness walk,
// tgpu_device.h struct_empty, keeps one level per terse struct member).
constexpr int kMaxTerseDepth = 16;

// Validation of a schema whose structs may be recursive (through containers
// and boxed fields): every struct and type node reachable from the root is
// checked once (visited sets), so recursion terminates; two shapes without a
// finite form are rejected — a struct holding itself by value (no layout)
// and a cycle of type nodes alone (list<list<...>> forever).
struct Validator {
  const Tables& T;
  SchemaFacts& facts;
  std::vector<uint8_t> sv, tv;  // visited structs / type nodes
  std::vector<uint32_t> work;   // structs to check

  int node(uint32_t ti, uint32_t want_ttype) {  // ti: 1 + index
    if (ti == 0 || ti > T.nt) return TGPU_ERR_INVALID_ARGUMENT;
    const tgpu_type_desc& n = T.t[ti - 1];
    if (n.ttype != want_ttype) return TGPU_ERR_INVALID_ARGUMENT;
    if (tv[ti - 1]) return TGPU_OK;
    tv[ti - 1] = 1;
    if (n.ttype == TGPU_T_STRUCT) return value(TGPU_T_STRUCT, n.struct_index, 0);
    return container(n.ttype, n.elem_ttype, n.val_ttype, n.struct_index, n.type_index, n.key_index);
  }
  // a container element / map value / map key of type t
  int value(uint32_t t, int32_t si, uint32_t ti) {
    if (t == TGPU_T_STRUCT) {
      if (si < 0 || (uint32_t)si >= T.ns) return TGPU_ERR_INVALID_ARGUMENT;
      if (!sv[si]) {
        sv[si] = 1;
        work.push_back((uint32_t)si);
      }
      return TGPU_OK;
    }
    if (is_container_t(t)) return node(ti, t);
    return (is_scalar(t) || t == TGPU_T_STRING) ? TGPU_OK : TGPU_ERR_UNSUPPORTED;
  }
  int container(uint32_t ttype, uint32_t elem, uint32_t val, int32_t si, uint32_t ti,
                uint32_t ki) {
    facts.has_lists = true;
    const bool is_map = ttype == TGPU_T_MAP;
    if (!is_container_t(ttype)) return TGPU_ERR_INVALID_ARGUMENT;
    const uint32_t v = is_map ? val : elem;
    if (is_complex_t(v)) facts.nested = true;
    int rc = value(v, si, ti);
    if (rc) return rc;
    if (!is_map) return ki ? TGPU_ERR_INVALID_ARGUMENT : TGPU_OK;
    if (!is_complex_t(elem)) {
      if (ki) return TGPU_ERR_INVALID_ARGUMENT;
      return value(elem, -1, 0);
    }
    facts.nested = true;
    return node(ki, elem);  // a struct key: a T_STRUCT node
  }
  int struct_(uint32_t si) {
    const tgpu_struct_desc& sd = T.s[si];
    if ((uint64_t)sd.first_field + sd.num_fields > T.nf || sd.size == 0 || sd.align == 0 ||
        sd.size % sd.align)
      return TGPU_ERR_INVALID_ARGUMENT;
    if (sd.flags & ~(uint32_t)(TGPU_STRUCT_UNION | TGPU_STRUCT_ENFORCE_REQUIRED))
      return TGPU_ERR_UNSUPPORTED;
    for (uint32_t k = 0; k < sd.num_fields; ++k) {
      const tgpu_field_desc& fd = T.f[sd.first_field + k];
      if ((sd.flags & TGPU_STRUCT_UNION) && fd.qualifier != TGPU_UNQUALIFIED)
        return TGPU_ERR_UNSUPPORTED;
      for (uint32_t j = 0; j < k; ++j)
        if (T.f[sd.first_field + j].id == fd.id) return TGPU_ERR_INVALID_ARGUMENT;
      if (fd.qualifier > TGPU_OPTIONAL_BOXED) return TGPU_ERR_UNSUPPORTED;
      if (is_boxed(fd) && fd.ttype != TGPU_T_STRUCT) return TGPU_ERR_UNSUPPORTED;
      if (fd.key_index && fd.ttype != TGPU_T_MAP) return TGPU_ERR_INVALID_ARGUMENT;
      // required fields are checked through a 64-bit per-struct mask
      if (fd.qualifier == TGPU_REQUIRED && k >= 64 && (sd.flags & TGPU_STRUCT_ENFORCE_REQUIRED))
        return TGPU_ERR_UNSUPPORTED;
      if (fd.isset_offset >= sd.size) return TGPU_ERR_INVALID_ARGUMENT;
      uint32_t sz;
      if (is_scalar(fd.ttype)) {
        sz = scalar_size(fd.ttype);
      } else if (fd.ttype == TGPU_T_STRING) {
        sz = 16;
      } else if (is_container_t(fd.ttype)) {
        const int rc = container(fd.ttype, fd.elem_ttype, fd.val_ttype, fd.struct_index,
                                 fd.type_index, fd.key_index);
        if (rc) return rc;
        sz = 16;
      } else if (fd.ttype == TGPU_T_STRUCT) {
        if (fd.struct_index < 0 || (uint32_t)fd.struct_index >= T.ns) return TGPU_ERR_INVALID_ARGUMENT;
        const int rc = value(TGPU_T_STRUCT, fd.struct_index, 0);
        if (rc) return rc;
        if (is_boxed(fd)) facts.nested = facts.has_lists = true;  // objects in the arena
        sz = is_boxed(fd) ? 16 : T.s[fd.struct_index].size;
      } else {
        return TGPU_ERR_UNSUPPORTED;
      }
      if ((uint64_t)fd.member_offset + sz > sd.size) return TGPU_ERR_INVALID_ARGUMENT;
      // natural alignment: a nested struct's own, else min(size, 8)
      const uint32_t al = (fd.ttype == TGPU_T_STRUCT && !is_boxed(fd))
                              ? T.s[fd.struct_index].align : (sz >= 8 ? 8 : sz);
      if (fd.member_offset % al) return TGPU_ERR_INVALID_ARGUMENT;
    }
    return TGPU_OK;
  }
  // struct si's by-value struct members never lead back to si; terse struct
  // members nest at most kMaxTerseDepth deep
  int by_value(uint32_t si, std::vector<uint8_t>& st, int terse_depth) {
    if (st[si] == 1) return TGPU_ERR_UNSUPPORTED;
    if (st[si] == 2 && terse_depth == 0) return TGPU_OK;
    if (terse_depth > kMaxTerseDepth) return TGPU_ERR_UNSUPPORTED;
    st[si] = 1;
    const tgpu_struct_desc& sd = T.s[si];
    for (uint32_t k = 0; k < sd.num_fields; ++k) {
      const tgpu_field_desc& fd = T.f[sd.first_field + k];
      if (fd.ttype != TGPU_T_STRUCT || is_boxed(fd)) continue;
      const int rc = by_value((uint32_t)fd.struct_index, st,
                              fd.qualifier == TGPU_TERSE ? terse_depth + 1 : 0);
      if (rc) return rc;
    }
    st[si] = 2;
    return TGPU_OK;
  }
  int run() {
    sv.assign(T.ns, 0);
    tv.assign(T.nt, 0);
    // type-node chains (type_index / key_index edges between nodes) are
    // finite: a colored DFS over the node graph finds any cycle
    std::vector<uint8_t> color(T.nt, 0);
    for (uint32_t k = 0; k < T.nt; ++k) {
      if (color[k]) continue;
      std::vector<std::pair<uint32_t, int>> stack{{k, 0}};
      color[k] = 1;
      while (!stack.empty()) {
        auto& [x, e] = stack.back();
        const tgpu_type_desc& n = T.t[x];
        const uint32_t nx = e == 0 ? n.type_index : e == 1 ? n.key_index : 0;
        if (e >= 2) {
          color[x] = 2;
          stack.pop_back();
          continue;
        }
        ++e;
        if (!nx || nx > T.nt) continue;
        if (color[nx - 1] == 1) return TGPU_ERR_INVALID_ARGUMENT;
        if (color[nx - 1] == 0) {
          color[nx - 1] = 1;
          stack.push_back({nx - 1, 0});
        }
      }
    }
    sv[0] = 1;
    work.push_back(0);
    while (!work.empty()) {
      const uint32_t si = work.back();
      work.pop_back();
      const int rc = struct_(si);
      if (rc) return rc;
    }
    std::vector<uint8_t> st(T.ns, 0);
    for (uint32_t si = 0; si < T.ns; ++si)
      if (sv[si]) {
        const int rc = by_value(si, st, 0);
        if (rc) return rc;
      }
    return TGPU_OK;
  }
};

int validate(const tgpu_struct_desc* s, uint32_t ns, const tgpu_field_desc* f, uint32_t nf,
             const tgpu_type_desc* t, uint32_t nt, SchemaFacts& facts) {
  const Tables T{s, ns, f, nf, t, nt};
  Validator v{T, facts, {}, {}, {}};
  return v.run();
}

// ---- arena regions of nested schemas (thrift_gpu.h tgpu_schema_arena_scale)
// Every arena byte of a record is charged to wire bytes of its own: an
// element's slot (scalar, span, struct, packed pair) to the element's own
// bytes (a struct element's own bytes can be one STOP), a container's
// allocation padding (<= 7) to its header, a boxed struct's object (+ its
// padding) to its field header and STOP. The region scale is the largest
// bytes-per-wire-byte ratio any element kind of the schema reaches; every
// container description (fields and type nodes) and every boxed field is
// looked at once, so recursive schemas are covered.
uint32_t min_wire(uint32_t t, bool compact) {
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
    default: return 1;  // struct: its STOP
  }
}
uint32_t slot_bytes(const Tables& T, uint32_t t, int32_t si) {
  if (t == TGPU_T_STRUCT) return T.s[si].size;
  if (t == TGPU_T_STRING || is_container_t(t)) return 16;
  return scalar_size(t);
}
// the struct of a key type node (T_STRUCT node), else -1
int32_t key_struct(const Tables& T, uint32_t elem, uint32_t ki) {
  return (elem == TGPU_T_STRUCT && ki) ? T.t[ki - 1].struct_index : -1;
}
void region_ratio(const Tables& T, uint32_t ttype, uint32_t elem, uint32_t val, int32_t si,
                  uint32_t ki, bool compact, double& ratio, uint32_t& slot) {
  if (!is_container_t(ttype)) return;
  const bool is_map = ttype == TGPU_T_MAP;
  const uint32_t v = is_map ? val : elem;
  const uint32_t kb = is_map ? slot_bytes(T, elem, key_struct(T, elem, ki)) : 0;
  const uint32_t kw = is_map ? min_wire(elem, compact) : 0;
  // a pair's bytes + the padding of the containers its key and value open
  const uint32_t pad = (is_container_t(v) ? 7 : 0) + (is_map && is_container_t(elem) ? 7 : 0);
  ratio = std::max(ratio, (double)(kb + slot_bytes(T, v, si) + pad) /
                              (double)(kw + min_wire(v, compact)));
  ratio = std::max(ratio, 7.0 / (double)min_wire(ttype, compact));  // this container's padding
  if (is_complex_t(v) || (is_map && is_complex_t(elem)))
    slot = std::max(slot, kb + slot_bytes(T, v, si));
}
void region_scale(const tgpu_schema& sc, bool compact, uint32_t& scale, uint32_t& slot) {
  const Tables T{sc.structs.data(), (uint32_t)sc.structs.size(), sc.fields.data(),
                 (uint32_t)sc.fields.size(), sc.types.data(), (uint32_t)sc.types.size()};
  double ratio = 8.0;
  slot = 16;
  for (const tgpu_field_desc& f : sc.fields) {
    region_ratio(T, f.ttype, f.elem_ttype, f.val_ttype, f.struct_index, f.key_index, compact,
                 ratio, slot);
    if (f.ttype == TGPU_T_STRUCT && is_boxed(f)) {
      // field header (Binary 3, Compact >= 1) + the struct's STOP
      const uint32_t sz = T.s[f.struct_index].size;
      ratio = std::max(ratio, (double)(sz + 7) / (compact ? 2.0 : 4.0));
      slot = std::max(slot, sz);
    }
  }
  for (const tgpu_type_desc& n : sc.types)
    region_ratio(T, n.ttype, n.elem_ttype, n.val_ttype, n.struct_index, n.key_index, compact,
                 ratio, slot);
  scale = ((uint32_t)std::ceil(ratio) + 7) & ~7u;
  slot = (slot + 15) & ~15u;
}

// Canonical Binary wire template (BinaryProtocol-inl.h:53-67 headers/STOP,
// :120-161 values) for schemas with only unqualified fixed-width fields.
bool build_template(const tgpu_schema& sc, uint32_t si, uint32_t base, FixedTemplate& t,
                    uint32_t& wire) {
  const tgpu_struct_desc& sd = sc.structs[si];
  if (sd.flags & TGPU_STRUCT_UNION) return false;
  for (uint32_t k = 0; k < sd.num_fields; ++k) {
    const tgpu_field_desc& fd = sc.fields[sd.first_field + k];
    // a required field is written always and read like an unqualified one;
    // a canonical record holds every field, so the enforcement never fires
    if (fd.qualifier != TGPU_UNQUALIFIED && fd.qualifier != TGPU_REQUIRED) return false;
    if (t.n_items >= (uint32_t)kMaxTemplateItems || t.n_isset >= 64) return false;
    TemplateItem it{};
    it.wire_off = (uint16_t)wire;
    it.hdr_len = 3;
    it.hdr = (uint32_t)fd.ttype | ((uint32_t)((uint16_t)fd.id >> 8) << 8) |
             ((uint32_t)((uint16_t)fd.id & 0xff) << 16);
    if (is_scalar(fd.ttype)) {
      it.width = (uint8_t)scalar_size(fd.ttype);
      it.member_off = (uint16_t)(base + fd.member_offset);
      it.is_bool = fd.ttype == TGPU_T_BOOL;
      t.items[t.n_items++] = it;
      wire += 3 + it.width;
    } else if (fd.ttype == TGPU_T_STRUCT) {
      t.items[t.n_items++] = it;
      wire += 3;
      if (!build_template(sc, (uint32_t)fd.struct_index, base + fd.member_offset, t, wire))
        return false;
    } else {
      return false;
    }
    t.isset_off[t.n_isset++] = (uint16_t)(base + fd.isset_offset);
  }
  if (t.n_items >= (uint32_t)kMaxTemplateItems) return false;
  TemplateItem stop{};
  stop.wire_off = (uint16_t)wire;
  stop.hdr_len = 1;
  stop.hdr = 0;
  t.items[t.n_items++] = stop;
  wire += 1;
  return true;
}

uint32_t compact_ctype(uint32_t t) {  // CompactProtocol-inl.h:48-69 TTypeToCType
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

bool push_op(VProgram& P, const VOp& op) {
  if (P.n_ops >= (uint32_t)kMaxNestedOps) return false;
  P.ops[P.n_ops++] = op;
  return true;
}

VOp make_op(uint8_t kind) {
  VOp op{};
  op.kind = kind;
  op.isset = 0xffff;
  return op;
}

// Compiles struct si (members at `base`) into the canonical-form program: the
// header bytes the generated writer emits (BinaryProtocol-inl.h:53-59,
// CompactProtocol-inl.h:133-160 incl. long-form ids, bools in the header) and
// each value's encoding.
bool emit_container(const tgpu_schema& sc, uint32_t ttype, uint32_t et, uint32_t vt, int32_t esi,
                    uint32_t eti, uint32_t ki, uint32_t member, uint32_t isset, int proto,
                    VProgram& P, uint32_t depth, uint32_t* max_depth);

// The structs whose ops are being emitted (nested programs): a struct that
// contains itself (a recursive schema, through a container or a boxed field)
// has no finite straight-line program. Its first t_unroll levels are
// unrolled; a value one level deeper is a VOP_DEFER, which hands the record
// to the general kernels when it is present (t_deferred: one was emitted).
// t_unroll 0: recursive schemas stay with the general kernels.
thread_local std::vector<uint32_t> t_open_structs;
thread_local uint32_t t_unroll = 0;
thread_local bool t_deferred = false;
struct OpenStruct {
  bool ok;
  explicit OpenStruct(uint32_t si) {
    ok = (uint32_t)std::count(t_open_structs.begin(), t_open_structs.end(), si) <
         std::max<uint32_t>(t_unroll, 1);
    if (ok) t_open_structs.push_back(si);
  }
  ~OpenStruct() {
    if (ok) t_open_structs.pop_back();
  }
};

// nested (build_nested_program): lists / sets of structs or of scalar lists
// become VOP_SEQ loops whose bodies address the element slot (base 0);
// `depth` tracks the container nesting for the height check.
bool emit_program(const tgpu_schema& sc, uint32_t si, uint32_t base, int proto, VProgram& P,
                  bool nested = false, uint32_t depth = 0, uint32_t* max_depth = nullptr) {
  const tgpu_struct_desc& sd = sc.structs[si];
  const bool un = (sd.flags & TGPU_STRUCT_UNION) != 0;
  if (un && !nested) return false;
  const OpenStruct open(si);
  if (nested && !open.ok) {  // recursive, past the unrolled levels
    if (!t_unroll) return false;
    t_deferred = true;
    return push_op(P, make_op(VOP_DEFER));
  }
  int32_t prev = 0;
  const uint32_t sbegin = P.n_ops;
  if (nested) {
    VOp sb = make_op(VOP_SBEGIN);
    sb.width = un ? 1 : 0;  // a union: at most one member, the first present / set
    if (!push_op(P, sb)) return false;
  }
  for (uint32_t k = 0; k < sd.num_fields; ++k) {
    const tgpu_field_desc& f = sc.fields[sd.first_field + k];
    // a terse field reads like an optional one and is written unless empty
    // (terse structs' emptiness rules stay with the general writer)
    const bool terse = nested && f.qualifier == TGPU_TERSE && f.ttype != TGPU_T_STRUCT;
    // a boxed struct field: the object in the record's region (VOP_BOX);
    // optional boxed ones read / written like optional fields
    const bool box = nested && f.ttype == TGPU_T_STRUCT &&
                     (f.qualifier == TGPU_BOXED || f.qualifier == TGPU_OPTIONAL_BOXED);
    const bool opt = nested && (f.qualifier == TGPU_OPTIONAL || un || terse ||
                                (box && f.qualifier == TGPU_OPTIONAL_BOXED));
    if (f.qualifier != TGPU_UNQUALIFIED && f.qualifier != TGPU_REQUIRED && !opt && !box)
      return false;
    const uint32_t member = base + f.member_offset, isset = base + f.isset_offset;
    if (member > 0xfffe || isset > 0xfffe) return false;
    const uint32_t fhdr = P.n_ops;
    if (nested) {
      // the field header, computed at run time (VOP_FHDR)
      VOp h = make_op(VOP_FHDR);
      h.member = (uint16_t)f.id;
      h.hdr = f.ttype | ((uint32_t)((uint16_t)f.id >> 8) << 8) |
              ((uint32_t)((uint16_t)f.id & 0xff) << 16);
      h.hdr_len = 3;
      h.elem_ct = (uint8_t)(f.ttype == TGPU_T_BOOL ? 0 : compact_ctype(f.ttype));
      h.is_bool = f.ttype == TGPU_T_BOOL;
      h.width = opt ? 1 : 0;
      h.elem_kind = terse ? 1 : 0;  // written when not empty (op::isEmpty), not by isset
      h.isset = (uint16_t)isset;
      if (!push_op(P, h)) return false;
      if (proto != TGPU_PROTOCOL_BINARY && f.ttype == TGPU_T_BOOL) {
        VOp cb = make_op(VOP_CBOOL);  // (its member / isset: the header carries the value)
        cb.member = (uint16_t)member;
        cb.isset = (uint16_t)isset;
        if (!push_op(P, cb)) return false;
        P.ops[fhdr].bits = 1;
        continue;
      }
    }
    VOp hdr = make_op(VOP_CONST);
    if (proto == TGPU_PROTOCOL_BINARY) {
      hdr.hdr_len = 3;
      hdr.hdr = f.ttype | ((uint32_t)((uint16_t)f.id >> 8) << 8) |
                ((uint32_t)((uint16_t)f.id & 0xff) << 16);
    } else {
      const int32_t id = f.id;
      const uint32_t ct = f.ttype == TGPU_T_BOOL ? 0 : compact_ctype(f.ttype);
      if (id > prev && id - prev <= 15) {
        hdr.hdr_len = 1;
        hdr.hdr = ((uint32_t)(id - prev) << 4) | ct;
      } else {
        uint32_t zz = ((uint32_t)id << 1) ^ (uint32_t)(id >> 31);
        uint32_t bytes = ct, n = 1;
        do {
          const uint32_t b = (zz & 0x7f) | (zz > 0x7f ? 0x80 : 0);
          bytes |= b << (8 * n++);
          zz >>= 7;
        } while (zz);
        if (n > 4) return false;
        hdr.hdr_len = (uint8_t)n;
        hdr.hdr = bytes;
      }
      prev = id;
      if (f.ttype == TGPU_T_BOOL) {
        hdr.kind = VOP_CBOOL;
        hdr.member = (uint16_t)member;
        hdr.isset = (uint16_t)isset;
        if (!push_op(P, hdr)) return false;
        continue;
      }
    }
    if (!nested && !push_op(P, hdr)) return false;
    VOp v = make_op(VOP_FIXED);
    v.member = (uint16_t)member;
    v.isset = (uint16_t)isset;
    if (is_scalar(f.ttype)) {
      const uint32_t w = scalar_size(f.ttype);
      if (proto != TGPU_PROTOCOL_BINARY &&
          (f.ttype == TGPU_T_I16 || f.ttype == TGPU_T_I32 || f.ttype == TGPU_T_I64)) {
        v.kind = VOP_VARINT;
        v.bits = f.ttype == TGPU_T_I64 ? 64 : 32;
      }
      v.width = (uint8_t)w;
      v.is_bool = f.ttype == TGPU_T_BOOL;
      if (proto == TGPU_PROTOCOL_COMPACT_V1 && f.ttype == TGPU_T_DOUBLE) v.bits = kFixedLE;
      if (!push_op(P, v)) return false;
    } else if (f.ttype == TGPU_T_STRING) {
      v.kind = VOP_STRING;
      if (!push_op(P, v)) return false;
    } else if (nested && (f.ttype == TGPU_T_MAP || ((f.ttype == TGPU_T_LIST ||
                                                     f.ttype == TGPU_T_SET) &&
                                                    !is_scalar(f.elem_ttype)))) {
      if (!emit_container(sc, f.ttype, f.elem_ttype, f.val_ttype, f.struct_index, f.type_index,
                          f.key_index, member, isset, proto, P, depth, max_depth))
        return false;
    } else if (f.ttype == TGPU_T_LIST || f.ttype == TGPU_T_SET) {
      v.kind = VOP_LIST;
      const uint32_t e = f.elem_ttype;
      if (!is_scalar(e)) return false;  // string elements: general kernels
      v.width = (uint8_t)scalar_size(e);
      v.elem_ttype = (uint8_t)e;
      v.elem_ct = (uint8_t)compact_ctype(e);
      v.elem_kind = VEL_FIXED;
      if (e == TGPU_T_BOOL) v.elem_kind = VEL_BOOL;
      if (proto == TGPU_PROTOCOL_COMPACT_V1 && e == TGPU_T_DOUBLE) v.bits = kFixedLE;
      if (proto != TGPU_PROTOCOL_BINARY &&
          (e == TGPU_T_I16 || e == TGPU_T_I32 || e == TGPU_T_I64)) {
        v.elem_kind = VEL_VARINT;
        v.bits = e == TGPU_T_I64 ? 64 : 32;
      }
      P.has_list = 1;
      if (max_depth) *max_depth = std::max(*max_depth, depth + 1);
      if (!push_op(P, v)) return false;
    } else if (box) {
      VOp bx = make_op(VOP_BOX);
      bx.member = (uint16_t)member;
      bx.hdr = sc.structs[f.struct_index].size;
      const uint32_t at = P.n_ops;
      if (!push_op(P, bx) ||
          !emit_program(sc, (uint32_t)f.struct_index, 0, proto, P, true, depth, max_depth) ||
          !push_op(P, make_op(VOP_BOX_END)))
        return false;
      P.ops[at].hdr_len = (uint8_t)P.n_ops;  // one past the VOP_BOX_END
      VOp is = make_op(VOP_ISSET);
      is.isset = (uint16_t)isset;
      if (!push_op(P, is)) return false;
    } else if (f.ttype == TGPU_T_STRUCT) {
      if (!emit_program(sc, (uint32_t)f.struct_index, member, proto, P, nested, depth, max_depth))
        return false;
      VOp stop = make_op(VOP_CONST);
      stop.hdr_len = 1;
      VOp is = make_op(VOP_ISSET);
      is.isset = (uint16_t)isset;
      if ((!nested && !push_op(P, stop)) || !push_op(P, is)) return false;
    } else {
      return false;
    }
    if (nested) {
      const uint32_t nv = P.n_ops - fhdr - 1;  // the field's value ops
      if (nv > 255) return false;
      P.ops[fhdr].bits = (uint8_t)nv;
    }
  }
  if (nested) {
    if (!push_op(P, make_op(VOP_SEND))) return false;
    P.ops[sbegin].hdr_len = (uint8_t)P.n_ops;  // one past its VOP_SEND
  }
  return true;
}

// A leaf value op at member: a scalar or a string view. A bool here is a
// container's (a map key / value): one byte, Binary 0 / 1, Compact 1 / 2
// (CompactProtocol-inl.h:692-701: byte == 1 is true).
bool emit_leaf(uint32_t t, uint32_t member, int proto, VProgram& P) {
  VOp v = make_op(VOP_FIXED);
  v.member = (uint16_t)member;
  if (t == TGPU_T_STRING) {
    v.kind = VOP_STRING;
  } else if (is_scalar(t)) {
    v.width = (uint8_t)scalar_size(t);
    v.is_bool = t == TGPU_T_BOOL;
    if (proto == TGPU_PROTOCOL_COMPACT_V1 && t == TGPU_T_DOUBLE) v.bits = kFixedLE;
    if (proto != TGPU_PROTOCOL_BINARY && (t == TGPU_T_I16 || t == TGPU_T_I32 || t == TGPU_T_I64)) {
      v.kind = VOP_VARINT;
      v.bits = t == TGPU_T_I64 ? 64 : 32;
    }
  } else {
    return false;
  }
  return push_op(P, v);
}

// One value of type t (struct si / type node ti) in a container slot at
// member: a struct's fields + STOP, a container, or a leaf.
bool emit_value(const tgpu_schema& sc, uint32_t t, int32_t si, uint32_t ti, uint32_t member,
                int proto, VProgram& P, uint32_t depth, uint32_t* max_depth) {
  if (t == TGPU_T_STRUCT) {
    if (si < 0 || (uint32_t)si >= sc.structs.size()) return false;
    return emit_program(sc, (uint32_t)si, member, proto, P, true, depth, max_depth);
  }
  if (t == TGPU_T_LIST || t == TGPU_T_SET || t == TGPU_T_MAP) {
    if (ti == 0 || ti > sc.types.size()) return false;
    const tgpu_type_desc& n = sc.types[ti - 1];
    if (n.ttype != t) return false;
    return emit_container(sc, t, n.elem_ttype, n.val_ttype, n.struct_index, n.type_index,
                          n.key_index, member, 0xffff, proto, P, depth, max_depth);
  }
  return emit_leaf(t, member, proto, P);
}

// Bytes of a container slot holding a value of type t.
uint32_t slot_bytes(const tgpu_schema& sc, uint32_t t, int32_t si) {
  if (t == TGPU_T_STRUCT) return si >= 0 && (uint32_t)si < sc.structs.size() ? sc.structs[si].size : 0;
  if (t == TGPU_T_STRING || t == TGPU_T_LIST || t == TGPU_T_SET || t == TGPU_T_MAP)
    return (uint32_t)sizeof(tgpu_span);
  return scalar_size(t);
}

// A container value (list / set / map) whose span is at member (isset:
// 0xffff inside containers). Lists of scalars / strings are one VOP_LIST;
// lists of structs / containers a VOP_SEQ loop; maps a VOP_MSEQ loop with
// the key (a non-bool scalar or a string) and the value in the body.
bool emit_container(const tgpu_schema& sc, uint32_t ttype, uint32_t et, uint32_t vt, int32_t esi,
                    uint32_t eti, uint32_t ki, uint32_t member, uint32_t isset, int proto,
                    VProgram& P, uint32_t depth, uint32_t* max_depth) {
  if (member > 0xfffe) return false;
  const uint32_t d = depth + 1;  // this container's level
  if (max_depth) *max_depth = std::max(*max_depth, d);
  if (ttype == TGPU_T_LIST || ttype == TGPU_T_SET) {
    if (is_scalar(et) || et == TGPU_T_STRING) {  // elements read in place
      VOp v = make_op(VOP_LIST);
      v.member = (uint16_t)member;
      v.isset = (uint16_t)isset;
      v.elem_ttype = (uint8_t)et;
      v.elem_ct = (uint8_t)compact_ctype(et);
      if (et == TGPU_T_STRING) {
        v.width = (uint8_t)sizeof(tgpu_span);
        v.elem_kind = VEL_STRING;
      } else {
        v.width = (uint8_t)scalar_size(et);
        v.elem_kind = et == TGPU_T_BOOL ? VEL_BOOL : VEL_FIXED;
        if (proto == TGPU_PROTOCOL_COMPACT_V1 && et == TGPU_T_DOUBLE) v.bits = kFixedLE;
        if (proto != TGPU_PROTOCOL_BINARY &&
            (et == TGPU_T_I16 || et == TGPU_T_I32 || et == TGPU_T_I64)) {
          v.elem_kind = VEL_VARINT;
          v.bits = et == TGPU_T_I64 ? 64 : 32;
        }
      }
      P.has_list = 1;
      return push_op(P, v);
    }
    VOp q = make_op(VOP_SEQ);
    q.member = (uint16_t)member;
    q.isset = (uint16_t)isset;
    q.elem_ttype = (uint8_t)et;
    q.elem_ct = (uint8_t)compact_ctype(et);
    q.hdr = slot_bytes(sc, et, esi);
    const uint32_t at = P.n_ops;
    if (!q.hdr || !push_op(P, q) || !emit_value(sc, et, esi, eti, 0, proto, P, d, max_depth) ||
        !push_op(P, make_op(VOP_SEQ_END)))
      return false;
    P.ops[at].hdr_len = (uint8_t)P.n_ops;  // one past the matching VOP_SEQ_END
    P.has_list = 1;
    return true;
  }
  if (ttype != TGPU_T_MAP) return false;
  // the key: a scalar or string leaf, or (key_index) a struct / container
  // key, whose node names its struct or is the key container's node
  int32_t ksi = -1;
  uint32_t kti = 0;
  if (ki) {
    if (ki > sc.types.size()) return false;
    const tgpu_type_desc& kn = sc.types[ki - 1];
    if (et == TGPU_T_STRUCT) {
      if (kn.ttype != TGPU_T_STRUCT) return false;
      ksi = kn.struct_index;
    } else if (et == TGPU_T_LIST || et == TGPU_T_SET || et == TGPU_T_MAP) {
      kti = ki;
    } else {
      return false;
    }
  } else if (!(et == TGPU_T_STRING || is_scalar(et))) {
    return false;
  }
  const uint32_t ks = slot_bytes(sc, et, ksi);
  if (!ks || ks > 255) return false;
  VOp q = make_op(VOP_MSEQ);
  q.member = (uint16_t)member;
  q.isset = (uint16_t)isset;
  q.width = (uint8_t)et;            // key ttype
  q.bits = (uint8_t)ks;             // key slot bytes
  q.elem_ttype = (uint8_t)vt;       // value ttype
  q.elem_ct = (uint8_t)((compact_ctype(et) << 4) | compact_ctype(vt));
  const uint32_t vs = slot_bytes(sc, vt, esi);
  q.hdr = q.bits + vs;
  const uint32_t at = P.n_ops;
  if (!vs || !push_op(P, q) ||
      !(ki ? emit_value(sc, et, ksi, kti, 0, proto, P, d, max_depth)
           : emit_leaf(et, 0, proto, P)) ||
      !emit_value(sc, vt, esi, eti, q.bits, proto, P, d, max_depth) ||
      !push_op(P, make_op(VOP_SEQ_END)))
    return false;
  P.ops[at].hdr_len = (uint8_t)P.n_ops;
  P.has_list = 1;
  return true;
}

// The nested program of a schema whose containers hold structs or scalar
// lists (every field unqualified / required, no maps, no strings inside
// containers): compiled by JIT_NESTED only. A recursive schema unrolls as
// many levels as fit the op budget, at most TGPU_NESTED_UNROLL (default 16;
// 0: none — such schemas keep the general kernels); *deferred: the program
// holds VOP_DEFERs (decode / measure only: the writer stays general).
bool build_nested_program(const tgpu_schema& sc, int proto, VProgram& P, uint32_t& depth,
                          bool* deferred = nullptr) {
  if (proto == kV1Slot) proto = TGPU_PROTOCOL_COMPACT_V1;  // (a program slot)
  const char* v = getenv("TGPU_NESTED_UNROLL");
  const uint32_t max_unroll = v ? (uint32_t)std::min(atoi(v) < 0 ? 0 : atoi(v), 64) : 16u;
  if (deferred) *deferred = false;
  for (uint32_t k = max_unroll ? max_unroll : 1; k >= 1; --k) {
    P = VProgram{};
    P.protocol = (uint32_t)(proto == TGPU_PROTOCOL_COMPACT_V1 ? TGPU_PROTOCOL_COMPACT : proto);
    P.rec_size = sc.structs[0].size;
    depth = 0;
    t_open_structs.clear();
    t_unroll = max_unroll ? k : 0;
    t_deferred = false;
    const bool ok = emit_program(sc, 0, 0, proto, P, true, 0, &depth);
    const bool rec = t_deferred;
    t_unroll = 0;
    if (ok) {
      if (deferred) *deferred = rec;
      return true;
    }
    // (a schema that is not recursive, or whose failure is not the op
    // budget, fails the same way at every level)
    if (!max_unroll || (!rec && P.n_ops < (uint32_t)kMaxNestedOps)) break;
  }
  return false;
}

// The bytes a record of the root struct can start with (IndexArgs::hmask):
// the header of a root field that can be the first one written. Generated
// writers emit fields in declaration order (serialize_struct.whisker), or in
// id order for a struct annotated @SerializeInFieldIdOrder
// (t_whisker_generator.cc:232-236, fields_in_serialization_order) — the
// schema descriptor does not say which, so both orders' candidates are taken:
// in each, the fields up to the first one always written (unqualified,
// required, boxed). Binary: the field's type byte; Compact: its short-form
// header (delta from 0, ids 1..15; a bool either value) or the long form's
// type nibble alone. STOP only when every field may be absent (an empty
// record; a union root). A record whose first field is unknown to the
// schema, or written in some third order, fails the filter: the
// speculation's fallback pass, which takes any record, covers it.
void record_first_bytes(const tgpu_schema& sc, int protocol, uint32_t m[8]) {
  for (int k = 0; k < 8; ++k) m[k] = 0;
  auto set = [&](uint32_t b) { m[(b & 0xff) >> 5] |= 1u << (b & 31); };
  const tgpu_struct_desc& root = sc.structs[0];
  const bool un = (root.flags & TGPU_STRUCT_UNION) != 0;
  std::vector<uint32_t> decl(root.num_fields), by_id;
  for (uint32_t k = 0; k < root.num_fields; ++k) decl[k] = root.first_field + k;
  by_id = decl;
  std::stable_sort(by_id.begin(), by_id.end(),
                   [&](uint32_t a, uint32_t b) { return sc.fields[a].id < sc.fields[b].id; });
  bool may_be_empty = true;
  for (const std::vector<uint32_t>* order : {&decl, &by_id}) {
    bool always = false;
    for (uint32_t k = 0; k < (uint32_t)order->size() && !always; ++k) {
      const tgpu_field_desc& f = sc.fields[(*order)[k]];
      always = !un && (f.qualifier == TGPU_UNQUALIFIED || f.qualifier == TGPU_REQUIRED ||
                       f.qualifier == TGPU_BOXED);
      if (protocol == TGPU_PROTOCOL_BINARY) {
        set(f.ttype);
        continue;
      }
      const uint32_t cts[2] = {f.ttype == TGPU_T_BOOL ? 1u : compact_ctype(f.ttype),
                               f.ttype == TGPU_T_BOOL ? 2u : compact_ctype(f.ttype)};
      for (uint32_t ct : cts) {
        if (f.id >= 1 && f.id <= 15) set(((uint32_t)f.id << 4) | ct);
        else set(ct);
      }
    }
    may_be_empty = !always;
  }
  if (may_be_empty) set(0);
}

// Whether a struct is reachable from itself (tgpu_schema::recursive): the
// nested emitter, one level unrolled, meets a struct already open. (A shape
// the emitter refuses before that reads as not recursive: one deep tier.)
bool schema_recursive(const tgpu_schema& sc) {
  VProgram P{};
  P.protocol = TGPU_PROTOCOL_BINARY;
  P.rec_size = sc.structs[0].size;
  uint32_t depth = 0;
  t_open_structs.clear();
  t_unroll = 1;
  t_deferred = false;
  (void)emit_program(sc, 0, 0, TGPU_PROTOCOL_BINARY, P, true, 0, &depth);
  const bool rec = t_deferred;
  t_unroll = 0;
  return rec;
}

// (proto: a protocol id or a program slot: kV1Slot is CompactV1's)
bool build_program(const tgpu_schema& sc, int proto, VProgram& P, bool tolerant = false) {
  if (proto == kV1Slot) proto = TGPU_PROTOCOL_COMPACT_V1;
  P = VProgram{};
  P.protocol = (uint32_t)(proto == TGPU_PROTOCOL_COMPACT_V1 ? TGPU_PROTOCOL_COMPACT : proto);
  P.rec_size = sc.structs[0].size;
  if (!emit_program(sc, 0, 0, proto, P) || P.n_ops >= (uint32_t)kMaxProgramOps) return false;
  VOp stop = make_op(VOP_CONST);
  stop.hdr_len = 1;
  const tgpu_struct_desc& root = sc.structs[0];
  if (tolerant && root.num_fields) {
    int32_t max_id = -32768;
    for (uint32_t k = 0; k < root.num_fields; ++k)
      max_id = std::max<int32_t>(max_id, sc.fields[root.first_field + k].id);
    const int16_t last = sc.fields[root.first_field + root.num_fields - 1].id;
    stop.elem_kind = kStopSkipsUnknown;
    stop.member = (uint16_t)(int16_t)max_id;
    stop.hdr = (uint32_t)(uint16_t)last << 8;
  }
  return push_op(P, stop);
}

// Regroups the template by 8-byte word of the record layout (FixedPlan).
bool build_plan(const FixedTemplate& t, FixedPlan& p) {
  if (t.record_size % 8 || t.record_size / 8 > (uint32_t)kMaxPlanWords || t.record_size == 0)
    return false;
  p = FixedPlan{};
  p.wire_len = t.wire_len;
  p.n_words = t.record_size / 8;
  std::vector<std::vector<PlanItem>> bucket(p.n_words);
  for (uint32_t i = 0; i < t.n_items; ++i) {
    const TemplateItem& ti = t.items[i];
    PlanItem pi{};
    pi.wire_off = ti.wire_off;
    pi.hdr_len = ti.hdr_len;
    pi.width = ti.width;
    pi.hdr = ti.hdr;
    pi.is_bool = ti.is_bool;
    uint32_t j = p.n_words - 1;
    if (ti.width) {
      j = ti.member_off / 8;
      pi.dst = (uint8_t)(ti.member_off % 8);
      if (pi.dst + ti.width > 8) return false;
    }
    bucket[j].push_back(pi);
  }
  for (uint32_t k = 0; k < t.n_isset; ++k)
    p.words[t.isset_off[k] / 8].const_bits |= 1ull << (8 * (t.isset_off[k] % 8));
  uint32_t at = 0;
  for (uint32_t j = 0; j < p.n_words; ++j) {
    p.words[j].first_item = (uint16_t)at;
    p.words[j].n_items = (uint8_t)bucket[j].size();
    for (const PlanItem& pi : bucket[j]) {
      p.words[j].has_value |= pi.width ? 1 : 0;
      p.items[at++] = pi;
    }
  }
  p.n_items = at;
  return true;
}

void classify(int code, int32_t* exc, int32_t* tp) {
  int32_t e = TGPU_EXC_RUNTIME, t = 0;
  switch (code) {
    case TGPU_OK: e = TGPU_EXC_NONE; break;
    case TGPU_ERR_UNDERFLOW: case TGPU_ERR_INVALID_VARINT: e = TGPU_EXC_OUT_OF_RANGE; break;
    case TGPU_ERR_BOOL_VALUE: case TGPU_ERR_INVALID_SKIP_TYPE: case TGPU_ERR_TRUNCATED:
    case TGPU_ERR_UNION_MISSING_STOP:
      e = TGPU_EXC_PROTOCOL; t = 1; break;
    case TGPU_ERR_NEGATIVE_SIZE: e = TGPU_EXC_PROTOCOL; t = 2; break;
    case TGPU_ERR_SIZE_LIMIT: case TGPU_ERR_WRITE_SIZE_LIMIT: e = TGPU_EXC_PROTOCOL; t = 3; break;
    case TGPU_ERR_DEPTH_LIMIT: e = TGPU_EXC_PROTOCOL; t = 8; break;
    case TGPU_ERR_MISSING_REQUIRED_FIELD: e = TGPU_EXC_PROTOCOL; t = 6; break;
    case TGPU_ERR_BAD_TYPE: e = TGPU_EXC_PROTOCOL; t = 0; break;
    case TGPU_ERR_INVALID_BOOL_WRITE: e = TGPU_EXC_ABORT; break;
    default: break;
  }
  if (exc) *exc = e;
  if (tp) *tp = t;
}

void fill_status(tgpu_status* st, int code, uint64_t rec, uint64_t off) {
  if (!st) return;
  std::memset(st, 0, sizeof(*st));
  st->code = code;
  classify(code, &st->exc_class, &st->tproto_type);
  st->record = rec;
  st->byte_offset = off;
}

// Fixed-layout decodes: exception list entries read at their stride (beyond
// it the stream is indexed from the first exception); blocking calls of at
// least kFixedProbeMin records check record 0's length first.
constexpr uint64_t kFixedExceptionCap = 1ull << 20;
constexpr uint64_t kFixedProbeMin = 1ull << 16;

int ensure_workspace(tgpu_context* ctx, uint64_t n) {
  if (n <= ctx->reserved && ctx->d_offs) return TGPU_OK;
  const uint64_t want = std::max<uint64_t>(n, 1024);
  if (ctx->d_offs) (void)hipFree(ctx->d_offs);
  if (ctx->d_block_sums) (void)hipFree(ctx->d_block_sums);
  if (ctx->d_scan_part) (void)hipFree(ctx->d_scan_part);
  if (ctx->d_irr) (void)hipFree(ctx->d_irr);
  if (ctx->d_deep) (void)hipFree(ctx->d_deep);
  if (ctx->d_deep2) (void)hipFree(ctx->d_deep2);
  ctx->d_offs = nullptr;
  ctx->d_block_sums = nullptr;
  ctx->d_scan_part = nullptr;
  ctx->d_irr = nullptr;
  ctx->d_deep = nullptr;
  ctx->d_deep2 = nullptr;
  ctx->reserved = 0;
  const uint64_t tiles = (want + 255) / 256;
  if (hipMalloc(&ctx->d_offs, (want + 1) * sizeof(uint64_t)) != hipSuccess) return TGPU_ERR_HIP;
  if (hipMalloc(&ctx->d_block_sums, (tiles + 1) * sizeof(unsigned long long)) != hipSuccess)
    return TGPU_ERR_HIP;
  if (hipMalloc(&ctx->d_scan_part, (scan_tiles_parts(tiles) + 1) * sizeof(unsigned long long)) !=
      hipSuccess)
    return TGPU_ERR_HIP;
  if (hipMalloc(&ctx->d_irr, want * sizeof(uint64_t)) != hipSuccess) return TGPU_ERR_HIP;
  if (hipMalloc(&ctx->d_deep, want * sizeof(uint64_t)) != hipSuccess) return TGPU_ERR_HIP;
  if (hipMalloc(&ctx->d_deep2, want * sizeof(uint64_t)) != hipSuccess) return TGPU_ERR_HIP;
  // the block rule's per-block marks (compared with the call's epoch: never
  // cleared, zeroed once here)
  if (ctx->d_pack_flags) (void)hipFree(ctx->d_pack_flags);
  ctx->d_pack_flags = nullptr;
  const uint64_t blocks = (want + kArenaBlock - 1) / kArenaBlock + 1;
  if (hipMalloc(&ctx->d_pack_flags, blocks * sizeof(uint32_t)) != hipSuccess ||
      hipMemset(ctx->d_pack_flags, 0, blocks * sizeof(uint32_t)) != hipSuccess)
    return TGPU_ERR_HIP;
  ctx->reserved = want;
  return TGPU_OK;
}

// A decode call of a block-rule schema: its epoch and marks (DecodeArgs
// pack_*), the program's list ops for the compiled decode tile's table.
void pack_args(tgpu_context* ctx, const tgpu_schema* schema, int protocol, DecodeArgs& a) {
  a.pack_flags = nullptr;
  a.pack_k = 0;
  if (!schema->pack.n || !a.arena) return;
  // (A/B only: TGPU_ARENA_PACK=0 keeps the position rule — the spans then
  // differ from the oracle's)
  if (const char* v = getenv("TGPU_ARENA_PACK"))
    if (v[0] == '0') return;
  if (++ctx->pack_epoch == 0) ++ctx->pack_epoch;  // (0: the flags' initial value)
  a.pack_flags = ctx->d_pack_flags;
  a.pack_epoch = ctx->pack_epoch;
  const int q = prog_protocol(schema, protocol);
  if (protocol == TGPU_PROTOCOL_BINARY && q >= 0 && schema->has_prog[q])
    a.pack_k = prog_list_ops(schema->prog[q]);
}

// After a decode call's finish kernel: the blocks the decode did not pack.
hipError_t finish_pack(const tgpu_schema* schema, int protocol, const DecodeArgs& a,
                       hipStream_t s) {
  if (!a.pack_flags) return hipSuccess;
  ArenaPack p = schema->pack;
  p.scale = protocol == TGPU_PROTOCOL_BINARY ? 1u : 8u;
  return launch_arena_pack(a, p, s);
}

// Frames for the deep pass: max_depth + 2 skip frames and as many record
// frames per lane (the skip's depth check fires first; records nest through
// containers, each a level of depth, or through boxed fields, past which
// the slab's record frames are the limit: TGPU_ERR_UNSUPPORTED), up to
// kMaxDeepFrames; as many lanes (<= 256) as fit 64 MiB. The pass's width
// only bounds its time, never its result; for a recursive schema (`wide`)
// whose slabs hold more than kWideFrames, the wide tier (DeepArgs, 256 MiB)
// reads the deferred records first (such a schema defers most of its
// records: TGPU_DEEP_WIDE=0 keeps one tier).
int ensure_deep(tgpu_context* ctx, int32_t max_depth, bool wide = false) {
  const uint64_t want = std::min<uint64_t>(std::max<int64_t>((int64_t)max_depth + 2, 1),
                                           kMaxDeepFrames);
  const char* wv = getenv("TGPU_DEEP_WIDE");
  if (wide && want > kWideFrames && !ctx->d_wslabs && !(wv && wv[0] == '0')) {
    // The wide tier only makes the pass faster (the max_depth tier alone
    // gives the same records), so it takes at most 256 MiB and an eighth of
    // the free device memory, and a device that cannot spare it runs one
    // tier: a failed allocation is cleared and the call goes on.
    const uint64_t lb = slab_lane_bytes(kWideFrames);
    size_t free_b = 0, total_b = 0;
    uint64_t cap = 256ull << 20;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) cap = std::min<uint64_t>(cap, free_b / 8);
    else (void)hipGetLastError();
    const uint32_t lanes = (uint32_t)std::min<uint64_t>(kWideLanes, cap / lb) & ~63u;
    if (lanes && hipMalloc(&ctx->d_wslabs, (uint64_t)lanes * lb) == hipSuccess) {
      ctx->wslab_lanes = lanes;
    } else {
      (void)hipGetLastError();
      ctx->d_wslabs = nullptr;
      ctx->wslab_lanes = 0;
    }
  }
  if (ctx->d_slabs && ctx->slab_frames >= want) return TGPU_OK;
  if (ctx->d_slabs) (void)hipFree(ctx->d_slabs);
  ctx->d_slabs = nullptr;
  ctx->slab_frames = 0;
  ctx->slab_lanes = 0;
  const uint64_t lane_bytes = slab_lane_bytes(want);
  const uint64_t lanes = std::min<uint64_t>(256, std::max<uint64_t>(1, (64ull << 20) / lane_bytes));
  if (hipMalloc(&ctx->d_slabs, lanes * lane_bytes) != hipSuccess) return TGPU_ERR_HIP;
  ctx->slab_frames = want;
  ctx->slab_lanes = (uint32_t)lanes;
  return TGPU_OK;
}

DeepArgs deep_args(tgpu_context* ctx) {
  // (the wide tier only when the slabs are deeper than it; TGPU_DEEP_WIDE=0:
  // one tier, A/B)
  const char* wv = getenv("TGPU_DEEP_WIDE");
  const bool wide = ctx->d_wslabs && ctx->d_deep2 && ctx->slab_frames > kWideFrames &&
                    !(wv && wv[0] == '0');
  return DeepArgs{ctx->d_deep, &ctx->d_res->n_deep, ctx->d_slabs, ctx->slab_frames,
                  ctx->slab_lanes, 0, wide ? ctx->d_wslabs : nullptr, wide ? ctx->wslab_lanes : 0u,
                  0, ctx->d_deep2, &ctx->d_res->n_deep2};
}

int32_t limit_depth(const tgpu_limits* limits) { return limits ? limits->max_depth : 12000; }

// TGPU_INDEX_ONEPASS=1: blocking calls try the single-pass stream index
// first (launch_index_onepass). Off by default: it measured slower than the
// two passes (config 5: 7.4 ms vs 3.0 + 3.0 ms).
bool onepass_enabled() {
  const char* e = getenv("TGPU_INDEX_ONEPASS");
  return e && e[0] == '1';
}
// The one pass over the candidate-list speculation with register records
// (index_onepass_rr_tile): the default for a decode of a stream a record
// program indexes; TGPU_INDEX_ONEPASS=0 keeps the two passes (A/B), =1 the
// round-2 slice-speculation one pass.
bool onepass_rr_enabled() {
  const char* e = getenv("TGPU_INDEX_ONEPASS");
  return !e || !e[0] || e[0] == '2';
}

// TGPU_PROGRAM_TAILS=1: every decode / index uses the programs that take
// appended unknown fields (A/B and tests; by default only the fixed-layout
// path's probe selects them).
bool tails_everywhere() {
  const char* e = getenv("TGPU_PROGRAM_TAILS");
  return e && e[0] == '1';
}

// The schema's compiled kernels for `protocol` (tgpu_jit.cpp policy), or
// nullptr: the interpreting kernels run.
const JitKernels* schema_jit(const tgpu_schema* s, int protocol, int group, uint64_t records,
                             uint64_t bytes) {
  if (!has_prog(s, protocol)) return nullptr;
  return jit_kernels(s->prog[prog_protocol(s, protocol)], s->device, group, records, bytes, false);
}

// Stream-ordered fixed-layout calls: the tolerant program's compiled decode
// group, whose strided tail decode re-reads the records from a misfit on
// (nullptr: a batch under the probe's size, no program, a height the program
// cannot read at, or the compile policy — the finish kernel's lane walks).
// TGPU_STREAM_TAIL=0 turns it off (A/B).
const JitKernels* stream_tail_jit(const tgpu_schema* s, int protocol, const DecodeArgs& a) {
  const char* v = getenv("TGPU_STREAM_TAIL");
  if (v && v[0] == '0') return nullptr;
  const int32_t height = a.height ? a.height : a.max_depth;
  if (a.n < kFixedProbeMin || !has_prog(s, protocol) || height < 2 || a.max_depth < 2 ||
      !stream_tail_max_stride(a.rec_size, s->tmpl.wire_len))
    return nullptr;
  const JitKernels* J =
      jit_kernels(s->prog_tol[prog_protocol(s, protocol)], s->device, JIT_DECODE, a.n, 0, false);
  return jit_has(J, 1) ? J : nullptr;
}

// Fixed-layout Binary schemas: the compiled program kernels instead of the
// word-gather plan kernels (TGPU_FIXED_PATH=jit; A/B).
const JitKernels* fixed_jit(const tgpu_schema* s, int protocol, int group, uint64_t n) {
  const char* e = getenv("TGPU_FIXED_PATH");
  if (!e || strcmp(e, "jit") != 0) return nullptr;
  if (!has_prog(s, protocol) || 256ull * s->tmpl.wire_len > 24 * 1024) return nullptr;
  return jit_kernels(s->prog[prog_protocol(s, protocol)], s->device, group, n, 0, false);
}

DevSchema dev_schema(const tgpu_schema* s, int protocol) {
  const uint32_t scale =
      s->nested ? s->region_scale[protocol == TGPU_PROTOCOL_BINARY ? 0 : 1] : 0u;
  return DevSchema{s->d_structs, s->d_fields, s->d_types, (uint32_t)s->structs.size(),
                   (uint32_t)s->fields.size(), s->str_elems ? 1u : 0u, scale, s->nest_slot,
                   (uint32_t)s->types.size()};
}

// Scratch bytes per record of a measuring read (stream index): the root
// record, then one element slot every nesting level shares (the measuring
// reader only writes objects, never reads them back).
uint64_t measure_scratch(const tgpu_schema* s) {
  const uint64_t root = (s->structs[0].size + 15) & ~15ull;
  return root + (s->nested ? (uint64_t)s->nest_slot : 0);
}

// Indexed decode (a.offs = record starts): compiled-program fast path, then
// the general decoder for the records it hands over; general decoder only
// when the schema has no program or the limits forbid its fast path (a list
// depth of 1 must be allowed: the program never skips, so max_depth is not
// reached otherwise).
// The nested program's compiled kernels for a call of n records (nullptr:
// none — no nested program, a height below its nesting (decode),
// TGPU_NESTED=0, not compiled).
const JitKernels* nested_jit(const tgpu_schema* schema, int protocol, uint64_t n, int32_t height,
                             int32_t max_depth) {
  const char* v = getenv("TGPU_NESTED");
  if (v && v[0] == '0') return nullptr;
  const int q = prog_protocol(schema, protocol);
  if (q < 0 || !schema->has_nprog[q] || n == 0) return nullptr;
  const int32_t need = (int32_t)schema->nprog_depth[q] + 1;
  if (height < need || max_depth < need) return nullptr;
  return jit_kernels(schema->nprog[q], schema->device, JIT_NESTED, n, 0, false);
}

// Whether the schema's nested program is a recursive schema's unrolled one
// (VOP_DEFER: its writer hands the records nesting past its levels to the
// general writer's deep pass).
bool nested_defers(const tgpu_schema* schema, int protocol) {
  const int q = prog_protocol(schema, protocol);
  return q >= 0 && schema->nprog_defer[q];
}

// The nested program's compiled decode (JIT_NESTED) of an indexed batch,
// then the general decoder over the records it left; false: no such kernel
// (no nested program, a height below its nesting, TGPU_NESTED=0, not
// compiled), the caller runs the general decoder.
// TGPU_NESTED_SRC=hbm / lds: the unstaged / staged variant (A/B).
bool launch_nested_decode(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                          const DecodeArgs& a, hipStream_t s, hipError_t& e) {
  const char* v = getenv("TGPU_NESTED_SRC");
  bool hbm = v && !strcmp(v, "hbm");
  const char* rv = getenv("TGPU_NESTED_RTILE");  // A/B: 0 = records straight to HBM, no LDS record tile
  bool rtile = !(rv && rv[0] == '0');
  const JitKernels* J =
      nested_jit(schema, protocol, a.n, a.height ? a.height : a.max_depth, a.max_depth);
  if (!J) return false;
  constexpr uint32_t kPT = 256;  // records per tile (prog::kPT)
  const uint64_t tiles = (a.n + kPT - 1) / kPT;
  // the wire tile: 1.15 x the mean tile + 1 KiB, within 80 KiB of LDS with
  // the record tile (half a CU's 160 KiB: two workgroups per CU; a larger
  // tile's records take the general decoder). TGPU_NESTED_LDS=<bytes>
  // overrides the 80 KiB (A/B).
  uint32_t rt = rtile ? (kPT * a.rec_size + 16 + 15) & ~15u : 0u;
  const double mean = (double)a.in_len / (double)a.n * kPT;
  double cap = 1.15 * mean + 1024.0;
  const char* lv = getenv("TGPU_NESTED_LDS");
  const double lds_max = lv ? std::min(atof(lv), 163840.0) : 81920.0;
  // a record tile that leaves no room for the smallest wire region (root
  // records of ~300 B and more) is dropped: records go straight to HBM
  // (entry 1), the wire tile keeps the LDS
  if (rt && rt + 4096.0 + 4096.0 + 32.0 > lds_max) rtile = false, rt = 0;
  double room = lds_max - rt - 4096.0 - 32.0;
  // a mean tile the wire tile cannot hold would fail every tile's staging
  // (all its records to the general decoder — the golden trees, ~1.5 KB a
  // record): the record tile gives way first, then the staging (records
  // read from HBM, entry 1 with wire_cap 0); TGPU_NESTED_SRC=lds keeps it
  if (cap > room && rt && cap <= lds_max - 4096.0 - 32.0)
    rtile = false, rt = 0, room = lds_max - 4096.0 - 32.0;
  if (cap > room && !hbm && !(v && !strcmp(v, "lds"))) hbm = true;
  if (cap > room) cap = room;
  if (cap < 4096.0) cap = 4096.0;
  const uint32_t wire_cap = (uint32_t)cap & ~15u;
  // (prog::decode_wire_region: whole 4 KiB staging rounds)
  const uint32_t lds = hbm ? 0 : (wire_cap + 32 + 4095) / 4096 * 4096 + rt;
  // (entry 1: the variant without the LDS record tile, or with wire_cap 0
  // the unstaged one)
  e = jit_launch_decode(J, a, tiles, hbm ? 0 : wire_cap, lds, ctx->d_irr,
                        &ctx->d_res->n_irregular, s, hbm || !rtile ? 1 : 0);
  if (e == hipSuccess)
    e = launch_general_decode_list(a, protocol, ctx->d_irr, &ctx->d_res->n_irregular, s);
  return true;
}

hipError_t launch_indexed_decode(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                                 const DecodeArgs& a, hipStream_t s) {
  {
    hipError_t e = hipSuccess;
    if (launch_nested_decode(ctx, schema, protocol, a, s, e)) return e;
  }
  const int32_t height = a.height ? a.height : a.max_depth;
  if (has_prog(schema, protocol) && height >= 2 && a.max_depth >= 2) {
    const int q = prog_protocol(schema, protocol);
    const bool tol = tails_everywhere();
    hipError_t e = launch_program_decode(
        a, tol ? schema->d_prog_tol[q] : schema->d_prog[q], a.rec_size, ctx->d_irr,
        &ctx->d_res->n_irregular, s,
        tol ? jit_kernels(schema->prog_tol[q], schema->device, JIT_DECODE, a.n, 0, false)
            : schema_jit(schema, protocol, JIT_DECODE, a.n, 0));
    if (e == hipSuccess)
      e = launch_general_decode_list(a, protocol, ctx->d_irr, &ctx->d_res->n_irregular, s);
    return e;
  }
  return launch_general_decode(a, protocol, s);
}

// Fewest wire bytes a record of the program can take (every value at its
// shortest: 1-byte varints, empty strings and lists).
uint32_t prog_min_len(const VProgram& P) {
  const bool compact = P.protocol != TGPU_PROTOCOL_BINARY;
  uint32_t n = 0;
  for (uint32_t k = 0; k < P.n_ops; ++k) {
    const VOp& o = P.ops[k];
    switch (o.kind) {
      case VOP_CONST: n += o.hdr_len; break;
      case VOP_CBOOL: n += compact && o.hdr_len == 0 ? 0 : o.hdr_len; break;
      case VOP_FIXED: n += o.width; break;
      case VOP_VARINT: n += 1; break;
      case VOP_STRING: n += compact ? 1 : 4; break;
      case VOP_LIST: n += compact ? 1 : 5; break;
      // nested programs: a header of each present field (an optional one
      // may be absent: its value ops skipped), containers empty, STOPs
      case VOP_FHDR:
        if (o.width) k += o.bits;
        else n += compact ? 1 : 3;
        break;
      case VOP_SEQ: case VOP_MSEQ:
        n += compact ? 1 : (o.kind == VOP_SEQ ? 5 : 6);
        if (o.hdr_len > k + 1) k = o.hdr_len - 1u;  // past the body
        break;
      case VOP_SEND: n += 1; break;
      default: break;
    }
  }
  return n;
}

// The nested program's index kernels (JIT_NINDEX) for an unindexed stream
// of `bytes` (nullptr: none — the general reader measures the records).
const JitKernels* nested_index_jit(const tgpu_schema* schema, int protocol, uint64_t bytes,
                                   int32_t height, int32_t max_depth) {
  const char* v = getenv("TGPU_NESTED");
  if (v && v[0] == '0') return nullptr;
  const int q = prog_protocol(schema, protocol);
  if (q < 0 || !schema->has_nprog[q] || !schema->d_nprog[q] || !bytes) return nullptr;
  const int32_t need = (int32_t)schema->nprog_depth[q] + 1;
  if (height < need || max_depth < need) return nullptr;
  return jit_kernels(schema->nprog[q], schema->device, JIT_NINDEX, 0, bytes, false);
}

// TGPU_INDEX_STARTS=0: the emit pass re-walks every tile instead of copying
// the speculation pass's stored starts, and unindexed decodes take the fused
// index + decode tiles (A/B).
bool index_starts_enabled() {
  const char* e = getenv("TGPU_INDEX_STARTS");
  return !(e && e[0] == '0');
}

// Stream index into offs (max_records + 1 entries); see launch_index_stream.
// Returns a TGPU_ERR_* for host-side failures; HIP launch errors go to `e`.
// dec (optional): decode the records during the index when the tile path
// allows it (*fused set); records [0, dec->n) into dec->recs / dec->arena,
// leftovers to ctx->d_irr for the general decoder.
int launch_index(tgpu_context* ctx, const tgpu_schema* schema, int protocol, const uint8_t* in,
                 uint64_t in_len, uint64_t begin, uint64_t end, int speculative, uint64_t* offs,
                 uint64_t max_records, uint64_t fill_to, const tgpu_limits* limits,
                 hipStream_t s, hipError_t& e, const DecodeArgs* dec = nullptr,
                 bool* fused = nullptr, bool tolerant = false, bool may_sync = false) {
  if (fused) *fused = false;
  tolerant = tolerant || tails_everywhere();
  IndexArgs x{};
  x.sc = dev_schema(schema, protocol);
  x.in = in;
  x.in_len = in_len;
  x.begin = begin;
  x.end = end;
  x.speculative = speculative;
  x.protocol = protocol;
  // record stride of the fused decode (schemas with a program) / scratch
  // stride of the measuring reads
  x.rec_size = schema->nested ? (uint32_t)measure_scratch(schema) : schema->structs[0].size;
  x.string_limit = limits ? limits->string_limit : 0;
  x.container_limit = limits ? limits->container_limit : 0;
  x.max_depth = limits ? limits->max_depth : 12000;
  x.height = limits ? limits->height : 0;
  const int32_t height = x.height ? x.height : x.max_depth;
  const int pq = prog_protocol(schema, protocol);
  x.prog = has_prog(schema, protocol) && height >= 2 && x.max_depth >= 2
               ? (tolerant ? schema->d_prog_tol[pq] : schema->d_prog[pq]) : nullptr;
  // no record program: the nested program's measuring walk when compiled
  // (index only — the nested decode runs after it, never a fused decode)
  const JitKernels* njit =
      x.prog ? nullptr : nested_index_jit(schema, protocol, end > begin ? end - begin : 0, height,
                                          x.max_depth);
  if (njit) {
    x.prog = schema->d_nprog[pq];
    dec = nullptr;
  }
  const char* hm = getenv("TGPU_INDEX_HMASK");  // "0": no first-byte filter (A/B, tests)
  if (x.prog || (hm && hm[0] == '0')) {
    for (uint32_t& w : x.hmask) w = ~0u;
  } else {
    record_first_bytes(*schema, protocol, x.hmask);
  }
  // program-less speculation runs the general reader from every candidate:
  // when the call says how many records it expects (a decode of n records),
  // chunks and the speculated chains' reach follow the mean record length —
  // a false candidate's chain costs its reach, and more, shorter chunks keep
  // more lanes busy (1 Mi-record adversarial V1 stream, first-byte filter
  // off: 5.5 s with 4 KiB chunks and a 256 KiB reach, 78 ms with 1 KiB and
  // 256 B). Otherwise a 256 KiB reach.
  const uint64_t span = end > begin ? end - begin : 0;
  const uint64_t mean = !x.prog && dec && dec->n && dec->n < span ? span / dec->n : 0;
  x.chunk = index_chunk_bytes(span, x.prog != nullptr, mean);
  x.window = (uint32_t)std::min<uint64_t>(x.chunk, 1024);
  x.spec_reach = mean ? (uint32_t)std::min<uint64_t>(std::max<uint64_t>(4 * mean, 256), 256u * 1024)
                      : 256u * 1024;
  if (const char* v = getenv("TGPU_INDEX_SPEC_REACH")) x.spec_reach = (uint32_t)atoi(v);
  x.x_reach = 4096;
  if (const char* v = getenv("TGPU_INDEX_XREACH"))
    x.x_reach = std::min<uint32_t>((uint32_t)atoi(v), 4096);
  x.n_chunks = end > begin ? (end - begin + x.chunk - 1) / x.chunk : 0;
  x.offs = offs;
  x.max_records = max_records;
  x.fill_to = fill_to;
  x.res = ctx->d_res;
  x.deep = deep_args(ctx);
  if (dec) {
    x.recs = dec->recs;
    x.arena = dec->arena;
    x.arena_cap = dec->arena_cap;
    x.n_decode = dec->n;
    x.irr = ctx->d_irr;
    x.nirr = &ctx->d_res->n_irregular;
    x.decode_tail = fill_to > 0;
  }
  const uint64_t C = std::max<uint64_t>(x.n_chunks, 1);
  const uint64_t rs = (x.rec_size + 7) & ~7u;
  const uint64_t parts = scan_tiles_parts(C) + 1;
  const uint64_t lane_words = x.chunk == index_tile_bytes() ? C * index_tile_lanes() : 0;
  // stored starts: a tile holds at most chunk / min_len + 1 record starts
  const bool starts = lane_words && x.prog && index_starts_enabled();
  // (x.prog set: pq >= 0 — a Compact V1 stream of a schema with doubles has
  // no program, and prog[-1] was read here)
  const uint32_t min_len =
      starts && pq >= 0 ? prog_min_len(njit ? schema->nprog[pq] : schema->prog[pq]) : 1u;
  x.st_cap = starts ? (uint32_t)std::min<uint64_t>(x.chunk / std::max<uint32_t>(min_len, 1) + 2,
                                                   2048)
                    : 0;
  const uint64_t st_bytes = (2 * (uint64_t)x.st_cap * C + 15) & ~15ull;
  const uint64_t need =
      8 * ((9 + kSpecStarts) * C + parts + 25) + C * rs + 4 * lane_words + 16 + st_bytes;
  if (need > ctx->index_bytes) {
    if (ctx->d_index) (void)hipFree(ctx->d_index);
    ctx->d_index = nullptr;
    ctx->index_bytes = 0;
    if (hipMalloc(&ctx->d_index, need) != hipSuccess) return TGPU_ERR_HIP;
    ctx->index_bytes = need;
  }
  uint64_t* w = (uint64_t*)ctx->d_index;
  x.s = w;
  x.e = w + C;
  x.cnt = (unsigned long long*)(w + 2 * C);
  x.base = (unsigned long long*)(w + 3 * C);
  x.bad = (unsigned long long*)(w + 4 * C);
  x.pf = w + 5 * C;
  x.ep = w + 6 * C;
  x.ec = (unsigned long long*)(w + 7 * C);
  x.part = (unsigned long long*)(w + 8 * C);
  x.scal = (unsigned long long*)(w + 8 * C + parts);
  x.scratch = (uint8_t*)(w + 8 * C + parts + 24);  // (scal: 24 words)
  x.lanes = (uint32_t*)(x.scratch + C * rs);
  x.deep_chunks = (uint64_t*)(x.lanes + lane_words + (lane_words & 1));
  x.sst = x.deep_chunks + C;
  x.st16 = starts ? (uint16_t*)(((uintptr_t)(x.sst + kSpecStarts * C) + 15) & ~(uintptr_t)15) : nullptr;
  // decode: the indexed program decode after the index (balanced: 256 records
  // per workgroup) instead of the emit tiles' per-lane chains
  x.st_decode = starts && dec && x.recs ? 1 : 0;
  if (x.n_chunks == 0) {
    // nothing starts in [begin, end): the index is just the end position
    if (e == hipSuccess) e = launch_index_empty(x.res, offs, x.begin, fill_to, s);
    return TGPU_OK;
  }
  const JitKernels* jit =
      njit ? njit
      : !x.prog ? nullptr
      : tolerant ? jit_kernels(schema->prog_tol[pq], schema->device, JIT_INDEX, 0, end - begin,
                               false)
                 : schema_jit(schema, protocol, JIT_INDEX, 0, end - begin);
  ctx->last_scal = x.scal;  // (tgpu_index_stats: this call's counters, either path)
  ctx->last_chunks = x.n_chunks;
  const bool rr1 = x.recs && x.st_decode && jit && jit_has(jit, 5) && !tolerant &&
                   onepass_rr_enabled();
  if (e == hipSuccess && may_sync && x.prog && !njit && x.chunk == index_tile_bytes() &&
      (onepass_enabled() || rr1)) {
    // single pass with look-back; a range it cannot finish alone (a record
    // off the program, a record longer than a tile, ...) goes to the two-pass
    // index below, which redoes it whole
    e = launch_index_onepass(x, s, jit, rr1 && !onepass_enabled());
    uint64_t sc[12] = {1};
    if (e == hipSuccess) e = hipMemcpyAsync(sc, x.scal, sizeof(sc), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    const uint64_t failed = sc[7];
    if (getenv("TGPU_ONEPASS_STATS"))  // counters with TGPU_JIT_DEFINES="#define TGPU_ONEPASS_STATS"
      fprintf(stderr, "tgpu onepass: tiles %llu failed %llu windows %llu restarts %llu repairs %llu "
              "failed tiles %llu\n", (unsigned long long)x.n_chunks, (unsigned long long)sc[7],
              (unsigned long long)sc[8], (unsigned long long)sc[9], (unsigned long long)sc[10],
              (unsigned long long)sc[11]);
    if (e == hipSuccess && !failed) {
      e = launch_index_finish(x, x.recs != nullptr, s);
      if (fused) *fused = x.recs != nullptr;
      return TGPU_OK;
    }
    if (e == hipSuccess && x.nirr) e = hipMemsetAsync(x.nirr, 0, sizeof(unsigned long long), s);
  }
  // TGPU_INDEX_TIMING=1: HIP events around the index and the decode (stderr)
  static const bool timing = getenv("TGPU_INDEX_TIMING") != nullptr;
  hipEvent_t tev[3] = {};
  if (timing)
    for (auto& v : tev) (void)hipEventCreate(&v);
  if (timing) (void)hipEventRecord(tev[0], s);
  // blocking calls let the index read its tile summary and total mid-call
  // (skipping the general-reader helper kernels when no tile needs them)
  uint64_t* h_sync = may_sync ? ctx->h_words : nullptr;
  if (h_sync) h_sync[3] = ~0ull;
  ctx->last_scal = x.scal;
  ctx->last_chunks = x.n_chunks;
  // (grow-only; a failed allocation leaves the verification walk to it)
  const XTabAlloc xalloc{ctx, [](void* u, uint64_t bytes) -> uint8_t* {
                           tgpu_context* c = static_cast<tgpu_context*>(u);
                           if (bytes <= c->xtab_bytes) return c->d_xtab;
                           if (c->d_xtab) (void)hipFree(c->d_xtab);
                           c->d_xtab = nullptr;
                           c->xtab_bytes = 0;
                           if (hipMalloc(&c->d_xtab, bytes) != hipSuccess) {
                             (void)hipGetLastError();
                             return nullptr;
                           }
                           c->xtab_bytes = bytes;
                           return c->d_xtab;
                         }};
  if (e == hipSuccess) e = launch_index_stream(x, s, jit, fused, h_sync, &xalloc);
  if (timing) (void)hipEventRecord(tev[1], s);
  struct TimingReport {
    hipEvent_t* ev;
    bool on;
    hipStream_t st;
    ~TimingReport() {
      if (!on) return;
      (void)hipEventRecord(ev[2], st);
      (void)hipEventSynchronize(ev[2]);
      float a = 0, b = 0;
      (void)hipEventElapsedTime(&a, ev[0], ev[1]);
      (void)hipEventElapsedTime(&b, ev[1], ev[2]);
      fprintf(stderr, "tgpu index %.3f ms, then %.3f ms\n", a, b);
      for (int k = 0; k < 3; ++k) (void)hipEventDestroy(ev[k]);
    }
  } report{tev, timing, s};
  if (e == hipSuccess && x.st_decode && x.chunk == index_tile_bytes()) {
    // the records the index found, [0, min(total, n_decode)): program decode,
    // the rest to the general decoder's list (as the fused tiles leave them)
    DecodeArgs t = *dec;
    t.offs = offs;
    t.n_dev = x.scal + 5;
    t.fixed_len = 0;
    if (may_sync) {
      // the record count sizes the decode's LDS wire tile (its mean record);
      // otherwise the caller's max_records bounds it (an overestimate makes
      // the cap too small: those tiles' records take the general decoder)
      // (into the context's pinned result slot: a pageable destination costs
      // a staged copy; the slot is rewritten by every later result read)
      if (h_sync[3] == ~0ull) {  // (the index did not read it)
        e = hipMemcpyAsync(&h_sync[3], x.scal + 5, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return TGPU_OK;
      }
      const uint64_t total = h_sync[3];
      t.n = std::min<uint64_t>(t.n, total);
    }
    e = launch_program_decode(
        t, x.prog, t.rec_size, ctx->d_irr, &ctx->d_res->n_irregular, s,
        tolerant ? jit_kernels(schema->prog_tol[pq], schema->device, JIT_DECODE, t.n, 0, false)
                 : schema_jit(schema, protocol, JIT_DECODE, t.n, 0),
        end - begin);
    if (fused) *fused = true;
  }
  return TGPU_OK;
}

// Blocking decode of a fixed-layout stream after the plan kernel: waits for
// its verdict. Every record canonical: the batch is done (returns 0; the
// finish kernel still records the result for tgpu_context_wait). Otherwise
// the records from the first non-canonical one on are read the way an
// unindexed stream is — parallel speculative index from its byte position
// i * L (the bytes before it are i canonical records), the records decoded
// with it (compiled program, general decoder for the rest) — and the status
// is left on the device (returns 1). -1: the caller's serial fallback
// (no program for the index); a HIP error goes to `e` (returns 0).
// first: the batch's first record not at its stride position when already
// known (the record-0 probe), else read from the device result.
int fixed_tail(tgpu_context* ctx, const tgpu_schema* schema, int protocol, const DecodeArgs& a,
               uint64_t L, const tgpu_limits* limits, hipStream_t s, hipError_t& e,
               uint64_t first = ~0ull, bool tolerant = false) {
  uint64_t irr = first;
  if (first == ~0ull) {
    if (e == hipSuccess)
      e = hipMemcpyAsync(ctx->h_res, ctx->d_res, sizeof(DevResult), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return 0;
    irr = ctx->h_res->first_irregular;
  }
  if (irr >= a.n) {
    e = launch_decode_finish(a, protocol, L, s);
    return 0;
  }
  DecodeArgs t = a;
  t.recs = a.recs + irr * a.rec_size;
  t.n = a.n - irr;
  t.offs = ctx->d_offs + irr;
  t.check_index = 1;
  bool fused = false;
  // a stream off the stride from record 0 on (the probe): most likely every
  // record carries appended fields, which the tolerant programs take
  const int rc = launch_index(ctx, schema, protocol, a.in, a.in_len, irr * L, a.in_len, 0,
                              ctx->d_offs + irr, t.n, t.n, limits, s, e, &t, &fused,
                              first == 0 || tolerant, true);
  if (rc) {
    e = hipErrorOutOfMemory;
    return 0;
  }
  if (e == hipSuccess && fused)
    e = launch_general_decode_list(t, protocol, ctx->d_irr, &ctx->d_res->n_irregular, s);
  else if (e == hipSuccess)
    e = launch_indexed_decode(ctx, schema, protocol, t, s);
  if (e == hipSuccess) e = launch_tail_decode_finish(t, protocol, irr, s);
  return 1;
}

}  // namespace

extern "C" {

int tgpu_abi_version(void) { return TGPU_ABI_VERSION; }

const char* tgpu_code_name(int code) {
  switch (code) {
    case TGPU_OK: return "OK";
    case TGPU_ERR_UNDERFLOW: return "UNDERFLOW";
    case TGPU_ERR_INVALID_VARINT: return "INVALID_VARINT";
    case TGPU_ERR_BOOL_VALUE: return "BOOL_VALUE";
    case TGPU_ERR_INVALID_SKIP_TYPE: return "INVALID_SKIP_TYPE";
    case TGPU_ERR_TRUNCATED: return "TRUNCATED";
    case TGPU_ERR_NEGATIVE_SIZE: return "NEGATIVE_SIZE";
    case TGPU_ERR_SIZE_LIMIT: return "SIZE_LIMIT";
    case TGPU_ERR_DEPTH_LIMIT: return "DEPTH_LIMIT";
    case TGPU_ERR_BAD_TYPE: return "BAD_TYPE";
    case TGPU_ERR_INVALID_BOOL_WRITE: return "INVALID_BOOL_WRITE";
    case TGPU_ERR_WRITE_SIZE_LIMIT: return "WRITE_SIZE_LIMIT";
    case TGPU_ERR_UNION_MISSING_STOP: return "UNION_MISSING_STOP";
    case TGPU_ERR_MISSING_REQUIRED_FIELD: return "MISSING_REQUIRED_FIELD";
    case TGPU_ERR_INDEX_MISMATCH: return "INDEX_MISMATCH";
    case TGPU_ERR_OUTPUT_OVERFLOW: return "OUTPUT_OVERFLOW";
    case TGPU_ERR_UNSUPPORTED: return "UNSUPPORTED";
    case TGPU_ERR_INVALID_ARGUMENT: return "INVALID_ARGUMENT";
    case TGPU_ERR_HIP: return "HIP";
    default: return "UNKNOWN";
  }
}

void tgpu_code_classify(int code, int32_t* exc_class, int32_t* tproto_type) {
  classify(code, exc_class, tproto_type);
}

int tgpu_layout_compute(tgpu_struct_desc* structs, uint32_t n_structs, tgpu_field_desc* fields,
                        uint32_t n_fields) {
  if (!structs || n_structs == 0 || (!fields && n_fields)) return TGPU_ERR_INVALID_ARGUMENT;
  std::vector<int> state(n_structs, 0);
  for (uint32_t si = 0; si < n_structs; ++si) {
    const int rc = layout_struct(structs, n_structs, fields, n_fields, si, state);
    if (rc) return rc;
  }
  return TGPU_OK;
}

int tgpu_schema_create(const tgpu_struct_desc* structs, uint32_t n_structs,
                       const tgpu_field_desc* fields, uint32_t n_fields, tgpu_schema** out) {
  return tgpu_schema_create_ex(structs, n_structs, fields, n_fields, nullptr, 0, out);
}

int tgpu_schema_create_ex(const tgpu_struct_desc* structs, uint32_t n_structs,
                          const tgpu_field_desc* fields, uint32_t n_fields,
                          const tgpu_type_desc* types, uint32_t n_types, tgpu_schema** out) {
  if (!out || !structs || n_structs == 0 || (!fields && n_fields) || (!types && n_types))
    return TGPU_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  SchemaFacts facts;
  int rc = validate(structs, n_structs, fields, n_fields, types, n_types, facts);
  if (rc) return rc;
  auto* s = new (std::nothrow) tgpu_schema();
  if (!s) return TGPU_ERR_HIP;
  s->structs.assign(structs, structs + n_structs);
  s->fields.assign(fields, fields + n_fields);
  if (n_types) s->types.assign(types, types + n_types);
  s->has_lists = facts.has_lists;
  s->nested = facts.nested;
  if (s->nested) {
    uint32_t slot_b = 0, slot_c = 0;
    region_scale(*s, false, s->region_scale[0], slot_b);
    region_scale(*s, true, s->region_scale[1], slot_c);
    s->nest_slot = std::max(slot_b, slot_c);
  }
  // element / value types anywhere: fields' and nested types'
  auto note = [&](uint32_t ttype, uint32_t elem, uint32_t val) {
    const bool container = ttype == TGPU_T_LIST || ttype == TGPU_T_SET || ttype == TGPU_T_MAP;
    const bool se = container && (elem == TGPU_T_STRING ||
                                  (ttype == TGPU_T_MAP && val == TGPU_T_STRING));
    s->str_elems |= se;
    s->has_strings |= ttype == TGPU_T_STRING || se;
    s->has_double |= ttype == TGPU_T_DOUBLE || (container && elem == TGPU_T_DOUBLE) ||
                     (ttype == TGPU_T_MAP && val == TGPU_T_DOUBLE);
  };
  for (uint32_t k = 0; k < n_fields; ++k) note(fields[k].ttype, fields[k].elem_ttype, fields[k].val_ttype);
  for (uint32_t k = 0; k < n_types; ++k) note(types[k].ttype, types[k].elem_ttype, types[k].val_ttype);
  // the block rule (ArenaPack): flat-list schemas only
  if (!s->nested && !s->str_elems && s->has_lists && !block_pack_slots(*s, 0, 0, s->pack, 0))
    s->pack.n = 0;
  if (n_types && (hipMalloc(&s->d_types, sizeof(tgpu_type_desc) * n_types) != hipSuccess ||
                  hipMemcpy(s->d_types, types, sizeof(tgpu_type_desc) * n_types,
                            hipMemcpyHostToDevice) != hipSuccess)) {
    tgpu_schema_destroy(s);
    return TGPU_ERR_HIP;
  }
  (void)hipGetDevice(&s->device);
  if (hipMalloc(&s->d_structs, sizeof(tgpu_struct_desc) * n_structs) != hipSuccess ||
      hipMalloc(&s->d_fields, sizeof(tgpu_field_desc) * std::max(n_fields, 1u)) != hipSuccess) {
    tgpu_schema_destroy(s);
    return TGPU_ERR_HIP;
  }
  if (hipMemcpy(s->d_structs, structs, sizeof(tgpu_struct_desc) * n_structs,
                hipMemcpyHostToDevice) != hipSuccess ||
      (n_fields && hipMemcpy(s->d_fields, fields, sizeof(tgpu_field_desc) * n_fields,
                             hipMemcpyHostToDevice) != hipSuccess)) {
    tgpu_schema_destroy(s);
    return TGPU_ERR_HIP;
  }
  s->recursive = schema_recursive(*s);
  // program slots: Binary, Compact, and CompactV1's (kV1Slot) for a schema
  // with doubles (without, CompactV1 runs Compact's)
  for (int proto : {(int)TGPU_PROTOCOL_BINARY, (int)TGPU_PROTOCOL_COMPACT, kV1Slot}) {
    if (proto == kV1Slot && !s->has_double) continue;
    const bool flat = build_program(*s, proto, s->prog[proto]);
    // the nested program: schemas with containers of structs / containers,
    // and schemas with no canonical record program (optional fields)
    if (s->nested || !flat)
      s->has_nprog[proto] = build_nested_program(*s, proto, s->nprog[proto], s->nprog_depth[proto],
                                                 &s->nprog_defer[proto]);
    if (s->has_nprog[proto] &&
        (hipMalloc(&s->d_nprog[proto], sizeof(VProgram)) != hipSuccess ||
         hipMemcpy(s->d_nprog[proto], &s->nprog[proto], sizeof(VProgram), hipMemcpyHostToDevice) !=
             hipSuccess)) {
      tgpu_schema_destroy(s);
      return TGPU_ERR_HIP;
    }
    if (!flat) continue;
    build_program(*s, proto, s->prog_tol[proto], true);
    if (hipMalloc(&s->d_prog[proto], sizeof(VProgram)) != hipSuccess ||
        hipMemcpy(s->d_prog[proto], &s->prog[proto], sizeof(VProgram), hipMemcpyHostToDevice) !=
            hipSuccess ||
        hipMalloc(&s->d_prog_tol[proto], sizeof(VProgram)) != hipSuccess ||
        hipMemcpy(s->d_prog_tol[proto], &s->prog_tol[proto], sizeof(VProgram),
                  hipMemcpyHostToDevice) != hipSuccess) {
      tgpu_schema_destroy(s);
      return TGPU_ERR_HIP;
    }
    s->has_prog[proto] = true;
  }
  FixedTemplate t{};
  uint32_t wire = 0;
  if (build_template(*s, 0, 0, t, wire) && wire <= kMaxFixedWire &&
      s->structs[0].size <= kMaxFixedRecord) {
    t.wire_len = wire;
    t.record_size = s->structs[0].size;
    s->tmpl = t;
    if (hipMalloc(&s->d_tmpl, sizeof(FixedTemplate)) != hipSuccess ||
        hipMemcpy(s->d_tmpl, &t, sizeof(FixedTemplate), hipMemcpyHostToDevice) != hipSuccess) {
      tgpu_schema_destroy(s);
      return TGPU_ERR_HIP;
    }
    s->fixed_binary = true;
    if (build_plan(t, s->plan)) {
      if (hipMalloc(&s->d_plan, sizeof(FixedPlan)) != hipSuccess ||
          hipMemcpy(s->d_plan, &s->plan, sizeof(FixedPlan), hipMemcpyHostToDevice) != hipSuccess) {
        tgpu_schema_destroy(s);
        return TGPU_ERR_HIP;
      }
      s->has_plan = true;
    }
  }
  *out = s;
  return TGPU_OK;
}

void tgpu_schema_destroy(tgpu_schema* s) {
  if (!s) return;
  if (s->d_structs) (void)hipFree(s->d_structs);
  if (s->d_fields) (void)hipFree(s->d_fields);
  if (s->d_types) (void)hipFree(s->d_types);
  if (s->d_tmpl) (void)hipFree(s->d_tmpl);
  if (s->d_plan) (void)hipFree(s->d_plan);
  for (VProgram* p : s->d_prog)
    if (p) (void)hipFree(p);
  for (VProgram* p : s->d_prog_tol)
    if (p) (void)hipFree(p);
  for (VProgram* p : s->d_nprog)
    if (p) (void)hipFree(p);
  delete s;
}

uint32_t tgpu_schema_record_size(const tgpu_schema* s) { return s ? s->structs[0].size : 0; }

int tgpu_schema_compile(const tgpu_schema* s, int protocol) {
  if (!s || !valid_protocol(protocol))
    return TGPU_ERR_INVALID_ARGUMENT;
  const int q = prog_protocol(s, protocol);
  if (q >= 0 && s->has_nprog[q])
    return jit_kernels(s->nprog[q], s->device, JIT_NESTED, 0, 0, true) ? TGPU_OK
                                                                       : TGPU_ERR_UNSUPPORTED;
  if (!has_prog(s, protocol)) return TGPU_ERR_UNSUPPORTED;
  for (int group : {JIT_DECODE, JIT_ENCODE, JIT_INDEX})
    if (!jit_kernels(s->prog[q], s->device, group, 0, 0, true)) return TGPU_ERR_UNSUPPORTED;
  return TGPU_OK;
}

int tgpu_schema_compile_check_ex(const tgpu_struct_desc* structs, uint32_t n_structs,
                                 const tgpu_field_desc* fields, uint32_t n_fields,
                                 const tgpu_type_desc* types, uint32_t n_types, int protocol,
                                 const char* arch, char* log, uint64_t log_capacity) {
  if (!structs || n_structs == 0 || (!fields && n_fields) || (!types && n_types) ||
      !valid_protocol(protocol))
    return TGPU_ERR_INVALID_ARGUMENT;
  SchemaFacts facts;
  const int rc = validate(structs, n_structs, fields, n_fields, types, n_types, facts);
  if (rc) return rc;
  tgpu_schema h;  // host tables only: nothing is uploaded
  h.structs.assign(structs, structs + n_structs);
  h.fields.assign(fields, fields + n_fields);
  if (n_types) h.types.assign(types, types + n_types);
  h.nested = facts.nested;
  for (uint32_t k = 0; k < n_fields; ++k)
    h.has_double |= fields[k].ttype == TGPU_T_DOUBLE || fields[k].elem_ttype == TGPU_T_DOUBLE ||
                    fields[k].val_ttype == TGPU_T_DOUBLE;
  for (uint32_t k = 0; k < n_types; ++k)
    h.has_double |= types[k].elem_ttype == TGPU_T_DOUBLE || types[k].val_ttype == TGPU_T_DOUBLE;
  const int q = prog_protocol(&h, protocol);
  VProgram P{};
  uint32_t depth = 0;
  // nested schemas: the nested program (JIT_NESTED); others: the canonical
  // record program's three groups
  if (q < 0) return TGPU_ERR_UNSUPPORTED;
  if (h.nested || !build_program(h, q, P)) {
    if (!build_nested_program(h, q, P, depth)) return TGPU_ERR_UNSUPPORTED;
    return jit_compile_check(P, arch, log, log_capacity);
  }
  const int rc2 = jit_compile_check(P, arch, log, log_capacity);
  // the tolerant variant's decode group (with the strided tail decode)
  VProgram T{};
  if (rc2 || !build_program(h, q, T, true)) return rc2;
  return jit_compile_check(T, arch, log, log_capacity, JIT_DECODE);
}

int tgpu_transcode_compile_check(const tgpu_struct_desc* structs, uint32_t n_structs,
                                 const tgpu_field_desc* fields, uint32_t n_fields,
                                 int from_protocol, int to_protocol, const char* arch, char* log,
                                 uint64_t log_capacity) {
  if (!structs || n_structs == 0 || (!fields && n_fields) || !valid_protocol(from_protocol) ||
      !valid_protocol(to_protocol))
    return TGPU_ERR_INVALID_ARGUMENT;
  SchemaFacts facts;
  const int rc = validate(structs, n_structs, fields, n_fields, nullptr, 0, facts);
  if (rc) return rc;
  tgpu_schema h;
  h.structs.assign(structs, structs + n_structs);
  h.fields.assign(fields, fields + n_fields);
  h.nested = facts.nested;
  for (uint32_t k = 0; k < n_fields; ++k)
    h.has_double |= fields[k].ttype == TGPU_T_DOUBLE || fields[k].elem_ttype == TGPU_T_DOUBLE ||
                    fields[k].val_ttype == TGPU_T_DOUBLE;
  const int qf = prog_protocol(&h, from_protocol), qt = prog_protocol(&h, to_protocol);
  VProgram Ps{}, Pd{};
  if (qf < 0 || qt < 0 || h.nested || !build_program(h, qf, Ps) || !build_program(h, qt, Pd))
    return TGPU_ERR_UNSUPPORTED;
  return jit_compile_check_xcode(Ps, Pd, arch, log, log_capacity);
}

int tgpu_schema_compile_check(const tgpu_struct_desc* structs, uint32_t n_structs,
                              const tgpu_field_desc* fields, uint32_t n_fields, int protocol,
                              const char* arch, char* log, uint64_t log_capacity) {
  for (uint32_t k = 0; fields && k < n_fields; ++k)
    if (fields[k].type_index) return TGPU_ERR_UNSUPPORTED;  // (needs the type table: _ex)
  return tgpu_schema_compile_check_ex(structs, n_structs, fields, n_fields, nullptr, 0, protocol,
                                      arch, log, log_capacity);
}

uint32_t tgpu_schema_arena_scale(const tgpu_schema* s, int protocol) {
  if (!s || !s->has_lists || !valid_protocol(protocol)) return 0;
  const bool bin = protocol == TGPU_PROTOCOL_BINARY;
  if (s->nested) return s->region_scale[bin ? 0 : 1];
  return s->str_elems ? (bin ? 4 : 16) : (bin ? 1 : 8);
}

uint64_t tgpu_schema_fixed_wire_size(const tgpu_schema* s, int protocol) {
  return (s && protocol == TGPU_PROTOCOL_BINARY && s->fixed_binary) ? s->tmpl.wire_len : 0;
}

int tgpu_context_create(tgpu_context** out) {
  if (!out) return TGPU_ERR_INVALID_ARGUMENT;
  auto* c = new (std::nothrow) tgpu_context();
  if (!c) return TGPU_ERR_HIP;
  (void)hipGetDevice(&c->device);
  if (hipMalloc(&c->d_res, sizeof(DevResult)) != hipSuccess ||
      hipHostMalloc(&c->h_res, sizeof(DevResult), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&c->h_words, 8 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess) {
    tgpu_context_destroy(c);
    return TGPU_ERR_HIP;
  }
  *out = c;
  return TGPU_OK;
}

void tgpu_context_destroy(tgpu_context* c) {
  if (!c) return;
  if (c->host_pipe) host_pipe_destroy(c->host_pipe);
  if (c->d_res) (void)hipFree(c->d_res);
  if (c->h_res) (void)hipHostFree(c->h_res);
  if (c->h_words) (void)hipHostFree(c->h_words);
  if (c->d_offs) (void)hipFree(c->d_offs);
  if (c->d_pack_flags) (void)hipFree(c->d_pack_flags);
  if (c->d_block_sums) (void)hipFree(c->d_block_sums);
  if (c->d_scan_part) (void)hipFree(c->d_scan_part);
  if (c->d_irr) (void)hipFree(c->d_irr);
  if (c->d_deep) (void)hipFree(c->d_deep);
  if (c->d_slabs) (void)hipFree(c->d_slabs);
  if (c->d_wslabs) (void)hipFree(c->d_wslabs);
  if (c->d_deep2) (void)hipFree(c->d_deep2);
  if (c->d_index) (void)hipFree(c->d_index);
  if (c->d_xrec) (void)hipFree(c->d_xrec);
  if (c->d_xarena) (void)hipFree(c->d_xarena);
  if (c->d_xoffs) (void)hipFree(c->d_xoffs);
  if (c->d_xtab) (void)hipFree(c->d_xtab);
  if (c->d_xstat) (void)hipFree(c->d_xstat);
  delete c;
}

int tgpu_context_reserve(tgpu_context* ctx, uint64_t n) {
  if (!ctx) return TGPU_ERR_INVALID_ARGUMENT;
  return ensure_workspace(ctx, n);
}

int tgpu_context_wait(tgpu_context* ctx, void* stream, tgpu_status* st, uint64_t* n_done,
                      uint64_t* bytes) {
  if (!ctx) return TGPU_ERR_INVALID_ARGUMENT;
  const hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemcpyAsync(ctx->h_res, ctx->d_res, sizeof(DevResult),
                                hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  const DevResult& r = *ctx->h_res;
  const int code = r.code;
  fill_status(st, code, code ? r.first_fail : r.n_records, code ? r.fail_offset : 0);
  if (n_done) *n_done = r.n_records;
  if (bytes) *bytes = r.total_bytes;
  return code;
}

int tgpu_index_stats(tgpu_context* ctx, void* stream, uint64_t* out) {
  if (!ctx || !out) return TGPU_ERR_INVALID_ARGUMENT;
  hipError_t e = hipMemcpyAsync(ctx->h_res, ctx->d_res, sizeof(DevResult), hipMemcpyDeviceToHost,
                                (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) return TGPU_ERR_HIP;
  out[TGPU_ISTAT_GENERAL] = ctx->h_res->n_irregular;
  if (!ctx->last_scal) return TGPU_ERR_INVALID_ARGUMENT;
  uint64_t sc[11] = {};
  e = hipMemcpyAsync(sc, ctx->last_scal, sizeof(sc), hipMemcpyDeviceToHost, (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) return TGPU_ERR_HIP;
  out[TGPU_ISTAT_CHUNKS] = ctx->last_chunks;
  out[TGPU_ISTAT_PARTIAL] = sc[8];
  out[TGPU_ISTAT_NO_START] = sc[9];
  out[TGPU_ISTAT_BROKEN] = sc[10];
  out[TGPU_ISTAT_REPAIRED] = sc[0];
  out[TGPU_ISTAT_REWALKED] = sc[6];
  return TGPU_OK;
}

int tgpu_encode_batch(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                      const void* records, uint64_t n, const void* string_base,
                      const void* list_base, void* out, uint64_t out_capacity,
                      uint64_t* out_offsets, void* stream, tgpu_status* st, uint64_t* out_size) {
  if (!ctx || !schema || !valid_protocol(protocol) ||
      (n && (!records || !out))) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const hipStream_t s = (hipStream_t)stream;
  const uint32_t rs = schema->structs[0].size;
  if (((uintptr_t)records) % schema->structs[0].align ||
      (n && schema->has_lists && !list_base) || (n && schema->has_strings && !string_base)) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  (void)hipGetLastError();  // drop a stale error left by another library
  hipError_t e = launch_result_init(ctx->d_res, n, s);
  EncodeArgs a{};
  a.sc = dev_schema(schema, protocol);
  a.recs = (const uint8_t*)records;
  a.n = n;
  a.sbase = (const uint8_t*)string_base;
  a.lbase = (const uint8_t*)list_base;
  a.out = (uint8_t*)out;
  a.cap = out_capacity;
  a.rec_size = rs;
  a.res = ctx->d_res;
  uint64_t fixed = 0;
  if (protocol == TGPU_PROTOCOL_BINARY && schema->fixed_binary &&
      n * schema->tmpl.wire_len <= out_capacity) {
    fixed = schema->tmpl.wire_len;
    const JitKernels* fj = fixed_jit(schema, protocol, JIT_ENCODE, n);
    if (e == hipSuccess && fj) {
      EncodeArgs f = a;
      f.fixed_len = fixed;
      f.offs = out_offsets;
      e = launch_program_write_fixed(f, schema->d_prog[prog_protocol(schema, protocol)], s, fj);
    } else if (e == hipSuccess && schema->has_plan && ((uintptr_t)records & 7) == 0)
      e = launch_plan_binary_encode(&schema->plan, schema->d_plan, a.recs, n, a.out, out_offsets,
                                    ctx->d_res, s);
    else if (e == hipSuccess)
      e = launch_fixed_binary_encode(&schema->tmpl, schema->d_tmpl, a.recs, n, a.out,
                                     out_offsets, ctx->d_res, s);
  } else {
    const uint64_t nb = (n + 255) / 256;
    int rc = ensure_workspace(ctx, n);
    if (!rc) rc = ensure_deep(ctx, 12000, schema->recursive);
    if (rc) {
      fill_status(st, rc, 0, 0);
      return rc;
    }
    a.deep = deep_args(ctx);
    a.offs = out_offsets ? out_offsets : ctx->d_offs;
    a.block_sums = ctx->d_block_sums;
    a.scan_part = ctx->d_scan_part;
    a.out_cap = enc_out_cap(schema, protocol);
    if (e == hipSuccess && n) {
      if (has_prog(schema, protocol) && program_encode_fits(rs))
        e = launch_program_encode(a, schema->d_prog[prog_protocol(schema, protocol)], ctx->d_scan_part, false, s,
                                  schema_jit(schema, protocol, JIT_ENCODE, n, 0));
      else {  // (the writer has no depth limit: height / max_depth do not apply)
        const JitKernels* nj = nested_jit(schema, protocol, n, INT32_MAX, INT32_MAX);
        if (nj) a.out_cap = nested_out_cap(schema, protocol);
        e = launch_general_encode(a, protocol, nb, s, nj, nj && nested_defers(schema, protocol));
      }
    }
  }
  if (e == hipSuccess && n) e = launch_encode_finish(a, protocol, fixed, s);
  ctx->last_op = 2;
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  if (st || out_size) {
    tgpu_status tmp;
    uint64_t bytes = 0;
    const int rc = tgpu_context_wait(ctx, stream, st ? st : &tmp, nullptr, &bytes);
    if (out_size) *out_size = bytes;
    if (rc == TGPU_OK) learn_mean(schema, protocol, bytes, n);
    return rc;
  }
  return TGPU_OK;
}

int tgpu_encoded_size(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                      const void* records, uint64_t n, const void* list_base,
                      uint64_t* out_offsets, void* stream, tgpu_status* st, uint64_t* total) {
  if (!ctx || !schema || !out_offsets ||
      !valid_protocol(protocol) ||
      (n && !records) || ((uintptr_t)records) % schema->structs[0].align) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const hipStream_t s = (hipStream_t)stream;
  int rc = ensure_workspace(ctx, n);
  if (!rc) rc = ensure_deep(ctx, 12000, schema->recursive);
  if (rc) {
    fill_status(st, rc, 0, 0);
    return rc;
  }
  EncodeArgs a{};
  a.deep = deep_args(ctx);
  a.sc = dev_schema(schema, protocol);
  a.recs = (const uint8_t*)records;
  a.n = n;
  a.offs = out_offsets;
  a.block_sums = ctx->d_block_sums;
  a.scan_part = ctx->d_scan_part;
  a.rec_size = schema->structs[0].size;
  a.res = ctx->d_res;
  a.cap = ~0ull;
  a.lbase = (const uint8_t*)list_base;
  if (schema->has_lists && n && !list_base) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  (void)hipGetLastError();  // drop a stale error left by another library
  hipError_t e = launch_result_init(ctx->d_res, n, s);
  if (e == hipSuccess && n) {
    if (has_prog(schema, protocol) && program_encode_fits(a.rec_size)) {
      e = launch_program_encode(a, schema->d_prog[prog_protocol(schema, protocol)], ctx->d_scan_part, true, s,
                                schema_jit(schema, protocol, JIT_ENCODE, n, 0));
      if (e == hipSuccess) e = launch_size_offsets(a, (n + 255) / 256, s);
    } else {
      const JitKernels* nj = nested_jit(schema, protocol, n, INT32_MAX, INT32_MAX);
      e = launch_general_size(a, protocol, (n + 255) / 256, s, nj,
                              nj && nested_defers(schema, protocol));
    }
  }
  if (e == hipSuccess && n) e = launch_encode_finish(a, protocol, 0, s);
  if (e == hipSuccess && !n) e = hipMemsetAsync(out_offsets, 0, sizeof(uint64_t), s);
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  if (st || total) {
    tgpu_status tmp;
    uint64_t bytes = 0;
    const int rc = tgpu_context_wait(ctx, stream, st ? st : &tmp, nullptr, &bytes);
    if (total) *total = bytes;
    if (rc == TGPU_OK) learn_mean(schema, protocol, bytes, n);
    return rc;
  }
  return TGPU_OK;
}

int tgpu_decode_batch(tgpu_context* ctx, const tgpu_schema* schema, int protocol, const void* in,
                      uint64_t in_len, const uint64_t* offsets, uint64_t n, void* records,
                      void* list_arena, uint64_t list_arena_capacity, const tgpu_limits* limits,
                      void* stream, tgpu_status* st, uint64_t* n_decoded, uint64_t* consumed) {
  if (!ctx || !schema || !valid_protocol(protocol) ||
      (n && (!records || (!in && in_len)))) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  if (((uintptr_t)records) % schema->structs[0].align) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const hipStream_t s = (hipStream_t)stream;
  int rc = ensure_workspace(ctx, n);
  if (!rc) rc = ensure_deep(ctx, limit_depth(limits), schema->recursive);
  if (rc) {
    fill_status(st, rc, 0, 0);
    return rc;
  }
  DecodeArgs a{};
  a.sc = dev_schema(schema, protocol);
  a.in = (const uint8_t*)in;
  a.in_len = in_len;
  a.n = n;
  a.recs = (uint8_t*)records;
  a.arena = (uint8_t*)list_arena;
  a.arena_cap = list_arena_capacity;
  a.string_limit = limits ? limits->string_limit : 0;
  a.container_limit = limits ? limits->container_limit : 0;
  a.max_depth = limits ? limits->max_depth : 12000;
  a.height = limits ? limits->height : 0;
  a.rec_size = schema->structs[0].size;
  a.res = ctx->d_res;
  a.deep = deep_args(ctx);
  (void)hipGetLastError();  // drop a stale error left by another library
  hipError_t e = launch_result_init(ctx->d_res, n, s);
  uint64_t fixed = 0;
  bool fused = false;
  if (n && protocol == TGPU_PROTOCOL_BINARY && schema->fixed_binary && !offsets &&
      in_len >= n * (uint64_t)schema->tmpl.wire_len) {
    fixed = schema->tmpl.wire_len;
    a.exc = ctx->d_irr;
    a.exc_cap = std::min<uint64_t>(ctx->reserved, kFixedExceptionCap);
    const bool blocking = st || n_decoded || consumed;
    if (blocking && n >= kFixedProbeMin && e == hipSuccess) {
      // a stream whose stride is not L from record 0 on (every record
      // carrying an unknown field, ...): index it directly
      e = launch_fixed_probe(a, protocol, fixed, s);
      if (e == hipSuccess)
        e = hipMemcpyAsync(ctx->h_res, ctx->d_res, sizeof(DevResult), hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e == hipSuccess && ctx->h_res->first_misfit == 0) {
        a.offs = ctx->d_offs;
        // record 0's length: a stream of records that all carry the same
        // appended fields is fixed-stride too, at this length — the tolerant
        // program decodes record i at i * L2, the exception list and the
        // misfit rule work as at L, and a stream that is not takes the index
        // from its first misfit
        const uint64_t L2 = ctx->h_res->total_bytes;
        const int32_t height = a.height ? a.height : a.max_depth;
        const bool stride2 = L2 && L2 != fixed && L2 <= (1ull << 20) && n * L2 <= in_len &&
                             has_prog(schema, protocol) && height >= 2 && a.max_depth >= 2;
        int trc;
        uint64_t len = fixed;
        if (stride2) {
          const int q = prog_protocol(schema, protocol);
          DecodeArgs f = a;
          f.fixed_len = len = L2;
          e = launch_result_init(ctx->d_res, n, s);
          if (e == hipSuccess)
            e = launch_program_decode(
                f, schema->d_prog_tol[q], a.rec_size, ctx->d_irr, &ctx->d_res->n_irregular, s,
                jit_kernels(schema->prog_tol[q], schema->device, JIT_DECODE, n, 0, false));
          if (e == hipSuccess) e = launch_fixed_exceptions(f, protocol, L2, s);
          // (the tail after a misfit is indexed: its decode is not fixed-stride)
          trc = fixed_tail(ctx, schema, protocol, a, L2, limits, s, e, ~0ull, true);
        } else {
          trc = fixed_tail(ctx, schema, protocol, a, fixed, limits, s, e, 0);
        }
        ctx->last_op = 1;
        if (e != hipSuccess || trc < 0) {
          fill_status(st, TGPU_ERR_HIP, 0, 0);
          if (st) st->reserved = (int32_t)e;
          return TGPU_ERR_HIP;
        }
        if (trc == 0) {  // every record at its stride L2
          fill_status(st, TGPU_OK, n, 0);
          if (n_decoded) *n_decoded = n;
          if (consumed) *consumed = n * len;
          return TGPU_OK;
        }
        tgpu_status tmp;
        return tgpu_context_wait(ctx, stream, st ? st : &tmp, n_decoded, consumed);
      }
      if (e == hipSuccess) e = launch_result_init(ctx->d_res, n, s);
    }
    const JitKernels* fj = fixed_jit(schema, protocol, JIT_DECODE, n);
    if (e == hipSuccess && fj) {
      DecodeArgs f = a;
      f.fixed_len = fixed;
      e = launch_program_decode(f, schema->d_prog[prog_protocol(schema, protocol)], a.rec_size, ctx->d_irr,
                                &ctx->d_res->n_irregular, s, fj);
    } else if (e == hipSuccess && schema->has_plan && ((uintptr_t)records & 7) == 0)
      e = launch_plan_binary_decode(&schema->plan, schema->d_plan, a.in, n, a.recs, ctx->d_res,
                                    a.exc, a.exc_cap, s);
    else if (e == hipSuccess)
      e = launch_fixed_binary_decode(&schema->tmpl, schema->d_tmpl, a.in, n, a.recs, ctx->d_res,
                                     a.exc, a.exc_cap, s);
    a.offs = ctx->d_offs;
    a.check_index = 0;
    // stream-ordered calls re-read the records from a misfit on without the
    // host: at the misfit's own length by the tolerant program (persistent,
    // returns at once when every record was at its stride), then one lane
    // from the first record off that stride too
    const JitKernels* tj = blocking ? nullptr : stream_tail_jit(schema, protocol, a);
    // exceptions read at their stride; first_irregular becomes the first
    // record not at its stride position
    if (e == hipSuccess)
      e = blocking ? launch_fixed_exceptions(a, protocol, fixed, s)
                   : launch_fixed_exceptions_stream(
                         a, protocol, fixed, tj ? stream_tail_max_stride(a.rec_size, fixed) : 0,
                         s);
    if (blocking) {
      // blocking call: look at the plan kernel's verdict, and index + decode
      // the tail after a non-canonical record in parallel
      const int trc = fixed_tail(ctx, schema, protocol, a, fixed, limits, s, e);
      if (trc >= 0) {
        ctx->last_op = 1;
        if (e != hipSuccess) {
          fill_status(st, TGPU_ERR_HIP, 0, 0);
          if (st) st->reserved = (int32_t)e;
          return TGPU_ERR_HIP;
        }
        if (trc == 0) {  // every record canonical: decoded by the plan kernel
          fill_status(st, TGPU_OK, n, 0);
          if (n_decoded) *n_decoded = n;
          if (consumed) *consumed = n * fixed;
          return TGPU_OK;
        }
        tgpu_status tmp;
        return tgpu_context_wait(ctx, stream, st ? st : &tmp, n_decoded, consumed);
      }
    }
    if (e == hipSuccess && tj)
      e = launch_stream_tail_decode(a, a.rec_size, (uint32_t)fixed, a.exc,
                                    &ctx->d_res->n_irregular, s, tj, schema->device);
    if (e == hipSuccess) e = launch_fixed_stream_finish(a, protocol, fixed, s);
  } else if (n) {
    pack_args(ctx, schema, protocol, a);
    if (offsets) {
      a.offs = offsets;
    } else {
      // unindexed: build the record index on the device first (k_index.hip);
      // records past the stream's end / its first bad record re-read that
      // position, so the decoder reports them exactly
      a.offs = ctx->d_offs;
      if (e == hipSuccess) {
        // the index tiles decode their records as they find them (fused);
        // whatever they leave goes to the general decoder below
        const int irc = launch_index(ctx, schema, protocol, a.in, in_len, 0, in_len, 0, ctx->d_offs,
                                     n, n, limits, s, e, &a, &fused, false,
                                     st || n_decoded || consumed);
        if (irc) {
          fill_status(st, irc, 0, 0);
          return irc;
        }
      }
    }
    a.check_index = 1;
    if (e == hipSuccess && fused)
      e = launch_general_decode_list(a, protocol, ctx->d_irr, &ctx->d_res->n_irregular, s);
    else if (e == hipSuccess)
      e = launch_indexed_decode(ctx, schema, protocol, a, s);
  }
  if (e == hipSuccess && n) e = launch_decode_finish(a, protocol, fixed, s);
  if (e == hipSuccess && n && !fixed) e = finish_pack(schema, protocol, a, s);
  ctx->last_op = 1;
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  if (st || n_decoded || consumed) {
    tgpu_status tmp;
    return tgpu_context_wait(ctx, stream, st ? st : &tmp, n_decoded, consumed);
  }
  return TGPU_OK;
}

namespace {
int grow(uint8_t*& p, uint64_t& have, uint64_t want) {
  if (want <= have) return TGPU_OK;
  if (p) (void)hipFree(p);
  p = nullptr;
  have = 0;
  if (hipMalloc(&p, want) != hipSuccess) return TGPU_ERR_HIP;
  have = want;
  return TGPU_OK;
}
}  // namespace

namespace {
// The wire-to-wire transcoder (tgpu_xcode.h, k_transcode.hip) applies when
// both protocols have the schema's flat record program and the stream is not
// a fixed-layout Binary stream without offsets (that one's fastest read is the
// plan kernel; it stays on the composed decode + encode). TGPU_XCODE=0: the
// composed form everywhere (A/B).
bool xcode_fused(const tgpu_schema* s, int from, int to, const uint64_t* offsets,
                 uint64_t in_len, uint64_t n) {
  if (const char* v = getenv("TGPU_XCODE"))
    if (v[0] == '0') return false;
  const int qf = prog_protocol(s, from), qt = prog_protocol(s, to);
  if (qf < 0 || qt < 0 || !s->has_prog[qf] || !s->has_prog[qt]) return false;
  // a fixed-layout Binary source: the composed decode + encode is faster
  // (unindexed: the plan kernel; indexed, config 2 measured: fused 4.98 ms
  // against 4.77 composed — one record per lane of 89 B, the fused tile's
  // LDS holds fewer of them than the decode's), so every such call composes
  if (from == TGPU_PROTOCOL_BINARY && s->fixed_binary) return false;
  return true;
}

int transcode_fused(tgpu_context* ctx, const tgpu_schema* schema, int from, int to,
                    const void* in, uint64_t in_len, const uint64_t* offsets, uint64_t n, void* out,
                    uint64_t out_capacity, uint64_t* out_offsets, const tgpu_limits* limits,
                    void* stream, tgpu_status* st, uint64_t* n_done, uint64_t* out_size) {
  const hipStream_t s = (hipStream_t)stream;
  const uint64_t rs = schema->structs[0].size;
  const uint64_t acap = schema->has_lists ? in_len * tgpu_schema_arena_scale(schema, from) : 0;
  int rc = ensure_workspace(ctx, n);
  if (!rc) rc = ensure_deep(ctx, limit_depth(limits), schema->recursive);
  if (!rc) rc = grow(ctx->d_xrec, ctx->xrec_bytes, std::max<uint64_t>(n * rs, 16));
  if (!rc && acap) rc = grow(ctx->d_xarena, ctx->xarena_bytes, acap);
  if (!rc && !out_offsets) rc = grow(ctx->d_xoffs, ctx->xoffs_bytes, (n + 1) * sizeof(uint64_t));
  // the single pass or the two tile passes (TGPU_XCODE_ONEPASS=1 / 0 force
  // one): the single pass saves the size pass's read and parse of the
  // stream, and adds a look-back round trip per tile (3-5 us of a resident
  // workgroup) — it wins where a tile holds more bytes (config 4, 22.8 KiB
  // of input per tile: 3.48 vs 4.24 ms) and loses on lighter tiles (config
  // 3, 13.6 KiB: 3.99 vs 3.51 ms)
  const char* op = getenv("TGPU_XCODE_ONEPASS");
  const bool one = op && *op ? op[0] != '0' : (n && in_len / n * 256 >= 16384);
  const uint64_t tiles = (n + 255) / 256;
  if (!rc && one) rc = grow(ctx->d_xstat, ctx->xstat_bytes, (tiles + 1) * sizeof(uint64_t));
  if (rc) {
    fill_status(st, rc, 0, 0);
    return rc;
  }
  const bool blocking = st || n_done || out_size;
  XcodeArgs x{};
  DecodeArgs& a = x.d;
  a.sc = dev_schema(schema, from);
  a.in = (const uint8_t*)in;
  a.in_len = in_len;
  a.n = n;
  a.recs = ctx->d_xrec;
  a.arena = acap ? ctx->d_xarena : nullptr;
  a.arena_cap = acap;
  a.string_limit = limits ? limits->string_limit : 0;
  a.container_limit = limits ? limits->container_limit : 0;
  a.max_depth = limits ? limits->max_depth : 12000;
  a.height = limits ? limits->height : 0;
  a.rec_size = (uint32_t)rs;
  a.check_index = 1;
  a.res = ctx->d_res;
  a.deep = deep_args(ctx);
  EncodeArgs& w = x.e;
  w.sc = dev_schema(schema, to);
  w.recs = ctx->d_xrec;
  w.n = n;
  w.sbase = a.in;
  w.lbase = a.arena;
  w.out = (uint8_t*)out;
  w.cap = out_capacity;
  w.offs = out_offsets ? out_offsets : (uint64_t*)ctx->d_xoffs;
  w.block_sums = ctx->d_block_sums;
  w.scan_part = ctx->d_scan_part;
  w.rec_size = (uint32_t)rs;
  w.res = ctx->d_res;
  w.deep = a.deep;
  x.irr = ctx->d_irr;
  x.nirr = &ctx->d_res->n_irregular;
  x.want_offs = out_offsets ? 1u : 0u;
  x.xstat = one ? (unsigned long long*)ctx->d_xstat : nullptr;
  {
    // the target's bytes per record for the LDS output tile: the source's
    // mean, or more where the target's smallest record is larger (Compact ->
    // Binary: fixed-width integers, 3-byte field headers)
    const int qs = prog_protocol(schema, from), qd = prog_protocol(schema, to);
    const uint64_t in_mean = n ? in_len / n : 0;
    const uint64_t ms = prog_min_len(schema->prog[qs]), md = prog_min_len(schema->prog[qd]);
    const uint64_t est = in_mean + (md > ms ? md - ms : 0);
    x.out_mean = (uint32_t)std::min<uint64_t>(est, 1u << 20);
  }
  (void)hipGetLastError();  // drop a stale error left by another library
  hipError_t e = launch_result_init(ctx->d_res, n, s);
  if (offsets) {
    a.offs = offsets;
  } else {
    // unindexed: the stream index first (records past the end / the first bad
    // record re-read that position, so the reader reports them exactly)
    a.offs = ctx->d_offs;
    const int irc = launch_index(ctx, schema, from, a.in, in_len, 0, in_len, 0, ctx->d_offs, n, n,
                                 limits, s, e, nullptr, nullptr, false, blocking);
    if (irc) {
      fill_status(st, irc, 0, 0);
      return irc;
    }
    // (the index counted its own general-reader records in n_irregular)
    if (e == hipSuccess)
      e = hipMemsetAsync(&ctx->d_res->n_irregular, 0, sizeof(unsigned long long), s);
  }
  const int qf = prog_protocol(schema, from), qt = prog_protocol(schema, to);
  const JitKernels* jit =
      jit_kernels_xcode(schema->prog[qf], schema->prog[qt], schema->device, n, false);
  if (e == hipSuccess)
    e = launch_xcode(x, from, to, schema->d_prog[qf], schema->d_prog[qt], s, jit);
  ctx->last_op = 2;
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  if (blocking) {
    tgpu_status tmp;
    return tgpu_context_wait(ctx, stream, st ? st : &tmp, n_done, out_size);
  }
  return TGPU_OK;
}
}  // namespace

int tgpu_transcode_batch(tgpu_context* ctx, const tgpu_schema* schema, int from_protocol,
                         int to_protocol, const void* in, uint64_t in_len,
                         const uint64_t* offsets, uint64_t n, void* out, uint64_t out_capacity,
                         uint64_t* out_offsets, const tgpu_limits* limits, void* stream,
                         tgpu_status* st, uint64_t* n_done, uint64_t* out_size) {
  if (n_done) *n_done = 0;
  if (out_size) *out_size = 0;
  if (!ctx || !schema || !valid_protocol(from_protocol) || !valid_protocol(to_protocol) ||
      (n && (!in || !out))) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  if (n && xcode_fused(schema, from_protocol, to_protocol, offsets, in_len, n))
    return transcode_fused(ctx, schema, from_protocol, to_protocol, in, in_len, offsets, n, out,
                           out_capacity, out_offsets, limits, stream, st, n_done, out_size);
  // records and list elements stay in HBM between the passes (grow-only)
  const uint64_t rs = schema->structs[0].size;
  const uint64_t acap = in_len * tgpu_schema_arena_scale(schema, from_protocol);
  int rc = grow(ctx->d_xrec, ctx->xrec_bytes, std::max<uint64_t>(n * rs, 16));
  if (!rc && acap) rc = grow(ctx->d_xarena, ctx->xarena_bytes, acap);
  if (rc) {
    fill_status(st, rc, 0, 0);
    return rc;
  }
  tgpu_status dst{};
  uint64_t nd = 0, consumed = 0;
  const int drc = tgpu_decode_batch(ctx, schema, from_protocol, in, in_len, offsets, n,
                                    ctx->d_xrec, acap ? ctx->d_xarena : nullptr, acap, limits,
                                    stream, &dst, &nd, &consumed);
  if (drc && nd == 0 && dst.exc_class == TGPU_EXC_RUNTIME) {  // usage / HIP error
    if (st) *st = dst;
    return drc;
  }
  tgpu_status est{};
  uint64_t total = 0;
  const int erc = tgpu_encode_batch(ctx, schema, to_protocol, ctx->d_xrec, nd, in,
                                    acap ? ctx->d_xarena : nullptr, out, out_capacity,
                                    out_offsets, stream, &est, &total);
  if (out_size) *out_size = total;
  // the first failure in record order: an encode failure is at a record
  // before the one the decoder rejected
  if (erc) {
    if (st) *st = est;
    if (n_done) *n_done = est.record;
    return erc;
  }
  if (n_done) *n_done = nd;
  if (st) *st = dst;
  return drc;
}

int tgpu_decode_stream(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                       const void* in, uint64_t in_len, uint64_t begin, uint64_t end,
                       int speculative, uint64_t* offsets, uint64_t max_records, void* records,
                       void* list_arena, uint64_t list_arena_capacity,
                       const tgpu_limits* limits, void* stream, tgpu_status* st,
                       uint64_t* n_records, uint64_t* first_start, uint64_t* last_end) {
  if (!ctx || !schema || !offsets || (max_records && !records) ||
      !valid_protocol(protocol) ||
      (!in && in_len) || begin > end || end > in_len ||
      ((uintptr_t)records) % schema->structs[0].align) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const hipStream_t s = (hipStream_t)stream;
  int rc = ensure_workspace(ctx, max_records + 1);
  if (!rc) rc = ensure_deep(ctx, limit_depth(limits), schema->recursive);
  if (rc) {
    fill_status(st, rc, 0, 0);
    return rc;
  }
  DecodeArgs a{};
  a.sc = dev_schema(schema, protocol);
  a.in = (const uint8_t*)in;
  a.in_len = in_len;
  a.n = max_records;
  a.offs = offsets;
  a.recs = (uint8_t*)records;
  a.arena = (uint8_t*)list_arena;
  a.arena_cap = list_arena_capacity;
  a.string_limit = limits ? limits->string_limit : 0;
  a.container_limit = limits ? limits->container_limit : 0;
  a.max_depth = limits ? limits->max_depth : 12000;
  a.height = limits ? limits->height : 0;
  a.rec_size = schema->structs[0].size;
  // lengths come from the same reader that found them; the failing record's
  // successor has no start to check against
  a.check_index = 0;
  a.res = ctx->d_res;
  a.deep = deep_args(ctx);
  if (max_records) pack_args(ctx, schema, protocol, a);
  (void)hipGetLastError();  // drop a stale error left by another library
  hipError_t e = launch_result_init(ctx->d_res, 0, s);
  bool fused = false;
  rc = launch_index(ctx, schema, protocol, a.in, in_len, begin, end, speculative, offsets,
                    max_records, 0, limits, s, e, max_records ? &a : nullptr, &fused, false,
                    st != nullptr);
  if (rc) {
    fill_status(st, rc, 0, 0);
    return rc;
  }
  if (e == hipSuccess && fused) {
    e = launch_general_decode_list(a, protocol, ctx->d_irr, &ctx->d_res->n_irregular, s);
    if (e == hipSuccess) e = launch_stream_decode_finish(a, protocol, s);
  } else if (e == hipSuccess && max_records) {
    // the range was indexed without the tile path: decode the records found
    e = hipMemcpyAsync(ctx->h_res, ctx->d_res, sizeof(DevResult), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) {
      const DevResult r = *ctx->h_res;
      uint64_t m = std::min<uint64_t>(r.n_records, max_records);
      if (r.code && r.n_records < max_records) m += 1;  // the failing record, partially
      if (m) {
        DecodeArgs b = a;
        b.n = m;
        e = launch_general_decode(b, protocol, s);
        if (e == hipSuccess) e = launch_deep_decode(b, protocol, s);
      }
      // the index's result stands (same records, same first failure)
      if (e == hipSuccess)
        e = hipMemcpyAsync(ctx->d_res, ctx->h_res, sizeof(DevResult), hipMemcpyHostToDevice, s);
    }
  }
  if (e == hipSuccess && max_records) e = finish_pack(schema, protocol, a, s);
  ctx->last_op = 3;
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  if (!st && !n_records && !first_start && !last_end) return TGPU_OK;
  e = hipMemcpyAsync(ctx->h_res, ctx->d_res, sizeof(DevResult), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  const DevResult& r = *ctx->h_res;
  int code = r.code;
  uint64_t rec = code ? r.first_fail : r.n_records, off = code ? r.fail_offset : 0;
  if (!code && r.n_records > max_records) {
    code = TGPU_ERR_OUTPUT_OVERFLOW;
    rec = max_records;
  }
  fill_status(st, code, rec, off);
  if (n_records) *n_records = r.n_records;
  if (first_start) *first_start = r.first_start;
  if (last_end) *last_end = r.total_bytes;
  return code;
}

int tgpu_skim_batch(tgpu_context* ctx, int protocol, const void* in, uint64_t in_len,
                    const uint64_t* offsets, uint64_t n, tgpu_skim_field* fields,
                    uint32_t max_fields, uint32_t* field_counts, const tgpu_limits* limits,
                    void* stream, tgpu_status* st, uint64_t* n_done) {
  return tgpu_skim_batch_ex(ctx, protocol, in, in_len, offsets, n, fields, max_fields,
                            field_counts, 0, limits, stream, st, n_done);
}

int tgpu_skim_batch_ex(tgpu_context* ctx, int protocol, const void* in, uint64_t in_len,
                       const uint64_t* offsets, uint64_t n, tgpu_skim_field* fields,
                       uint32_t max_fields, uint32_t* field_counts, uint32_t max_nest,
                       const tgpu_limits* limits, void* stream, tgpu_status* st,
                       uint64_t* n_done) {
  if (!ctx || !valid_protocol(protocol) || max_nest > TGPU_SKIM_MAX_NEST ||
      (n && (!offsets || !field_counts || (max_fields && !fields) || (!in && in_len))) ||
      ((uintptr_t)fields & 15)) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const hipStream_t s = (hipStream_t)stream;
  int rc = ensure_workspace(ctx, n);
  if (!rc) rc = ensure_deep(ctx, limit_depth(limits));  // (schemaless: the skim's deep pass has one tier)
  if (rc) {
    fill_status(st, rc, 0, 0);
    return rc;
  }
  SkimArgs a{};
  a.in = (const uint8_t*)in;
  a.in_len = in_len;
  a.offs = offsets;
  a.n = n;
  a.fields = fields;
  a.counts = field_counts;
  a.max_fields = max_fields;
  a.string_limit = limits ? limits->string_limit : 0;
  a.container_limit = limits ? limits->container_limit : 0;
  a.max_depth = limits ? limits->max_depth : 12000;
  a.height = limits ? limits->height : 0;
  a.res = ctx->d_res;
  a.deep = deep_args(ctx);
  a.nt_stores = getenv("TGPU_SKIM_NT") ? atoi(getenv("TGPU_SKIM_NT")) : 1;
  a.max_nest = max_nest;
  (void)hipGetLastError();
  hipError_t e = launch_result_init(ctx->d_res, n, s);
  if (e == hipSuccess) e = launch_skim(a, protocol, s);
  ctx->last_op = 1;
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  if (st || n_done) {
    tgpu_status tmp;
    return tgpu_context_wait(ctx, stream, st ? st : &tmp, n_done, nullptr);
  }
  return TGPU_OK;
}

int tgpu_index_stream(tgpu_context* ctx, const tgpu_schema* schema, int protocol, const void* in,
                      uint64_t in_len, uint64_t begin, uint64_t end, int speculative,
                      uint64_t* offsets, uint64_t max_records, const tgpu_limits* limits,
                      void* stream, tgpu_status* st, uint64_t* n_records, uint64_t* first_start,
                      uint64_t* last_end) {
  if (!ctx || !schema || !offsets ||
      !valid_protocol(protocol) ||
      (!in && in_len) || begin > end || end > in_len) {
    fill_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const hipStream_t s = (hipStream_t)stream;
  const int drc = ensure_deep(ctx, limit_depth(limits), schema->recursive);
  if (drc) {
    fill_status(st, drc, 0, 0);
    return drc;
  }
  (void)hipGetLastError();  // drop a stale error left by another library
  hipError_t e = launch_result_init(ctx->d_res, 0, s);
  const int rc = launch_index(ctx, schema, protocol, (const uint8_t*)in, in_len, begin, end,
                              speculative, offsets, max_records, 0, limits, s, e, nullptr,
                              nullptr, false, st || n_records || first_start || last_end);
  if (rc) {
    fill_status(st, rc, 0, 0);
    return rc;
  }
  ctx->last_op = 3;
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  if (!st && !n_records && !first_start && !last_end) return TGPU_OK;
  e = hipMemcpyAsync(ctx->h_res, ctx->d_res, sizeof(DevResult), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    fill_status(st, TGPU_ERR_HIP, 0, 0);
    if (st) st->reserved = (int32_t)e;
    return TGPU_ERR_HIP;
  }
  const DevResult& r = *ctx->h_res;
  int code = r.code;
  uint64_t rec = code ? r.first_fail : r.n_records, off = code ? r.fail_offset : 0;
  if (!code && r.n_records > max_records) {
    code = TGPU_ERR_OUTPUT_OVERFLOW;
    rec = max_records;
  }
  fill_status(st, code, rec, off);
  if (n_records) *n_records = r.n_records;
  if (first_start) *first_start = r.first_start;
  if (last_end) *last_end = r.total_bytes;
  return code;
}

}  // extern "C"
