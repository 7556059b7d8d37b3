// k_skim.hip — schemaless skim of an indexed stream (tgpu_skim_batch).
//
// One lane per record walks its top-level fields (and, with max_nest, those of
// struct-valued fields, pre-order) exactly like the parse loop of
// protocol::parseObject (thrift/lib/cpp2/protocol/detail/Object.h:416-432):
// readFieldBegin until STOP; a bool is read (FieldMaskUtil.h:441-450), any
// other value is passed over by the protocol's skip and kept as (offset,
// length) of its encoded bytes, the masked parse's setMaskedDataFull
// (FieldMaskUtil.h:373-388). The reader, skip and limits are the decoder's
// (tgpu_device.h), so depth / size / varint / bool errors are the ones the
// decoder reports for the same bytes. The first failing record in record
// order is re-diagnosed by one lane and published like a decode result.
#include <cstdlib>

#include "tgpu_device.h"

namespace tgpu {
namespace {

using namespace dev;

// Skims record i into its field slots; returns the reader (error latched).
// The reader walks `src` (the stream, or an LDS copy of bytes
// [base, base + src_len) of it) in positions relative to `base`; stored
// offsets and error offsets are absolute.
// kNest: the nested form (a.max_nest > 0) — its level stack costs ~35 VGPRs,
// so the flat skim is its own instantiation.
template <int P, bool kNest = false>
__device__ Reader skim_one(const SkimArgs& a, uint64_t i, bool store, const uint8_t* src,
                           uint64_t base, uint64_t src_len, int lane) {
  // slot k of record i at fields[k * n + i] (field-major: a wave's k-th
  // stores are 64 consecutive entries)
  tgpu_skim_field* out = a.fields + i;
  using Pr = Proto<P>;
  const uint64_t start = a.offs[i];
  Reader r = make_reader(src, start - base, src_len, a.string_limit, a.container_limit,
                         a.max_depth, a.height);
  if (lane >= 0) attach_slab(r, a.deep, (uint32_t)lane);
  if (start > a.in_len || a.offs[i + 1] < start) {
    r.fail(TGPU_ERR_INDEX_MISMATCH, start - base);
    r.err_off += base;
    return r;
  }
  uint32_t count = 0;
  int32_t prev = 0;
  // struct-valued fields descended into (a.max_nest levels): the entry slot
  // reserved for the struct, its value start, its id and the enclosing
  // level's last field id (Compact's pushed lastFieldId_)
  uint32_t lvl = 0;
  constexpr uint32_t kLv = kNest ? TGPU_SKIM_MAX_NEST : 1;
  uint32_t nslot[kLv];
  uint64_t nstart[kLv];
  int32_t nid[kLv];
  const uint32_t max_nest = kNest ? a.max_nest : 0;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  auto put = [&](uint32_t k, int32_t id, uint32_t wt, uint32_t flags, uint64_t len, uint64_t off) {
    // one 16-byte entry {id, ttype, flags | length | offset}
    const uint64_t o = off + base;
    const u32x4 e = {(uint32_t)(uint16_t)id | (wt << 16) | (flags << 24), (uint32_t)len,
                     (uint32_t)o, (uint32_t)(o >> 32)};
    u32x4* dst = (u32x4*)(out + (uint64_t)k * a.n);
    if (a.nt_stores) __builtin_nontemporal_store(e, dst);
    else *dst = e;
  };
  while (r.ok()) {
    uint32_t wt = 0;
    int32_t id = 0;
    if (!Pr::field_header(r, prev, wt, id)) {  // STOP or error
      if (!r.ok() || !kNest || lvl == 0) break;
      // a descended struct's STOP: readStructEnd, then its entry
      r.ascend();
      --lvl;
      if (r.pos - nstart[lvl] > 0xffffffffull) {
        r.fail(TGPU_ERR_UNSUPPORTED, nstart[lvl]);
        break;
      }
      if (store && nslot[lvl] < a.max_fields)
        put(nslot[lvl], nid[lvl], TGPU_T_STRUCT, lvl << TGPU_SKIM_LEVEL_SHIFT,
            r.pos - nstart[lvl], nstart[lvl]);
      prev = nid[lvl];
      continue;
    }
    prev = id;
    const uint64_t off = r.pos;
    if (kNest && wt == TGPU_T_STRUCT && lvl < max_nest) {
      // parseValue -> parseObjectInplace: the struct's own fields, with the
      // checks skip(T_STRUCT, lvl) makes (max_depth, readStructBegin)
      if ((int32_t)lvl >= r.max_depth) {
        r.fail(TGPU_ERR_DEPTH_LIMIT, r.pos);
        break;
      }
      r.descend(r.pos);
      if (!r.ok()) break;
      nslot[lvl] = count;
      nstart[lvl] = off;
      nid[lvl] = id;
      ++count;
      ++lvl;
      prev = 0;
      continue;
    }
    uint32_t flags = lvl << TGPU_SKIM_LEVEL_SHIFT;
    if (wt == TGPU_T_BOOL) flags |= TGPU_SKIM_BOOL | (Pr::read_bool(r) ? TGPU_SKIM_TRUE : 0);
    // leaves inline (skip's explicit stack lives in scratch); structs and
    // containers take the full skip
    else if (r.max_depth <= (int32_t)lvl || !Pr::skip_leaf(r, wt)) skip<P>(r, wt, (int32_t)lvl);
    if (!r.ok()) break;
    // an entry's length is 32 bits: a value of 4 GiB or more is reported
    if (r.pos - off > 0xffffffffull) {
      r.fail(TGPU_ERR_UNSUPPORTED, off);
      break;
    }
    if (store && count < a.max_fields) put(count, id, wt, flags, r.pos - off, off);
    ++count;
  }
  if (store) a.counts[i] = count;
  if (r.ok() && r.pos + base != a.offs[i + 1]) r.fail(TGPU_ERR_INDEX_MISMATCH, r.pos);
  r.pos += base;
  r.err_off += base;
  return r;
}

template <int P, bool kNest = false>
__device__ __forceinline__ Reader skim_global(const SkimArgs& a, uint64_t i, bool store,
                                              int lane) {
  return skim_one<P, kNest>(a, i, store, a.in, 0, a.in_len, lane);
}

// One 256-record tile per workgroup: the tile's wire bytes
// [offs[r0], offs[r1]) are copied to LDS with 16-byte loads when they fit
// (kSkimTile), and each lane parses its record there; a record whose parse
// fails on the copy (damaged input, a length running off the tile) is parsed
// again from HBM, so every status is the stream's own. Tiles too large for
// LDS parse from HBM directly. kSkimTile: LDS bytes of the wire copy.
template <int P, uint32_t kSkimTile, bool kNest>
__global__ __launch_bounds__(256) void skim_kernel(SkimArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kSkimTile + 16];
  const uint64_t r0 = (uint64_t)blockIdx.x * 256;
  const uint64_t r1 = min(r0 + 256, a.n);
  const uint64_t b0 = a.offs[r0], b1 = a.offs[r1];
  const uint64_t a0 = b0 & ~15ull;
  const bool staged = b0 <= b1 && b1 <= a.in_len && b1 - a0 <= kSkimTile;
  if (staged) {
    const uint32_t nbytes = (uint32_t)(b1 - a0);
    const uint32_t nvec = (nbytes + 15) >> 4;
    for (uint32_t v = threadIdx.x; v < nvec; v += 256) {
      const uint64_t g = a0 + 16ull * v;
      if (g + 16 <= a.in_len) {
        *(uint4*)(tile + 16 * v) = *(const uint4*)(a.in + g);
      } else {
        for (uint32_t b = 0; b < 16 && g + b < a.in_len; ++b) tile[16 * v + b] = a.in[g + b];
      }
    }
  }
  __syncthreads();
  const uint64_t i = r0 + threadIdx.x;
  if (i >= a.n) return;
  Reader r = staged ? skim_one<P, kNest>(a, i, true, tile, a0, b1 - a0, -1)
                    : skim_global<P, kNest>(a, i, true, -1);
  if (staged && !r.ok() && r.err != kErrDeep) r = skim_global<P, kNest>(a, i, true, -1);
  if (!r.ok()) defer_or_fail(r, a.deep, &a.res->first_fail, i);
}

// Records the skim deferred (a value nested past the private skip frames).
template <int P>
__global__ __launch_bounds__(64) void deep_skim_kernel(SkimArgs a) {
  const uint32_t lane = blockIdx.x * 64 + threadIdx.x;
  if (lane >= a.deep.lanes) return;
  const uint64_t m = *a.deep.count;
  for (uint64_t k = lane; k < m; k += a.deep.lanes) {
    const uint64_t i = a.deep.list[k];
    const Reader r = a.max_nest ? skim_global<P, true>(a, i, true, (int)lane)
                                : skim_global<P>(a, i, true, (int)lane);
    if (!r.ok()) atomicMin(&a.res->first_fail, (unsigned long long)i);
  }
}

template <int P>
__global__ void skim_finish_kernel(SkimArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DevResult* res = a.res;
  const uint64_t f = res->first_fail;
  if (f < a.n) {
    const Reader r = a.max_nest ? skim_global<P, true>(a, f, false, 0)
                                : skim_global<P>(a, f, false, 0);
    res->code = r.ok() ? TGPU_ERR_INDEX_MISMATCH : r.err;
    res->fail_offset = r.ok() ? r.pos : r.err_off;
    res->n_records = f;
    res->total_bytes = a.offs[f] - a.offs[0];
  } else {
    res->code = 0;
    res->n_records = a.n;
    res->total_bytes = a.n ? a.offs[a.n] - a.offs[0] : 0;
  }
}

}  // namespace

// Wire copy per 256-record tile: 24 KB (6 workgroups per CU; a config-2 tile
// is 22.8 KB) unless the stream's mean tile is larger, then 32 KB (4 per CU).
// Measured on MI355X (tools/skim_ab.py): 24 KB beats 32 KB on configs 2-4
// even where a share of the tiles overflows to HBM parsing (config 4: 1.52
// vs 1.96 ms), and 16 KB gains nothing on config 3. TGPU_SKIM_TILE=24|32
// forces one (A/B).
hipError_t launch_skim(const SkimArgs& a, int protocol, hipStream_t stream) {
  if (a.n) {
    const uint32_t g = (uint32_t)((a.n + 255) / 256);
    uint32_t kb = a.in_len / a.n * 256 <= 24560 ? 24 : 32;
    if (const char* e = getenv("TGPU_SKIM_TILE")) kb = (uint32_t)atoi(e);
#define TGPU_SKIM(KB, NEST)                                                                \
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL((skim_kernel<P_, KB, NEST>), dim3(g), dim3(256), \
                                                0, stream, a))
    if (kb == 24 && !a.max_nest) TGPU_SKIM(24560, false);
    else if (kb == 24) TGPU_SKIM(24560, true);
    else if (!a.max_nest) TGPU_SKIM(32752, false);
    else TGPU_SKIM(32752, true);
#undef TGPU_SKIM
  }
  if (a.deep.lanes)
    TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(deep_skim_kernel<P_>,
                                                  dim3((a.deep.lanes + 63) / 64), dim3(64), 0,
                                                  stream, a));
  TGPU_BY_PROTOCOL(protocol,
                   hipLaunchKernelGGL(skim_finish_kernel<P_>, dim3(1), dim3(64), 0, stream, a));
  return hipGetLastError();
}

}  // namespace tgpu
