// k_general.hip — table-driven gfx950 kernels for arbitrary schemas:
//   general_decode   one lane per record, full readNoXfer semantics
//   walk_offsets     record boundary discovery by skip-parsing (one lane;
//                    fallback for unindexed irregular streams)
//   encode_size /    three-pass variable-length encode: per-record wire size,
//   scan_blocks /    exclusive scan of block sums, block-local scan + emit
//   encode_write
//   *_finish         single-lane epilogues: re-run the first failing record to
//                    recover its exact error code and byte offset (the
//                    exception the reference would have thrown) and publish
//                    the batch result.
// All state lives in the caller's stream order; nothing is read back to the
// host inside a call, so calls can be captured into a hipGraph.
#include <algorithm>
#include <cstdlib>

#include "tgpu_device.h"

namespace tgpu {
namespace {

using namespace dev;

constexpr unsigned long long kNone = ~0ull;

__global__ void result_init_kernel(DevResult* res, uint64_t n) {
  res->first_fail = kNone;
  res->first_irregular = kNone;
  res->code = 0;
  res->pad = 0;
  res->fail_offset = 0;
  res->total_bytes = 0;
  res->n_records = n;
  res->n_irregular = 0;
  res->first_start = kNone;
  res->n_deep = 0;
  res->n_deep2 = 0;
  res->n_deep_chunks = 0;
  res->first_misfit = kNone;
  res->tail_first = kNone;
  res->tail_pos = 0;
  res->tail_stride = 0;
  res->tail_min = kNone;
}

// Parses record i (record buffer zeroed first); lane: deep-pass lane or -1.
template <int P>
__device__ __forceinline__ Reader decode_one(const DecodeArgs& a, uint64_t i, int lane = 0) {
  return decode_record<P>(a, i, lane);
}

// Indexed streams: one lane per record, records independent. scap: dynamic
// LDS bytes for the schema tables (stage_schema).
template <int P>
__global__ __launch_bounds__(256) void general_decode_kernel(DecodeArgs a, uint32_t scap) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sch[];
  DecodeArgs b = a;
  b.sc = stage_schema(a.sc, sch, scap);
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    const Reader r = decode_one<P>(b, i, -1);
    if (!r.ok()) defer_or_fail(r, a.deep, &a.res->first_fail, i);
  }
}

// Indexed streams, 256 records per workgroup: the tile's wire bytes
// [offs[r0], offs[r1]) are copied to LDS with 16-byte loads when they fit
// (tile_cap, sized by the caller from the mean record) and each lane reads
// its record there (the general reader is byte-serial: LDS latency instead of
// HBM's per byte); a record whose read fails on the copy is read again from
// HBM, so every status is the stream's own; a tile too large reads from HBM.
template <int P>
__global__ __launch_bounds__(256) void general_decode_tile_kernel(DecodeArgs a,
                                                                  uint32_t tile_cap,
                                                                  uint32_t scap) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
  DecodeArgs b = a;  // the schema tables after the wire tile
  b.sc = stage_schema(a.sc, (uint32_t*)(tile + tile_cap + 16), scap);
  const uint64_t r0 = (uint64_t)blockIdx.x * 256;
  const uint64_t r1 = min(r0 + 256, a.n);
  const uint64_t b0 = a.offs[r0], b1 = a.offs[r1];
  const uint64_t a0 = b0 & ~15ull;
  const bool staged = b0 <= b1 && b1 <= a.in_len && b1 - a0 <= tile_cap;
  if (staged) {
    const uint32_t nvec = (uint32_t)((b1 - a0 + 15) >> 4);
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
  // one decode_record call site (the copy, then HBM when the copy failed)
  Reader r;
  for (int from_lds = staged ? 1 : 0;; from_lds = 0) {
    r = decode_record<P>(b, i, -1, kIndexed, from_lds ? tile : nullptr, a0, b1);
    if (!from_lds || r.ok() || r.err == kErrDeep) break;
  }
  if (!r.ok()) defer_or_fail(r, a.deep, &a.res->first_fail, i);
}

// The records the bulk passes deferred (a skip nested past the private
// frames): each lane keeps max_depth frames in HBM. With a wide tier
// (a.deep.wlanes), `wide` reads the deferred list on its wlanes lanes of
// kWideFrames frames and passes a record nesting deeper still (kErrDeep from
// its full slab) to list2, which the max_depth lanes then read.
template <int P>
__global__ __launch_bounds__(64) void deep_decode_kernel(DecodeArgs a, int wide) {
  const uint32_t lane = blockIdx.x * 64 + threadIdx.x;
  DecodeArgs b = a;
  const uint64_t* list = a.deep.list;
  uint64_t m;
  if (wide) {
    b.deep.slabs = a.deep.wslabs;
    b.deep.slab_frames = kWideFrames;
    b.deep.lanes = a.deep.wlanes;
    b.deep.more = 1;
    m = *a.deep.count;
  } else if (a.deep.wlanes) {
    list = a.deep.list2;
    m = *a.deep.count2;
  } else {
    m = *a.deep.count;
  }
  if (lane >= b.deep.lanes) return;
  for (uint64_t k = lane; k < m; k += b.deep.lanes) {
    const uint64_t i = list[k];
    const Reader r = decode_one<P>(b, i, (int)lane);
    if (r.ok()) continue;
    if (wide && r.err == kErrDeep) a.deep.list2[atomicAdd(a.deep.count2, 1ull)] = i;
    else atomicMin(&a.res->first_fail, (unsigned long long)i);
  }
}

// Fixed-stride batches (Binary, fixed-layout schema): the records the fast
// kernel could not take (its exception list: fields reordered, a bool byte
// above 1, ...) are read by the general reader at their stride position i * L.
// One that reads exactly L bytes keeps every later record in place; one that
// does not (other length, reader error, a skip nested past the private
// frames) moves first_misfit, from where the caller re-reads the stream
// (index or serial path), which also reports any error exactly. A list that
// overflowed (n_irregular > cap) is left alone: first_irregular stands.
template <int P>
__global__ __launch_bounds__(256) void fixed_exception_kernel(DecodeArgs a, uint64_t L) {
  const unsigned long long cnt = a.res->n_irregular;
  if (cnt > a.exc_cap) return;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < cnt; k += stride) {
    const uint64_t i = a.exc[k];
    if (i >= a.n) continue;
    const Reader r = decode_record<P>(a, i, -1, i * L);
    if (!r.ok() || r.pos != i * L + L) atomicMin(&a.res->first_misfit, (unsigned long long)i);
  }
}

__global__ void fixed_exception_resolve_kernel(DevResult* res, uint64_t cap) {
  if (res->n_irregular <= cap) res->first_irregular = res->first_misfit;
  res->n_irregular = 0;
  res->first_misfit = kNone;
}

// Stream-ordered form of the resolve step: then, when record m =
// first_irregular is off the stride (or the list overflowed), record m's
// length L2 by the general reader at m * L. A stream whose records all carry
// the same appended fields from m on continues at stride L2 — the strided tail
// decode takes it in parallel; no usable L2 (m fails, or L2 > max_stride, the
// tail decode's tile) leaves the walk from m to the finish kernel.
template <int P>
__global__ void fixed_tail_setup_kernel(DecodeArgs a, uint64_t cap, uint64_t L,
                                        uint64_t max_stride) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DevResult* res = a.res;
  if (res->n_irregular <= cap) res->first_irregular = res->first_misfit;
  res->n_irregular = 0;
  res->first_misfit = kNone;
  const uint64_t m = res->first_irregular;
  if (m >= a.n || !max_stride) return;
  const uint64_t p0 = m * L;
  const Reader r = decode_record<P>(a, m, -1, p0);
  if (!r.ok() || r.pos <= p0 || r.pos - p0 > max_stride) return;
  res->tail_first = m;
  res->tail_pos = p0;
  res->tail_min = kNone;
  res->tail_stride = r.pos - p0;
}

// Stream-ordered fixed-layout calls, last step (one workgroup): the strided
// tail decode's exception records read by the general reader at their stride
// positions (one not exactly L2 long, or failing, is a misfit; an overflowed
// list leaves tail_min), then one lane walks record boundaries from the first
// record off the strides — the reference's sequential deserialize<T>(Cursor&)
// loop (Serializer.h:97-100) — writing offs. Without a strided tail the walk
// starts at first_irregular.
template <int P>
__global__ __launch_bounds__(256) void fixed_stream_finish_kernel(DecodeArgs a, uint64_t cap,
                                                                  uint64_t L) {
  __shared__ unsigned long long from_s;
  DevResult* res = a.res;
  const uint64_t L2 = res->tail_stride, m = res->tail_first, p0 = res->tail_pos;
  if (threadIdx.x == 0) from_s = L2 ? kNone : res->first_irregular;
  __syncthreads();
  if (L2) {
    const unsigned long long cnt = res->n_irregular;
    if (cnt > cap) {
      if (threadIdx.x == 0) from_s = res->tail_min;
    } else {
      for (uint64_t k = threadIdx.x; k < cnt; k += blockDim.x) {
        const uint64_t i = a.exc[k];
        if (i >= a.n) continue;
        const uint64_t at = p0 + (i - m) * L2;
        const Reader r = decode_record<P>(a, i, -1, at);
        if (!r.ok() || r.pos != at + L2) atomicMin(&from_s, (unsigned long long)i);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const uint64_t first = from_s;
  if (first >= a.n) return;
  uint64_t* offs = const_cast<uint64_t*>(a.offs);
  uint64_t pos = L2 ? p0 + (first - m) * L2 : first * L;
  for (uint64_t i = first; i < a.n; ++i) {
    offs[i] = pos;
    const Reader r = decode_one<P>(a, i);
    if (!r.ok()) {
      atomicMin(&a.res->first_fail, (unsigned long long)i);
      return;
    }
    pos = r.pos;
  }
  offs[a.n] = pos;
}

// Record 0 of a fixed-stride batch read at 0: first_misfit = 0 unless it is
// exactly L bytes (the plan kernel's work is wasted on a stream whose stride
// is not L, e.g. every record carrying a field the schema does not know).
template <int P>
__global__ void fixed_probe_kernel(DecodeArgs a, uint64_t L) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const Reader r = decode_record<P>(a, 0, -1, 0);
  a.res->first_misfit = (r.ok() && r.pos == L) ? kNone : 0;
  a.res->total_bytes = r.ok() ? r.pos : 0;  // record 0's length (the caller's second stride)
}

template <int P>
__global__ void decode_finish_kernel(DecodeArgs a, uint64_t fixed_len) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DevResult* res = a.res;
  const uint64_t f = res->first_fail;
  const uint64_t irr = res->first_irregular;
  // start offset of record i (fixed path: i * L below the first irregular one)
  auto start_of = [&](uint64_t i) -> uint64_t {
    if (fixed_len && i <= irr && irr != kNone) return i * fixed_len;
    if (fixed_len && irr == kNone) return i * fixed_len;
    return a.offs[i];
  };
  const uint64_t base = start_of(0);
  if (f < a.n) {
    const Reader r = decode_one<P>(a, f);
    res->code = r.ok() ? TGPU_ERR_INDEX_MISMATCH : r.err;
    res->fail_offset = r.ok() ? r.pos : r.err_off;
    res->n_records = f;
    res->total_bytes = start_of(f) - base;
  } else {
    res->code = 0;
    res->n_records = a.n;
    res->total_bytes = (fixed_len && irr == kNone) ? a.n * fixed_len : a.offs[a.n] - base;
  }
}

// Status of a fixed-layout batch whose tail [rec_base, n) was indexed and
// decoded after its first non-canonical record: `a` covers the tail (records,
// offsets and indices relative to rec_base; offsets are absolute stream
// positions of a stream that starts at 0).
template <int P>
__global__ void tail_decode_finish_kernel(DecodeArgs a, uint64_t rec_base) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DevResult* res = a.res;
  const uint64_t f = res->first_fail;
  if (f < a.n) {
    const Reader r = decode_one<P>(a, f);
    res->code = r.ok() ? TGPU_ERR_INDEX_MISMATCH : r.err;
    res->fail_offset = r.ok() ? r.pos : r.err_off;
    res->first_fail = rec_base + f;
    res->n_records = rec_base + f;
    res->total_bytes = a.offs[f];
  } else {
    res->code = 0;
    res->first_fail = kNone;
    res->n_records = rec_base + a.n;
    res->total_bytes = a.offs[a.n];
  }
}

// After a fused index + decode of a stream range (tgpu_decode_stream): the
// index left n_records / total_bytes / first_start (and a reader error's
// code); a record it accepted that the decode could not store (list arena
// overflow) is re-diagnosed here and ends the range.
template <int P>
__global__ void stream_decode_finish_kernel(DecodeArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DevResult* res = a.res;
  const uint64_t f = res->first_fail;
  if (f < res->n_records) {
    const Reader r = decode_one<P>(a, f);
    res->code = r.ok() ? TGPU_ERR_INDEX_MISMATCH : r.err;
    res->fail_offset = r.ok() ? r.pos : r.err_off;
    res->n_records = f;
    res->total_bytes = a.offs[f];
  }
}

// ------------------------------------------------------------------ encode --
// lane >= 0: the deep-pass lane whose HBM frames the writer may use.
__device__ __forceinline__ void attach_slab(Writer& w, const DeepArgs& d, int lane) {
  if (lane < 0 || !d.slabs) return;
  w.deep = d.slabs + (uint64_t)lane * slab_lane_bytes(d.slab_frames);
  w.deep_cap = d.slab_frames;
  w.deep_more = d.more != 0;
}

// A deep encode pass's tier (deep_decode_kernel's two tiers): the wide one
// (wide != 0) reads the deferred list with the wide slabs; the max_depth
// one reads list2 when there is a wide tier, else the deferred list.
__device__ __forceinline__ EncodeArgs deep_tier(const EncodeArgs& a, int wide,
                                                const uint64_t*& list, uint64_t& m) {
  EncodeArgs b = a;
  list = a.deep.list;
  if (wide) {
    b.deep.slabs = a.deep.wslabs;
    b.deep.slab_frames = kWideFrames;
    b.deep.lanes = a.deep.wlanes;
    b.deep.more = 1;
    m = *a.deep.count;
  } else if (a.deep.wlanes) {
    list = a.deep.list2;
    m = *a.deep.count2;
  } else {
    m = *a.deep.count;
  }
  return b;
}

// Size of record i; lane >= 0: a deep-pass lane (HBM frames).
template <int P>
__device__ __forceinline__ Writer size_one(const EncodeArgs& a, uint64_t i, int lane = -1) {
  Writer w{nullptr, 0, 0, 0, 0};
  if (lane >= 0 && a.deep.slabs) {
    attach_slab(w, a.deep, lane);
    write_record<P, true>(w, a.sc, a.recs + i * a.rec_size, a.sbase, a.lbase);
  } else {
    write_record<P>(w, a.sc, a.recs + i * a.rec_size, a.sbase, a.lbase);
  }
  return w;
}

__device__ __forceinline__ unsigned long long block_sum(unsigned long long v) {
  __shared__ unsigned long long part[4];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) part[wid] = v;
  __syncthreads();
  unsigned long long t = 0;
  if (threadIdx.x == 0) t = part[0] + part[1] + part[2] + part[3];
  return t;
}

// Block-wide exclusive scan (256 threads).
__device__ __forceinline__ unsigned long long block_exscan(unsigned long long v) {
  __shared__ unsigned long long part[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) part[wid] = x;
  __syncthreads();
  unsigned long long pre = 0;
  for (int w = 0; w < wid; ++w) pre += part[w];
  return pre + x - v;
}

// A record nested past the private frames is sized 0 here and deferred: the
// deep size pass adds its size to its tile's sum before the scan.
template <int P>
__global__ __launch_bounds__(256) void encode_size_kernel(EncodeArgs a, uint32_t scap) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sch[];
  EncodeArgs b = a;
  b.sc = stage_schema(a.sc, sch, scap);
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  unsigned long long sz = 0;
  if (i < a.n) {
    const Writer w = size_one<P>(b, i);
    if (w.err == kErrDeep) a.deep.list[atomicAdd(a.deep.count, 1ull)] = i;
    else if (!w.ok()) atomicMin(&a.res->first_fail, (unsigned long long)i);
    else sz = w.pos;
    a.offs[i] = sz;
  }
  const unsigned long long t = block_sum(sz);
  if (threadIdx.x == 0) a.block_sums[blockIdx.x] = t;
}

// (the wide tier hands a record nesting past its slab to list2, sized by
// the max_depth tier)
template <int P>
__global__ __launch_bounds__(64) void deep_size_kernel(EncodeArgs a, int wide) {
  const uint32_t lane = blockIdx.x * 64 + threadIdx.x;
  const uint64_t* list;
  uint64_t m;
  const EncodeArgs b = deep_tier(a, wide, list, m);
  if (lane >= b.deep.lanes) return;
  for (uint64_t k = lane; k < m; k += b.deep.lanes) {
    const uint64_t i = list[k];
    const Writer w = size_one<P>(b, i, (int)lane);
    if (wide && w.err == kErrDeep) {
      a.deep.list2[atomicAdd(a.deep.count2, 1ull)] = i;
      continue;
    }
    if (!w.ok()) {
      atomicMin(&a.res->first_fail, (unsigned long long)i);
      continue;
    }
    a.offs[i] = w.pos;
    atomicAdd(&a.block_sums[i / 256], (unsigned long long)w.pos);
  }
}

template <int P>
__global__ __launch_bounds__(256) void encode_write_kernel(EncodeArgs a, uint32_t scap) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sch[];
  const DevSchema sc = stage_schema(a.sc, sch, scap);
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const unsigned long long sz = i < a.n ? a.offs[i] : 0;
  const unsigned long long start = a.block_sums[blockIdx.x] + block_exscan(sz);
  if (i >= a.n) return;
  a.offs[i] = start;
  if (start + sz > a.cap) {
    atomicMin(&a.res->first_fail, (unsigned long long)i);
    return;
  }
  // (a deferred record stops at its private frames; the deep write pass
  // writes it whole)
  Writer w{a.out, start, a.cap, 0, 0};
  write_record<P>(w, sc, a.recs + i * a.rec_size, a.sbase, a.lbase);
}

// (the wide tier stops at a record its size pass handed on — same record,
// same frames, same verdict — and the max_depth tier writes it whole)
template <int P>
__global__ __launch_bounds__(64) void deep_write_kernel(EncodeArgs a, int wide) {
  const uint32_t lane = blockIdx.x * 64 + threadIdx.x;
  const uint64_t* list;
  uint64_t m;
  const EncodeArgs b = deep_tier(a, wide, list, m);
  if (lane >= b.deep.lanes) return;
  for (uint64_t k = lane; k < m; k += b.deep.lanes) {
    const uint64_t i = list[k];
    const uint64_t start = a.offs[i];
    if (a.res->first_fail <= i) continue;
    Writer w{a.out, start, a.cap, 0, 0};
    attach_slab(w, b.deep, (int)lane);
    write_record<P, true>(w, a.sc, a.recs + i * a.rec_size, a.sbase, a.lbase);
  }
}

// sizes -> exclusive offsets (block-local scan + scanned block sums)
__global__ __launch_bounds__(256) void size_offsets_kernel(EncodeArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const unsigned long long sz = i < a.n ? a.offs[i] : 0;
  const unsigned long long start = a.block_sums[blockIdx.x] + block_exscan(sz);
  if (i < a.n) a.offs[i] = start;
}

template <int P>
__global__ void encode_finish_kernel(EncodeArgs a, uint64_t fixed_len) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DevResult* res = a.res;
  const uint64_t f = res->first_fail;
  if (f < a.n) {
    const Writer w = size_one<P>(a, f, a.deep.slabs ? 0 : -1);
    const uint64_t start = fixed_len ? f * fixed_len : a.offs[f];
    res->code = w.ok() ? TGPU_ERR_OUTPUT_OVERFLOW : w.err;
    res->fail_offset = start + (w.ok() ? 0 : w.err_off);
    res->n_records = f;
    res->total_bytes = start;
  } else {
    res->code = 0;
    res->n_records = a.n;
    res->total_bytes = fixed_len ? a.n * fixed_len : a.offs[a.n];
  }
}

// Dynamic LDS for the schema tables of a general kernel (0: they stay in
// global memory, when larger than 16 KiB).
uint32_t schema_stage_bytes(const DevSchema& sc) {
  const uint32_t b = sc.ns * (uint32_t)sizeof(tgpu_struct_desc) +
                     sc.nf * (uint32_t)sizeof(tgpu_field_desc) +
                     sc.nt * (uint32_t)sizeof(tgpu_type_desc);
  return b <= 16 * 1024 ? (b + 15) & ~15u : 0;
}

uint32_t grid_for(uint64_t n) {
  const uint64_t b = (n + 255) / 256;
  return (uint32_t)(b < 4096 ? (b ? b : 1) : 4096);
}

}  // namespace

hipError_t launch_result_init(DevResult* res, uint64_t n, hipStream_t stream) {
  hipLaunchKernelGGL(result_init_kernel, dim3(1), dim3(1), 0, stream, res, n);
  return hipGetLastError();
}

hipError_t launch_general_decode(const DecodeArgs& a, int protocol, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  if (a.offs && !getenv("TGPU_GENERAL_HBM")) {
    // LDS tile for 256 records of the stream's mean size, with slack
    const uint64_t mean = (a.in_len + a.n - 1) / a.n;
    const uint64_t want = ((mean * 256 * 5 / 4 + 15) & ~15ull) + 32;
    // (cap + 16 bytes of dynamic LDS stay within 64 KiB per workgroup)
    // (cap + 16 + the schema tables stay within 64 KiB per workgroup)
    const uint32_t sb = schema_stage_bytes(a.sc);
    const uint32_t cap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(want, 4096),
                                                      64 * 1024 - 16 - sb) & ~15u;
    const uint64_t blocks = (a.n + 255) / 256;
    TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(general_decode_tile_kernel<P_>,
                                                  dim3((uint32_t)blocks), dim3(256), cap + 16 + sb,
                                                  stream, a, cap, sb));
    return hipGetLastError();
  }
  const uint32_t g = grid_for(a.n);
  const uint32_t sb = schema_stage_bytes(a.sc);
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(general_decode_kernel<P_>, dim3(g), dim3(256), sb,
                                                stream, a, sb));
  return hipGetLastError();
}

hipError_t launch_fixed_exceptions(const DecodeArgs& a, int protocol, uint64_t L,
                                   hipStream_t stream) {
  // a small grid striding over the list: usually empty, and a launch of
  // thousands of workgroups that only read the count cost 29 us
  const uint64_t most = a.exc_cap < a.n ? a.exc_cap : a.n;
  const uint32_t g = (uint32_t)std::min<uint64_t>((most + 255) / 256, 256);
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(fixed_exception_kernel<P_>, dim3(g ? g : 1),
                                                dim3(256), 0, stream, a, L));
  hipLaunchKernelGGL(fixed_exception_resolve_kernel, dim3(1), dim3(1), 0, stream, a.res, a.exc_cap);
  return hipGetLastError();
}

hipError_t launch_fixed_exceptions_stream(const DecodeArgs& a, int protocol, uint64_t L,
                                          uint64_t max_stride, hipStream_t stream) {
  const uint64_t most = a.exc_cap < a.n ? a.exc_cap : a.n;
  const uint32_t g = (uint32_t)std::min<uint64_t>((most + 255) / 256, 256);
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(fixed_exception_kernel<P_>, dim3(g ? g : 1),
                                                dim3(256), 0, stream, a, L));
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(fixed_tail_setup_kernel<P_>, dim3(1), dim3(64), 0,
                                                stream, a, a.exc_cap, L, max_stride));
  return hipGetLastError();
}

hipError_t launch_fixed_stream_finish(const DecodeArgs& a, int protocol, uint64_t L,
                                      hipStream_t stream) {
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(fixed_stream_finish_kernel<P_>, dim3(1), dim3(256),
                                                0, stream, a, a.exc_cap, L));
  return hipGetLastError();
}

hipError_t launch_fixed_probe(const DecodeArgs& a, int protocol, uint64_t L, hipStream_t stream) {
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(fixed_probe_kernel<P_>, dim3(1), dim3(64), 0,
                                                stream, a, L));
  return hipGetLastError();
}

hipError_t launch_deep_decode(const DecodeArgs& a, int protocol, hipStream_t stream) {
  if (!a.deep.lanes) return hipSuccess;
  if (a.deep.wlanes)  // the wide tier first (its lanes return at once when none was deferred)
    TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(deep_decode_kernel<P_>,
                                                  dim3((a.deep.wlanes + 63) / 64), dim3(64), 0,
                                                  stream, a, 1));
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(deep_decode_kernel<P_>, dim3((a.deep.lanes + 63) / 64),
                                                dim3(64), 0, stream, a, 0));
  return hipGetLastError();
}

hipError_t launch_decode_finish(const DecodeArgs& a, int protocol, uint64_t fixed_len,
                                hipStream_t stream) {
  const hipError_t e = launch_deep_decode(a, protocol, stream);
  if (e != hipSuccess) return e;
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(decode_finish_kernel<P_>, dim3(1), dim3(64), 0, stream, a,
                       fixed_len));
  return hipGetLastError();
}

hipError_t launch_stream_decode_finish(const DecodeArgs& a, int protocol, hipStream_t stream) {
  const hipError_t e = launch_deep_decode(a, protocol, stream);
  if (e != hipSuccess) return e;
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(stream_decode_finish_kernel<P_>, dim3(1), dim3(64), 0,
                       stream, a));
  return hipGetLastError();
}

hipError_t launch_tail_decode_finish(const DecodeArgs& a, int protocol, uint64_t rec_base,
                                     hipStream_t stream) {
  const hipError_t e = launch_deep_decode(a, protocol, stream);
  if (e != hipSuccess) return e;
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(tail_decode_finish_kernel<P_>, dim3(1), dim3(64), 0,
                                                stream, a, rec_base));
  return hipGetLastError();
}

// The deep passes of the general encode (a record nested past the private
// frames): launched on every call, their lanes exit on an empty list.
hipError_t launch_deep_size(const EncodeArgs& a, int protocol, hipStream_t stream) {
  if (!a.deep.lanes) return hipSuccess;
  if (a.deep.wlanes)
    TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(deep_size_kernel<P_>,
                                                  dim3((a.deep.wlanes + 63) / 64), dim3(64), 0,
                                                  stream, a, 1));
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(deep_size_kernel<P_>, dim3((a.deep.lanes + 63) / 64),
                                                dim3(64), 0, stream, a, 0));
  return hipGetLastError();
}

// The deep pass's writes (wide tier first, then the max_depth tier).
hipError_t launch_deep_write(const EncodeArgs& a, int protocol, hipStream_t stream) {
  if (a.deep.lanes && a.deep.wlanes)
    TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(deep_write_kernel<P_>,
                                                  dim3((a.deep.wlanes + 63) / 64), dim3(64), 0,
                                                  stream, a, 1));
  if (a.deep.lanes)
    TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(deep_write_kernel<P_>, dim3((a.deep.lanes + 63) / 64),
                                                  dim3(64), 0, stream, a, 0));
  return hipGetLastError();
}

hipError_t launch_general_encode(const EncodeArgs& a, int protocol, uint64_t n_blocks,
                                 hipStream_t stream, const JitKernels* nj, bool defer) {
  if (a.n == 0) return hipSuccess;
  const dim3 grid((uint32_t)n_blocks);
  const uint32_t sb = schema_stage_bytes(a.sc);
  if (nj) {  // the nested program's passes
    hipError_t e = jit_launch_encode(nj, false, a, n_blocks, 0, stream, 2);
    // (a recursive schema's unrolled writer: the records it deferred)
    if (e == hipSuccess && defer) e = launch_deep_size(a, protocol, stream);
    if (e == hipSuccess)
      e = launch_scan_tiles(a.block_sums, n_blocks, a.scan_part, &a.res->total_bytes,
                            a.offs + a.n, stream);
    // (a.out_cap: the write pass's LDS output tile, 0 = none)
    if (e == hipSuccess)
      e = jit_launch_encode(nj, true, a, n_blocks, a.out_cap ? a.out_cap + 16 : 0, stream, 2);
    if (e == hipSuccess && defer) e = launch_deep_write(a, protocol, stream);
    return e;
  }
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(encode_size_kernel<P_>, grid, dim3(256), sb, stream, a,
                                                sb));
  hipError_t e = launch_deep_size(a, protocol, stream);
  if (e != hipSuccess) return e;
  e = launch_scan_tiles(a.block_sums, n_blocks, a.scan_part, &a.res->total_bytes, a.offs + a.n,
                        stream);
  if (e != hipSuccess) return e;
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(encode_write_kernel<P_>, grid, dim3(256), sb, stream, a,
                                                sb));
  return launch_deep_write(a, protocol, stream);
}

hipError_t launch_general_size(const EncodeArgs& a, int protocol, uint64_t n_blocks,
                               hipStream_t stream, const JitKernels* nj, bool defer) {
  if (a.n == 0) return hipSuccess;
  const dim3 grid((uint32_t)n_blocks);
  const uint32_t sb = schema_stage_bytes(a.sc);
  hipError_t e;
  if (nj) {
    e = jit_launch_encode(nj, false, a, n_blocks, 0, stream, 2);
    if (e == hipSuccess && defer) e = launch_deep_size(a, protocol, stream);
  } else {
    TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(encode_size_kernel<P_>, grid, dim3(256), sb, stream,
                                                  a, sb));
    e = launch_deep_size(a, protocol, stream);
  }
  if (e != hipSuccess) return e;
  e = launch_scan_tiles(a.block_sums, n_blocks, a.scan_part, &a.res->total_bytes, a.offs + a.n,
                        stream);
  if (e != hipSuccess) return e;
  return launch_size_offsets(a, n_blocks, stream);
}

hipError_t launch_size_offsets(const EncodeArgs& a, uint64_t n_blocks, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(size_offsets_kernel, dim3((uint32_t)n_blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_encode_finish(const EncodeArgs& a, int protocol, uint64_t fixed_len,
                                hipStream_t stream) {
  TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(encode_finish_kernel<P_>, dim3(1), dim3(64), 0, stream, a,
                       fixed_len));
  return hipGetLastError();
}

}  // namespace tgpu
