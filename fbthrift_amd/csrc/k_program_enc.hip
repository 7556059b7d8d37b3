// k_program_enc.hip — compiled-program encode of variable-length records
// (BASELINE configs 3 and 4 encode), plus the multi-block scan of per-tile
// byte counts shared with the general encoder.
//
// The schema's VProgram (tgpu_api.cpp build_program) is the canonical wire
// form the generated T::write emits for an all-unqualified schema: fields in
// declaration order (serialize_struct.whisker:40-67), each header
// (BinaryProtocol-inl.h:41-67 / CompactProtocol-inl.h:133-180) then its value
// (BinaryProtocol-inl.h:120-222 / CompactProtocol-inl.h:252-373).
//
// Three launches, one record per lane, 256-record tiles:
//   1. program_size_kernel  — record tile HBM -> LDS (16-byte loads); each
//      lane sizes its record; sizes -> out_offsets[i]; tile sum -> sums[t];
//      validation failures (validate_bool, > INT32_MAX sizes) -> first_fail.
//   2. scan of the tile sums (scan_tiles_*: reduce, top-level scan, apply).
//   3. program_write_kernel — record tile -> LDS again, block exclusive scan
//      of the sizes gives each lane its position in the tile; the lane emits
//      its record into an LDS output tile (records past the LDS cap go to HBM
//      directly); the tile leaves with coalesced 16-byte stores (byte stores
//      only on the two edge chunks shared with the neighbouring tiles).
#include "tgpu_device.h"

namespace tgpu {
namespace {

constexpr uint32_t kET = 256;               // records per tile = threads per workgroup
constexpr uint32_t kOutCap = 24 * 1024;     // LDS bytes for one tile's wire output

__device__ __forceinline__ uint32_t varint_len(uint64_t v) {
  const uint32_t bits = 64 - (uint32_t)__builtin_clzll(v | 1);
  return (bits + 6) / 7;
}

__device__ __forceinline__ uint64_t load_member(const uint8_t* p, uint32_t width) {
  switch (width) {
    case 8: return *(const uint64_t*)p;
    case 4: return *(const uint32_t*)p;
    case 2: return *(const uint16_t*)p;
    default: return *p;
  }
}

// zigzag of a signed member of `width` bytes, as i32 (bits 32) or i64
__device__ __forceinline__ uint64_t zz_member(uint64_t raw, uint32_t width, uint32_t bits) {
  int64_t v;
  switch (width) {
    case 2: v = (int16_t)(uint16_t)raw; break;
    case 4: v = (int32_t)(uint32_t)raw; break;
    default: v = (int64_t)raw; break;
  }
  if (bits == 32) return dev::i32_to_zz((int32_t)v);
  return dev::i64_to_zz(v);
}

// ---- record size ------------------------------------------------------------
// Bytes T::write emits for the record at `rec`; ok = false where the writer
// would throw or abort (the finish kernel re-derives the exact code).
__device__ uint64_t program_size(const VProgram* __restrict__ P, const uint8_t* rec,
                                 const uint8_t* __restrict__ lbase, bool& ok) {
  const bool compact = P->protocol == TGPU_PROTOCOL_COMPACT;
  const uint32_t n_ops = P->n_ops;
  uint64_t n = 0;
  for (uint32_t k = 0; k < n_ops; ++k) {
    const VOp op = P->ops[k];
    switch (op.kind) {
      case VOP_CONST:
        n += op.hdr_len;
        break;
      case VOP_CBOOL:
        if (rec[op.member] > 1) ok = false;
        n += op.hdr_len;
        break;
      case VOP_FIXED:
        if (op.is_bool && rec[op.member] > 1) ok = false;
        n += op.width;
        break;
      case VOP_VARINT:
        n += varint_len(zz_member(load_member(rec + op.member, op.width), op.width, op.bits));
        break;
      case VOP_STRING: {
        const uint32_t len = ((const tgpu_span*)(rec + op.member))->length;
        if (len > 0x7fffffffu) ok = false;
        n += (compact ? varint_len(len) : 4) + (uint64_t)len;
        break;
      }
      case VOP_LIST: {
        const tgpu_span sp = *(const tgpu_span*)(rec + op.member);
        const uint32_t len = sp.length;
        if (len > 0x7fffffffu) {
          ok = false;
          break;
        }
        n += compact ? (len <= 14 ? 1 : 1 + varint_len(len)) : 5;
        const uint8_t* e = lbase + sp.offset;
        if (op.elem_kind == VEL_VARINT) {
          for (uint32_t i = 0; i < len; ++i)
            n += varint_len(zz_member(load_member(e + (uint64_t)i * op.width, op.width), op.width,
                                      op.bits));
        } else if (op.elem_kind == VEL_BOOL) {
          for (uint32_t i = 0; i < len; ++i)
            if (e[i] > 1) ok = false;
          n += len;
        } else {
          n += (uint64_t)len * op.width;
        }
        break;
      }
      default:
        break;
    }
  }
  return n;
}

// ---- record emission ----------------------------------------------------------
// Sinks: the LDS output tile (position q relative to the tile's LDS base) or
// HBM directly (q relative to the record's HBM start).
struct LdsSink {
  uint8_t* base;
  __device__ __forceinline__ void put(uint32_t q, uint32_t b) const { base[q] = (uint8_t)b; }
};
struct HbmSink {
  uint8_t* base;
  __device__ __forceinline__ void put(uint32_t q, uint32_t b) const { base[q] = (uint8_t)b; }
};

template <class Sink>
__device__ __forceinline__ uint32_t put_be(const Sink& s, uint32_t q, uint64_t v, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) s.put(q + i, (uint32_t)(v >> (8 * (n - 1 - i))));
  return q + n;
}
template <class Sink>
__device__ __forceinline__ uint32_t put_varint(const Sink& s, uint32_t q, uint64_t v) {
  while (v & ~0x7full) {
    s.put(q++, (uint32_t)((v & 0x7f) | 0x80));
    v >>= 7;
  }
  s.put(q++, (uint32_t)v);
  return q;
}
// len bytes from HBM (any alignment): aligned dword loads, bytes out
template <class Sink>
__device__ __forceinline__ uint32_t put_bytes(const Sink& s, uint32_t q,
                                              const uint8_t* __restrict__ src, uint32_t len) {
  if (!len) return q;
  const uintptr_t a = (uintptr_t)src;
  const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
  uint32_t sh = (uint32_t)(a & 3);
  uint32_t i = 0;
  while (i < len) {
    const uint32_t word = *w++;
    for (uint32_t b = sh; b < 4 && i < len; ++b, ++i) s.put(q + i, (word >> (8 * b)) & 0xff);
    sh = 0;
  }
  return q + len;
}

template <class Sink>
__device__ void program_emit(const VProgram* __restrict__ P, const uint8_t* rec,
                             const uint8_t* __restrict__ sbase, const uint8_t* __restrict__ lbase,
                             const Sink& s) {
  const bool compact = P->protocol == TGPU_PROTOCOL_COMPACT;
  const uint32_t n_ops = P->n_ops;
  uint32_t q = 0;
  for (uint32_t k = 0; k < n_ops; ++k) {
    const VOp op = P->ops[k];
    switch (op.kind) {
      case VOP_CONST:
        for (uint32_t i = 0; i < op.hdr_len; ++i) s.put(q + i, (op.hdr >> (8 * i)) & 0xff);
        q += op.hdr_len;
        break;
      case VOP_CBOOL: {
        // the bool's value rides in the header's type nibble (CT_BOOLEAN_TRUE/FALSE)
        const uint32_t h = op.hdr | (rec[op.member] ? 1u : 2u);
        for (uint32_t i = 0; i < op.hdr_len; ++i) s.put(q + i, (h >> (8 * i)) & 0xff);
        q += op.hdr_len;
        break;
      }
      case VOP_FIXED:
        q = put_be(s, q, load_member(rec + op.member, op.width), op.width);
        break;
      case VOP_VARINT:
        q = put_varint(s, q, zz_member(load_member(rec + op.member, op.width), op.width, op.bits));
        break;
      case VOP_STRING: {
        const tgpu_span sp = *(const tgpu_span*)(rec + op.member);
        q = compact ? put_varint(s, q, sp.length) : put_be(s, q, sp.length, 4);
        q = put_bytes(s, q, sbase + sp.offset, sp.length);
        break;
      }
      case VOP_LIST: {
        const tgpu_span sp = *(const tgpu_span*)(rec + op.member);
        const uint32_t len = sp.length;
        if (compact) {
          if (len <= 14) {
            s.put(q++, (len << 4) | op.elem_ct);
          } else {
            s.put(q++, 0xf0 | op.elem_ct);
            q = put_varint(s, q, len);
          }
        } else {
          s.put(q++, op.elem_ttype);
          q = put_be(s, q, len, 4);
        }
        const uint8_t* e = lbase + sp.offset;
        if (op.elem_kind == VEL_VARINT) {
          for (uint32_t i = 0; i < len; ++i)
            q = put_varint(s, q, zz_member(load_member(e + (uint64_t)i * op.width, op.width),
                                           op.width, op.bits));
        } else if (op.elem_kind == VEL_BOOL) {
          for (uint32_t i = 0; i < len; ++i) s.put(q++, compact ? (e[i] ? 1u : 2u) : e[i]);
        } else {
          for (uint32_t i = 0; i < len; ++i)
            q = put_be(s, q, load_member(e + (uint64_t)i * op.width, op.width), op.width);
        }
        break;
      }
      default:
        break;
    }
  }
}

// ---- block helpers (256 threads) --------------------------------------------
__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long x) {
  const int lane = threadIdx.x & 63;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// exclusive scan across the block; *total = block sum (all threads)
__device__ __forceinline__ unsigned long long block_exscan256(unsigned long long v,
                                                              unsigned long long* part,
                                                              unsigned long long* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long x = wave_incl_scan(v);
  if (lane == 63) part[wid] = x;
  __syncthreads();
  unsigned long long pre = 0;
  for (int w = 0; w < wid; ++w) pre += part[w];
  *total = part[0] + part[1] + part[2] + part[3];
  return pre + x - v;
}

// Records [r0, r0+nrec) of stride S into LDS; returns the 16-byte phase.
__device__ __forceinline__ uint32_t stage_records(const uint8_t* recs, uint64_t r0, uint32_t nrec,
                                                  uint32_t S, uint8_t* rtile) {
  const uint8_t* g = recs + r0 * S;
  const uint32_t sh = (uint32_t)((uintptr_t)g & 15);
  const uint4* src = (const uint4*)(g - sh);
  const uint32_t nvec = (nrec * S + sh + 15) >> 4;
  for (uint32_t i = threadIdx.x; i < nvec; i += kET) ((uint4*)rtile)[i] = src[i];
  return sh;
}

__global__ __launch_bounds__(kET) void program_size_kernel(EncodeArgs a,
                                                           const VProgram* __restrict__ P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ unsigned long long part[4];
  const uint64_t r0 = (uint64_t)blockIdx.x * kET;
  const uint32_t S = a.rec_size;
  const uint32_t nrec = (uint32_t)min((uint64_t)kET, a.n - r0);
  const uint32_t sh = stage_records(a.recs, r0, nrec, S, smem);
  __syncthreads();
  unsigned long long sz = 0;
  if (threadIdx.x < nrec) {
    bool ok = true;
    sz = program_size(P, smem + sh + threadIdx.x * S, a.lbase, ok);
    if (!ok) atomicMin(&a.res->first_fail, (unsigned long long)(r0 + threadIdx.x));
    a.offs[r0 + threadIdx.x] = sz;
  }
  unsigned long long total;
  (void)block_exscan256(sz, part, &total);
  if (threadIdx.x == 0) a.block_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kET) void program_write_kernel(EncodeArgs a,
                                                            const VProgram* __restrict__ P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ unsigned long long part[4];
  __shared__ unsigned int lds_end;
  const uint64_t r0 = (uint64_t)blockIdx.x * kET;
  const uint32_t S = a.rec_size;
  const uint32_t nrec = (uint32_t)min((uint64_t)kET, a.n - r0);
  uint8_t* rtile = smem;
  uint8_t* otile = smem + ((kET * S + 16 + 15) & ~15u);
  const uint32_t rsh = stage_records(a.recs, r0, nrec, S, rtile);
  const uint32_t r = threadIdx.x;
  const unsigned long long sz = r < nrec ? a.offs[r0 + r] : 0;
  unsigned long long tile_total;
  const unsigned long long rel = block_exscan256(sz, part, &tile_total);
  const unsigned long long tile_base = a.block_sums[blockIdx.x];
  if (r == 0) lds_end = (unsigned int)min(tile_total, (unsigned long long)kOutCap);
  __syncthreads();  // record tile staged, lds_end initialised
  uint8_t* gtile = a.out + tile_base;
  const uint32_t osh = (uint32_t)((uintptr_t)gtile & 15);
  bool fits = false;
  if (r < nrec) {
    const unsigned long long start = tile_base + rel;
    a.offs[r0 + r] = start;
    if (start + sz > a.cap) {
      atomicMin(&a.res->first_fail, (unsigned long long)(r0 + r));
      atomicMin(&lds_end, (unsigned int)min(rel, (unsigned long long)kOutCap));
    } else {
      fits = rel + sz <= kOutCap;
      if (!fits) atomicMin(&lds_end, (unsigned int)rel);
    }
  }
  __syncthreads();
  if (r < nrec) {
    const uint8_t* rec = rtile + rsh + r * S;
    if (fits && rel + sz <= lds_end) {
      program_emit(P, rec, a.sbase, a.lbase, LdsSink{otile + osh + (uint32_t)rel});
    } else if (tile_base + rel + sz <= a.cap) {
      program_emit(P, rec, a.sbase, a.lbase, HbmSink{gtile + rel});
    }
  }
  __syncthreads();
  // LDS tile [osh, osh + lds_end) -> HBM [gtile, gtile + lds_end)
  const uint32_t end = osh + lds_end;
  const uint32_t nvec = (end + 15) >> 4;
  uint8_t* gb = gtile - osh;
  for (uint32_t i = threadIdx.x; i < nvec; i += kET) {
    const uint32_t lo = i << 4, hi = lo + 16;
    if (lo >= osh && hi <= end) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(((const u32x4*)otile)[i], (u32x4*)gb + i);
    } else {
      for (uint32_t b = (lo < osh ? osh : lo); b < (hi < end ? hi : end); ++b) gb[b] = otile[b];
    }
  }
}

// ---- scan of per-tile sums (exclusive, in place; total -> res, offs[n]) ----
constexpr uint32_t kScanChunk = 2048;  // sums per workgroup (8 per thread)

__global__ __launch_bounds__(256) void scan_tiles_reduce(const unsigned long long* __restrict__ sums,
                                                         uint64_t nb,
                                                         unsigned long long* __restrict__ part) {
  __shared__ unsigned long long wp[4];
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanChunk;
  unsigned long long s = 0;
  for (uint32_t j = 0; j < kScanChunk / 256; ++j) {
    const uint64_t k = b0 + j * 256 + threadIdx.x;
    if (k < nb) s += sums[k];
  }
  unsigned long long total;
  (void)block_exscan256(s, wp, &total);
  if (threadIdx.x == 0) part[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void scan_tiles_top(unsigned long long* part, uint64_t np,
                                                       unsigned long long* total1,
                                                       uint64_t* total2) {
  __shared__ unsigned long long sm[1024];
  const uint64_t per = (np + 1023) / 1024;
  const uint64_t b = threadIdx.x * per, e = min(np, b + per);
  unsigned long long s = 0;
  for (uint64_t k = b; k < e; ++k) s += part[k];
  sm[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const unsigned long long y = threadIdx.x >= (unsigned)o ? sm[threadIdx.x - o] : 0;
    __syncthreads();
    sm[threadIdx.x] += y;
    __syncthreads();
  }
  unsigned long long run = sm[threadIdx.x] - s;
  for (uint64_t k = b; k < e; ++k) {
    const unsigned long long v = part[k];
    part[k] = run;
    run += v;
  }
  if (threadIdx.x == 1023) {
    if (total1) *total1 = sm[1023];
    if (total2) *total2 = sm[1023];
  }
}

__global__ __launch_bounds__(256) void scan_tiles_apply(unsigned long long* __restrict__ sums,
                                                        uint64_t nb,
                                                        const unsigned long long* __restrict__ part) {
  __shared__ unsigned long long wp[4];
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanChunk + threadIdx.x * (kScanChunk / 256);
  unsigned long long v[kScanChunk / 256];
  unsigned long long s = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanChunk / 256; ++j) {
    v[j] = b0 + j < nb ? sums[b0 + j] : 0;
    s += v[j];
  }
  unsigned long long total;
  unsigned long long run = part[blockIdx.x] + block_exscan256(s, wp, &total);
#pragma unroll
  for (uint32_t j = 0; j < kScanChunk / 256; ++j) {
    if (b0 + j < nb) sums[b0 + j] = run;
    run += v[j];
  }
}

}  // namespace

hipError_t launch_scan_tiles(unsigned long long* sums, uint64_t nb, unsigned long long* part,
                             unsigned long long* total1, uint64_t* total2, hipStream_t stream) {
  const uint64_t np = (nb + kScanChunk - 1) / kScanChunk;
  hipLaunchKernelGGL(scan_tiles_reduce, dim3((uint32_t)np), dim3(256), 0, stream, sums, nb, part);
  hipLaunchKernelGGL(scan_tiles_top, dim3(1), dim3(1024), 0, stream, part, np, total1, total2);
  hipLaunchKernelGGL(scan_tiles_apply, dim3((uint32_t)np), dim3(256), 0, stream, sums, nb, part);
  return hipGetLastError();
}

uint64_t scan_tiles_parts(uint64_t nb) { return (nb + kScanChunk - 1) / kScanChunk; }

bool program_encode_fits(uint32_t rec_size) {
  return kET * rec_size + 32 <= 32 * 1024;  // record tile + 24 KiB output tile <= 64 KiB LDS
}

hipError_t launch_program_encode(const EncodeArgs& a, const VProgram* d_prog,
                                 unsigned long long* part, bool size_only, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  const uint64_t tiles = (a.n + kET - 1) / kET;
  const uint32_t rt = (kET * a.rec_size + 16 + 15) & ~15u;
  hipLaunchKernelGGL(program_size_kernel, dim3((uint32_t)tiles), dim3(kET), rt, stream, a, d_prog);
  hipError_t e = launch_scan_tiles(a.block_sums, tiles, part, &a.res->total_bytes, a.offs + a.n,
                                   stream);
  if (e != hipSuccess || size_only) return e;
  hipLaunchKernelGGL(program_write_kernel, dim3((uint32_t)tiles), dim3(kET), rt + kOutCap + 32,
                     stream, a, d_prog);
  return hipGetLastError();
}

}  // namespace tgpu
