// k_arena.hip — the block rule's packing pass (round 6; ArenaPack in
// tgpu_internal.h, thrift_gpu.h tgpu_schema_arena_scale).
//
// The reference reads a list field into its own std::vector
// (protocol_methods.h:390-441 -> readArithmeticVector, BinaryProtocol.cpp:
// 49-72): the elements of one list are contiguous, and nothing else sits
// between them. The device decoders place each list's elements at scale x
// the wire position of its first element (the position rule: no scan, no
// record can reach another's slot), which leaves the arena as sparse as the
// wire. For flat-list schemas the batch's arrays are then packed per block of
// kArenaBlock records — records in order, a record's arrays in wire order,
// each 8-byte aligned, from align8(scale x the block's first wire byte) — so
// the arena holds the element arrays back to back. The compiled Binary decode
// tile packs each wave's block as it stores it (tgpu_prog_kernels.h
// pack_wave) and marks it; this pass packs every other block of a finished
// call: one wave per block, a lane per record.
//
// In place: an array's packed start is never above its source (each array
// is at most as long as the wire bytes it came from, and its own header
// bytes cover its alignment padding), so the block is moved in packed order
// in chunks that are read whole before any of them is written.
#include <algorithm>

#include "tgpu_device.h"
#include "tgpu_prog_kernels.h"

namespace tgpu {
namespace {

struct PackEnt {
  unsigned long long src;    // arena offset of the array (position rule)
  unsigned long long d;      // packed offset in the block
  unsigned long long bytes;  // array bytes (0: an empty list, after the record's arrays)
};

constexpr uint32_t kChunk = kArenaBlock * 16;  // packed bytes per read / write round (2 words a lane)

// One block (one wave: a lane per record) moved to the block rule.
__device__ __forceinline__ void pack_block(const DecodeArgs& a, const ArenaPack& p, uint64_t blk,
                                           uint64_t m, PackEnt* tab) {
  const uint64_t r0 = blk * kArenaBlock;
  const uint32_t nrec = (uint32_t)min((uint64_t)kArenaBlock, m - r0);
  const uint32_t r = threadIdx.x, K = p.n;
  uint8_t* rec = a.recs + (r0 + r) * a.rec_size;
  uint64_t off[kPackSlots], bytes[kPackSlots];
#pragma unroll
  for (uint32_t k = 0; k < kPackSlots; ++k) {
    off[k] = 0;
    bytes[k] = 0;
    if (k < K && r < nrec) {
      const tgpu_span sp = *(const tgpu_span*)(rec + p.member[k]);
      bytes[k] = (uint64_t)sp.length * p.es[k];
      off[k] = sp.offset;
    }
  }
  // wire order = source order (the position rule is monotone in the wire);
  // d[k]: the 8-byte aligned bytes of the record's arrays before array k
  uint64_t size = 0, d[kPackSlots];
  uint32_t nonempty = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPackSlots; ++k) {
    size += (bytes[k] + 7) & ~7ull;
    nonempty += bytes[k] ? 1u : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < kPackSlots; ++k) {
    d[k] = 0;
#pragma unroll
    for (uint32_t q = 0; q < kPackSlots; ++q)
      if (bytes[q] && (off[q] < off[k] || (off[q] == off[k] && q < k))) d[k] += (bytes[q] + 7) & ~7ull;
  }
  const uint64_t incl = prog::wave_incl_scan(size);
  const uint64_t pre = incl - size, total = __shfl(incl, 63, 64);
  const uint64_t base = (p.scale * a.offs[r0] + 7) & ~7ull;
  if (r < nrec) {
    uint32_t empties = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPackSlots; ++k) {
      if (k >= K) continue;
      uint32_t rank;
      if (bytes[k]) {
        rank = 0;
#pragma unroll
        for (uint32_t q = 0; q < kPackSlots; ++q)
          rank += (bytes[q] && (off[q] < off[k] || (off[q] == off[k] && q < k))) ? 1u : 0u;
      } else {
        rank = nonempty + empties++;
      }
      PackEnt& e = tab[r * K + rank];
      e.src = off[k];
      e.d = pre + (bytes[k] ? d[k] : size);
      e.bytes = bytes[k];
      tgpu_span* sp = (tgpu_span*)(rec + p.member[k]);
      sp->offset = bytes[k] ? base + pre + d[k] : 0;
    }
  }
  __syncthreads();  // table complete
  const uint32_t M = nrec * K;
  const uint64_t T = total, cap = a.arena_cap;
  uint8_t* ar = a.arena;
  // whole 8-byte words where the arena allows (an array's packed start is
  // 8-byte aligned, so a word holds one array's bytes and its padding), each
  // read as the two aligned words its bytes span; bytes otherwise
  const bool words = ((uintptr_t)ar & 7) == 0;
  for (uint64_t c = 0; c < T; c += kChunk) {
    const uint64_t j0 = c + 16ull * r;
    uint64_t w[2] = {0, 0};
    uint32_t nb[2] = {0, 0};  // valid leading bytes of each word (8: whole)
    if (j0 < T) {
      uint32_t lo = 0, hi = M;  // the last entry whose packed offset is <= j0
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tab[mid].d <= j0) lo = mid + 1;
        else hi = mid;
      }
      uint32_t e = lo ? lo - 1 : 0;
#pragma unroll
      for (uint32_t q = 0; q < 2; ++q) {
        const uint64_t j = j0 + 8 * q;
        if (j >= T) continue;
        while (e + 1 < M && tab[e + 1].d <= j) ++e;
        const uint64_t t = j - tab[e].d;
        if (t >= tab[e].bytes) continue;  // alignment padding: unspecified, not written
        const uint32_t n = (uint32_t)min((uint64_t)8, tab[e].bytes - t);
        const uint64_t s = tab[e].src + t;
        const uint64_t al = s & ~7ull;
        if (words && al + 16 <= cap) {
          const uint64_t a0 = *(const uint64_t*)(ar + al), a1 = *(const uint64_t*)(ar + al + 8);
          const uint32_t sh = (uint32_t)(s & 7) * 8;
          w[q] = sh ? (a0 >> sh) | (a1 << (64 - sh)) : a0;
        } else {
          for (uint32_t b = 0; b < n; ++b)  // (a failing record's list resized past the arena: 0)
            w[q] |= (uint64_t)(s + b < cap ? ar[s + b] : 0) << (8 * b);
        }
        nb[q] = n;
      }
    }
    __syncthreads();  // every source byte of the chunk read
#pragma unroll
    for (uint32_t q = 0; q < 2; ++q) {
      const uint64_t dst = base + j0 + 8 * q;
      if (nb[q] == 8 && words && dst + 8 <= cap) {
        *(uint64_t*)(ar + dst) = w[q];
      } else {
        for (uint32_t b = 0; b < nb[q]; ++b)
          if (dst + b < cap) ar[dst + b] = (uint8_t)(w[q] >> (8 * b));
      }
    }
    __syncthreads();  // before the next chunk's reads (and the next block's table)
  }
}

// Persistent over the call's blocks: each wave reads 64 blocks' marks at
// once and packs the ones the decode did not (a call whose decode tiles
// packed every block costs one pass over the marks).
__global__ __launch_bounds__(kArenaBlock) void arena_pack_kernel(DecodeArgs a, ArenaPack p) {
  static_assert(kArenaBlock == 64, "one wave per block");
  __shared__ PackEnt tab[kArenaBlock * kPackSlots];
  const DevResult* res = a.res;
  // the call's records, the failing one included (it is partially written)
  uint64_t m = res->n_records + (res->code ? 1 : 0);
  if (m > a.n) m = a.n;
  const uint64_t nb = (m + kArenaBlock - 1) / kArenaBlock;
  for (uint64_t g = (uint64_t)blockIdx.x * 64; g < nb; g += (uint64_t)gridDim.x * 64) {
    const uint64_t b = g + threadIdx.x;
    uint64_t todo = __ballot(b < nb && !(a.pack_flags && a.pack_flags[b] == a.pack_epoch));
    while (todo) {
      const uint32_t i = (uint32_t)__builtin_ctzll(todo);
      todo &= todo - 1;
      pack_block(a, p, g + i, m, tab);
    }
  }
}

}  // namespace

hipError_t launch_arena_pack(const DecodeArgs& a, const ArenaPack& p, hipStream_t stream) {
  if (!a.n || !p.n || !a.arena || !a.offs) return hipSuccess;
  // (one wave per group of 64 blocks, at most 2048 waves: the marks are
  // read in one or a few passes, the blocks left to pack spread over them)
  const uint64_t groups = ((a.n + kArenaBlock - 1) / kArenaBlock + 63) / 64;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(groups ? groups : 1, 2048);
  hipLaunchKernelGGL(arena_pack_kernel, dim3(grid), dim3(kArenaBlock), 0, stream, a, p);
  return hipGetLastError();
}

}  // namespace tgpu
