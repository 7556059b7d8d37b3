// k_index.hip — record index of an unindexed stream: the bulk form of the
// reference's file-reading loop `while (!cursor.isAtEnd()) deserialize<T>(c)`
// (Serializer.h:97-100), which is sequential because record k+1 starts where
// record k's readNoXfer stopped. Here the dependency is broken by speculation:
//
//   1. index_spec_kernel — one lane per chunk of `chunk` bytes. The lane tries
//      candidate starts (chunk 0 of a non-speculative call: `begin` only) and
//      accepts the first from which records parse back to back to the chunk's
//      end, the first record in the canonical form (tgpu_program.h) and the
//      rest canonical or, failing that, read by the general reader (exact
//      readNoXfer consumption, tgpu_device.h). Result per chunk: s (first
//      start), e (first start at or past the chunk's end), cnt (records).
//   2. index_flag_kernel + scan + index_list_kernel — chunks whose link is
//      broken (s[j] != e[j-1], or nothing accepted) in ascending order.
//   3. index_fix_kernel — one lane walks the broken links in order from the
//      true start, re-parses each with the general reader and follows the
//      cascade until the chain agrees again; the first reader error ends the
//      stream exactly where the reference would throw.
//   4. scan of the per-chunk counts, index_emit_kernel writes every start
//      (one lane per chunk, re-walking its chain), index_finish_kernel writes
//      the end, the status and (decode) pads the index to the requested count.
// Speculation only decides speed: every chunk the result uses was either
// parsed from its verified true start or is linked to one by s[j] == e[j-1].
#include "tgpu_device.h"
#include "tgpu_prog_kernels.h"

namespace tgpu {
namespace {

using prog::chunk_hi;
using prog::chunk_lo;
using prog::kErr;
using prog::kNo;
using prog::kPartial;
using prog::kPosCap;
using prog::kTile;
using prog::kTileLanes;

// A speculated chain reads at most spec_reach bytes (IndexArgs; 256 KiB
// unless TGPU_INDEX_SPEC_REACH) past its chunk's end. A
// false start can parse as a container of many elements that are true
// records (a list<struct> count read from value bytes), which would otherwise
// walk the rest of the stream on one lane, for every such candidate; past the
// reach the candidate is rejected like any other that fails to read, and a
// chunk whose true straddling record is longer than that is left to the
// repair lane (unbounded).
__device__ __forceinline__ uint64_t spec_limit(const IndexArgs& a, uint64_t hi) {
  return hi + a.spec_reach < a.in_len ? hi + a.spec_reach : a.in_len;
}

// lane >= 0: the deep-pass lane whose HBM skip frames the reader may use.
// limit: the reader's end (a.in_len, or a speculated chain's reach).
__device__ __forceinline__ dev::Reader reader_at(const IndexArgs& a, uint64_t pos, int lane,
                                                 uint64_t limit) {
  dev::Reader r = dev::make_reader(a.in, pos, limit, a.string_limit, a.container_limit,
                                   a.max_depth, a.height);
  if (lane >= 0) dev::attach_slab(r, a.deep, (uint32_t)lane);
  return r;
}

struct Chain {
  uint64_t end;    // first record start >= hi (or the failing record's start)
  uint64_t second; // start of the chain's second record (kNo: fewer than two)
  uint64_t count;  // records parsed
  int32_t code;    // reader error (0: none)
  uint64_t err_off;
};

// One record at p (reader end `limit`): the program first, then (general)
// the reader. Returns 1 (q = the next record's start), 0 (not canonical and
// !general) or -1 (reader error in out.code / out.err_off).
template <int P>
__device__ __forceinline__ int one_record(const IndexArgs& a, uint64_t p, uint64_t limit,
                                          uint8_t* scratch, int lane, bool general, uint64_t& q,
                                          Chain& out) {
  if (a.prog && p < limit) {
    const prog::Ctx pc{0, nullptr, 0, a.string_limit, a.container_limit};
    const uint64_t avail = limit - p;
    const prog::HbmSrc src{a.in + p, (uint32_t)(avail < kPosCap ? avail : kPosCap)};
    uint32_t rel = 0;
    if (prog::run_program<false>(prog::DynProg{a.prog}, src, pc, rel, src.avail, nullptr)) {
      q = p + rel;
      return 1;
    }
  }
  if (!general) return 0;
  dev::Reader r = reader_at(a, p, lane, limit);
  // measuring read: the root into scratch, nested elements into per-level
  // slots after it (the index's scratch stride holds both)
  const uint32_t root = (a.sc.s[0].size + 15) & ~15u;
  dev::Arena A = dev::record_arena<P>(a.sc, nullptr, kDiscardArena, p, scratch + root);
  dev::read_record_any<P>(r, a.sc, scratch, A);
  if (!r.ok()) {
    out.code = r.err;
    out.err_off = r.err_off;
    return -1;
  }
  q = r.pos;
  return 1;
}

// Records back to back from p while p < hi. canonical_first: the first record
// must match the program (speculation); returns false if it does not.
// emit: record starts written to emit[0..) (at most emit_cap).
// A record nested past the private skip frames (lane < 0) ends the chain
// with out.code = kErrDeep: speculation treats it as a failed chain (the
// repair lane, which has HBM frames, walks it), emission defers the chunk.
// spec: a speculated chain (bounded reach, see spec_limit).
template <int P>
__device__ bool chain(const IndexArgs& a, uint64_t p, uint64_t hi, bool canonical_first,
                      uint8_t* scratch, Chain& out, uint64_t* emit, uint64_t emit_cap,
                      uint64_t max_count, int lane = -1, bool spec = false) {
  const uint64_t limit = spec ? spec_limit(a, hi) : a.in_len;
  out.count = 0;
  out.code = 0;
  out.err_off = 0;
  out.second = kNo;
  while (p < hi && out.count < max_count) {
    // speculation without a program: a record starts with a root field's
    // header or STOP (a false start's chain of garbage records dies early)
    if (spec && canonical_first && !a.prog && p < a.in_len) {
      const uint32_t b = a.in[p];
      if (!((a.hmask[b >> 5] >> (b & 31)) & 1u)) {
        out.code = TGPU_ERR_INDEX_MISMATCH;  // (internal: the candidate is rejected)
        out.end = p;
        return false;
      }
    }
    uint64_t q = 0;
    const int got = one_record<P>(a, p, limit, scratch, lane,
                                  !(canonical_first && out.count == 0 && a.prog), q, out);
    if (got == 0) return false;  // speculation: the first record is not canonical
    if (got < 0) {
      if (canonical_first && out.count == 0) return false;
      out.end = p;
      return true;
    }
    if (emit && out.count < emit_cap) emit[out.count] = p;
    if (out.count == 1) out.second = p;
    ++out.count;
    p = q;
  }
  out.end = p;
  return true;
}

// Program-only chain (light: no general reader, so the speculation and emit
// kernels keep a small register footprint): records back to back from p while
// p < hi and fewer than max_count; stops early (*stuck) at the first record
// the program does not take, p then being that record's start.
__device__ __forceinline__ uint64_t prog_chain(const IndexArgs& a, uint64_t& p, uint64_t hi,
                                               uint64_t max_count, uint64_t* emit,
                                               uint64_t emit_cap, bool& stuck) {
  const prog::Ctx pc{0, nullptr, 0, a.string_limit, a.container_limit};
  uint64_t count = 0;
  stuck = false;
  while (p < hi && count < max_count) {
    if (p >= a.in_len) {
      stuck = true;
      break;
    }
    const uint64_t avail = a.in_len - p;
    const prog::HbmSrc src{a.in + p, (uint32_t)(avail < kPosCap ? avail : kPosCap)};
    uint32_t rel = 0;
    if (!prog::run_program<false>(prog::DynProg{a.prog}, src, pc, rel, src.avail, nullptr)) {
      stuck = true;
      break;
    }
    if (emit && count < emit_cap) emit[count] = p;
    ++count;
    p += rel;
  }
  return count;
}

// Speculation, program-only (schemas with a program). A chain the program
// cannot finish is accepted as partial (e = kPartial, pf = where it stopped)
// when at least its first record was canonical; index_cont_kernel finishes it.
__global__ __launch_bounds__(256) void index_spec_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n_chunks) return;
  const uint64_t lo = chunk_lo(a, j), hi = chunk_hi(a, j);
  bool stuck;
  if (j == 0 && !a.speculative) {
    uint64_t p = a.begin;
    a.cnt[0] = prog_chain(a, p, hi, kNo, nullptr, 0, stuck);
    a.s[0] = a.begin;
    a.e[0] = stuck ? kPartial : p;
    a.pf[0] = p;
    return;
  }
  const uint64_t w = j == 0 ? a.chunk : a.window;  // a shard's first record may start late
  const uint64_t last = lo + w < hi ? lo + w : hi;
  // candidates are the positions holding the program's first header byte,
  // found 8 bytes per load (zero-byte test on w ^ broadcast(h0))
  const uint64_t h0 = a.prog->ops[0].kind == VOP_CONST ? (a.prog->ops[0].hdr & 0xff) : 0x100;
  const prog::HbmSrc src{a.in + lo, (uint32_t)(a.in_len - lo < kPosCap ? a.in_len - lo : kPosCap)};
  for (uint64_t base = lo; base < last; base += 8) {
    uint64_t m;
    if (h0 < 0x100) {
      const uint64_t x = src.win8((uint32_t)(base - lo)) ^ (h0 * 0x0101010101010101ull);
      m = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
    } else {
      m = 0x8080808080808080ull;  // CBOOL first: every position is a candidate
    }
    while (m) {
      const uint64_t cand = base + ((uint32_t)__builtin_ctzll(m) >> 3);
      m &= m - 1;
      if (cand >= last) break;
      uint64_t p = cand;
      const uint64_t c = prog_chain(a, p, hi, kNo, nullptr, 0, stuck);
      if (c == 0) continue;  // the candidate's first record is not canonical
      a.s[j] = cand;
      a.e[j] = stuck ? kPartial : p;
      a.pf[j] = p;
      a.cnt[j] = c;
      return;
    }
  }
  a.s[j] = kNo;
  a.e[j] = kNo;
  a.cnt[j] = 0;
}

// Kernels whose lanes run the general reader keep its frame stacks in
// scratch (1.5-2.5 KB per lane). The runtime backs a dispatch's scratch for as
// many waves as the grid can keep resident, and re-backs it when a call
// finds it released: a one-lane-per-chunk grid over a 3.5 GB stream (850
// workgroups) cost 0.3-0.5 ms per such kernel per call, where the work itself
// (nothing to do for almost every chunk) takes microseconds. These run a
// small grid (kScratchGrid workgroups) that strides over the chunks.
#define SCRATCH_KERNEL(name, body)                                            \
  template <int P>                                                            \
  __global__ __launch_bounds__(256) void name(IndexArgs a) {                  \
    const uint64_t stride = (uint64_t)gridDim.x * 256;                        \
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < a.n_chunks; \
         j += stride)                                                         \
      body<P>(a, j);                                                          \
  }

// Finishes partial chains with the general reader (program first per record).
// A reader error rejects a speculated start (kNo: the repair pass decides);
// from a verified start (chunk 0 of a non-speculative call) it is final (kErr).
template <int P>
__device__ __forceinline__ void index_cont_one(const IndexArgs& a, uint64_t j) {
  if (a.e[j] != kPartial) return;
  Chain c;
  const bool verified = j == 0 && !a.speculative;
  chain<P>(a, a.pf[j], chunk_hi(a, j), false, a.scratch + j * a.rec_size, c, nullptr, 0, kNo, -1,
           !verified);
  if (c.code) {
    if (j == 0 && !a.speculative) {
      a.e[0] = kErr;
    } else {
      a.s[j] = kNo;
      a.e[j] = kNo;
      a.cnt[j] = 0;
    }
    return;
  }
  a.e[j] = c.end;
  a.cnt[j] += c.count;
  a.pf[j] = 0;
}
SCRATCH_KERNEL(index_cont_kernel, index_cont_one)

// Speculation for schemas without a program: any record the general reader
// accepts may open a chain.
template <int P>
__global__ __launch_bounds__(256) void index_spec_general_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n_chunks) return;
  uint8_t* scratch = a.scratch + j * a.rec_size;
  const uint64_t lo = chunk_lo(a, j), hi = chunk_hi(a, j);
  Chain c;
  uint64_t* starts = a.sst + j * kSpecStarts;
  starts[0] = kNo;
  if (j == 0 && !a.speculative) {
    chain<P>(a, a.begin, hi, false, scratch, c, nullptr, 0, kNo);
    a.s[0] = a.begin;
    a.e[0] = c.code ? kErr : c.end;
    a.cnt[j] = c.count;
    return;
  }
  const uint64_t w = j == 0 ? a.chunk : a.window;
  const uint64_t last = lo + w < hi ? lo + w : hi;
  for (uint64_t cand = lo; cand < last; ++cand) {
    if (chain<P>(a, cand, hi, true, scratch, c, starts, kSpecStarts, kNo, -1, true) &&
        c.code == 0) {
      a.s[j] = cand;
      a.e[j] = c.end;
      a.cnt[j] = c.count;
      return;
    }
  }
  starts[0] = kNo;
  a.s[j] = kNo;
  a.e[j] = kNo;
  a.cnt[j] = 0;
}

// Speculation fallback for chunks in which no candidate opened a canonical
// chain (kNo): any record the general reader accepts may open it (records
// that left the canonical form: reordered, unknown or missing fields, as after
// schema evolution). A candidate inside the record straddling the chunk's
// start can parse as a record of its own and then run in step with the true
// records; the chain's first kSpecStarts starts (sst) let the repair pass
// take it over in O(1) when the true start is one of them.
template <int P>
__device__ __forceinline__ void index_spec_fallback_one(const IndexArgs& a, uint64_t j) {
  uint64_t* starts = a.sst + j * kSpecStarts;
  starts[0] = kNo;
  if (a.s[j] != kNo || a.e[j] != kNo) return;
  uint8_t* scratch = a.scratch + j * a.rec_size;
  const uint64_t lo = chunk_lo(a, j), hi = chunk_hi(a, j);
  Chain c;
  if (j == 0 && !a.speculative) {
    chain<P>(a, a.begin, hi, false, scratch, c, nullptr, 0, kNo);
    a.s[0] = a.begin;
    a.e[0] = c.code ? kErr : c.end;
    a.cnt[0] = c.count;
    return;
  }
  const uint64_t w = j == 0 ? a.chunk : a.window;
  const uint64_t last = lo + w < hi ? lo + w : hi;
  for (uint64_t cand = lo; cand < last; ++cand) {
    if (chain<P>(a, cand, hi, false, scratch, c, starts, kSpecStarts, kNo, -1, true) &&
        c.code == 0 && c.count) {
      a.s[j] = cand;
      a.e[j] = c.end;
      a.cnt[j] = c.count;
      a.pf[j] = 0;
      return;
    }
  }
  starts[0] = kNo;
}
SCRATCH_KERNEL(index_spec_fallback_kernel, index_spec_fallback_one)

// The chain of chunk j from a start T, walked only until it meets the
// chunk's speculated chain (s[j], cnt[j] records to e[j]): a false start
// inside the record straddling the chunk's start parses as records of its own
// and soon lands on a true record start, after which it runs in step with the
// true chain. Two pointers, the one behind advances; met: from the meeting
// point the speculated chain is T's, so e[j] stands and the count is the
// records from T to there + the speculated chain's from there. A walk from T
// that passes the chunk's end first is the chunk's chain (out.end). limit: the
// reader's end; lane: deep-pass lane (-1: none). Returns false on a reader
// error of the walk from T (out.code / err_off / end = the failing start).
template <int P>
__device__ bool walk_meet(const IndexArgs& a, uint64_t j, uint64_t T, uint64_t limit,
                          uint8_t* scratch, int lane, Chain& out, bool& met) {
  const uint64_t hi = chunk_hi(a, j);
  const uint64_t s0 = a.s[j], e0 = a.e[j];
  const bool spec = s0 != kNo && e0 != kNo && e0 != kErr && e0 != kPartial;
  uint64_t pt = T, pf = spec ? s0 : kNo, ct = 0, cf = 0;
  met = false;
  out.code = 0;
  for (;;) {
    if (pt == pf) {
      met = true;
      break;
    }
    if (pt < pf) {
      if (pt >= hi) break;
      uint64_t q;
      Chain c{};
      if (one_record<P>(a, pt, limit, scratch, lane, true, q, c) < 0) {
        out.code = c.code;
        out.err_off = c.err_off;
        out.end = pt;
        out.count = ct;
        return false;
      }
      pt = q;
      ++ct;
    } else {
      uint64_t q;
      Chain c{};
      // past the speculated chain's end, or a record it cannot read again
      // (a reach-bounded chain): finish from T alone
      if (pf >= hi || one_record<P>(a, pf, limit, scratch, lane, true, q, c) < 0) {
        pf = kNo;
        continue;
      }
      pf = q;
      ++cf;
    }
  }
  out.count = met ? ct + (a.cnt[j] - cf) : ct;
  out.end = met ? e0 : pt;
  return true;
}

// Parallel link repair, one lane per chunk whose start s[j] is not its
// predecessor's end T: the chain from T (walk_meet), as of the previous
// round's ends (ep, a snapshot: every chunk of a round reads the same ends,
// Jacobi). A chunk whose predecessor was right after round r - 1 is right
// after round r; chains converge within a few records, so one or two rounds
// usually leave every link consistent. index_fix_kernel then verifies the
// links from the true start in order, so these rounds only decide speed. A
// reader error leaves the chunk to index_fix_kernel. Returns whether the
// chunk changed.
template <int P>
__device__ __forceinline__ bool index_merge_one(const IndexArgs& a, uint64_t j) {
  if (j == 0) return false;
  const uint64_t T = a.ep[j - 1];
  if (T == kNo || T == kErr || T == kPartial) return false;
  const uint64_t s0 = a.s[j], e0 = a.e[j];
  if (s0 == T || e0 == kErr || e0 == kPartial) return false;
  const uint64_t hi = chunk_hi(a, j);
  Chain c{};
  bool met;
  if (!walk_meet<P>(a, j, T, spec_limit(a, hi), a.scratch + j * a.rec_size, -1, c, met))
    return false;
  a.cnt[j] = c.count;
  a.e[j] = c.end;
  a.s[j] = T;
  a.pf[j] = 0;
  return true;
}

// One merge round: snapshot of the ends (ep), then the chunks' walks. The
// counter of round r is scal[16 + (r & 1)]; a round after one that changed
// nothing returns at once (stream-ordered, no host read).
__global__ __launch_bounds__(256) void index_merge_snap_kernel(IndexArgs a, int round) {
  if (round > 0 && a.scal[16 + ((round - 1) & 1)] == 0) {
    // skipped: this round's counter still holds round - 2's count, so zero
    // it, or round + 1 would see it and run a full round again
    if (blockIdx.x == 0 && threadIdx.x == 0) a.scal[16 + (round & 1)] = 0;
    return;
  }
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < a.n_chunks; j += stride)
    a.ep[j] = a.e[j];
  if (blockIdx.x == 0 && threadIdx.x == 0) a.scal[16 + (round & 1)] = 0;
}

template <int P>
__global__ __launch_bounds__(256) void index_merge_round_kernel(IndexArgs a, int round) {
  if (round > 0 && a.scal[16 + ((round - 1) & 1)] == 0) return;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  unsigned int changed = 0;
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < a.n_chunks; j += stride)
    changed += index_merge_one<P>(a, j) ? 1u : 0u;
  const int n = __syncthreads_count(changed != 0);
  if (threadIdx.x == 0 && n) atomicAdd(&a.scal[16 + (round & 1)], (unsigned long long)n);
}


// ---- LDS tiles (schemas with a program; tgpu_prog_kernels.h) ---------------
__global__ __launch_bounds__(kTileLanes) void index_tile_spec_kernel(IndexArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];
  __shared__ prog::IndexTileShared sm;
  prog::index_spec_tile(a, prog::DynProg{a.prog}, lds, sm);
}

__global__ __launch_bounds__(kTileLanes) void index_tile_emit_kernel(IndexArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];
  __shared__ prog::IndexTileShared sm;
  prog::index_emit_kernel_body(a, prog::DynProg{a.prog}, lds, sm);
}

// Stored starts (a.st16): tile j's current starts go to offs[base[j] ..], one
// wave per tile, four tiles per workgroup; a tile whose starts are not
// current (no stored list, or the repair re-chained or moved it) is listed
// in bad[] (count scal[6]) for the emit kernel's re-walk.
__global__ __launch_bounds__(256) void index_starts_copy_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (j >= a.n_chunks) return;
  // every word the tile's verdict needs and its first 64 starts, loaded
  // together: one memory round trip before the copy instead of four
  // dependent ones (starts_current's test, inline)
  const uint64_t in_effect = a.scal[1], n = a.cnt[j], pf = a.pf[j], s = a.s[j], b = a.base[j];
  const uint16_t* st = a.st16 + j * a.st_cap;
  const uint32_t s0 = lane < a.st_cap ? st[lane] : 0u;
  if (lane == 0) a.ep[j] = kNo;
  if (j >= in_effect || n == 0) return;
  const uint64_t lo = chunk_lo(a, j);
  const uint64_t gb = lo - ((uintptr_t)(a.in + lo) & 15);
  if (pf != prog::kStartsValid || gb + __shfl(s0, 0, 64) != s) {
    if (lane == 0) a.bad[atomicAdd(&a.scal[6], 1ull)] = j;
    return;
  }
  for (uint64_t i = lane; i < n; i += 64)
    if (b + i <= a.max_records) a.offs[b + i] = gb + (i < 64 ? s0 : st[i]);
}

__global__ __launch_bounds__(kTileLanes) void index_tile_decode_kernel(IndexArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];
  __shared__ __attribute__((aligned(16))) uint8_t rtile[prog::kRecTileBytes + 32];
  __shared__ prog::IndexTileShared sm;
  prog::index_emit_tile<true>(a, prog::DynProg{a.prog}, lds, sm, rtile, blockIdx.x);
}

// Single pass (tgpu_prog_kernels.h index_onepass_tile), interpreted program.
template <bool kDecode>
__global__ __launch_bounds__(kTileLanes) void index_onepass_kernel(IndexArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];
  __shared__ __attribute__((aligned(16))) uint8_t rtile[kDecode ? prog::kRecTileBytes + 32 : 16];
  __shared__ prog::IndexTileShared sm;
  __shared__ prog::OnePassShared op;
  prog::index_onepass_tile<kDecode>(a, prog::DynProg{a.prog}, lds, sm, rtile, op);
}

__global__ __launch_bounds__(256) void index_onepass_init_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < a.n_chunks) {
    a.pf[j] = 0;
    a.ep[j] = 0;
  }
  if (j == 0) {
    a.scal[0] = 0;  // (tgpu_index_stats: no repairs)
    a.scal[1] = a.n_chunks;
    a.scal[2] = kNo;
    for (int k = 6; k < 12; ++k) a.scal[k] = 0;
  }
}

__device__ __forceinline__ bool link_broken(const IndexArgs& a, uint64_t j) {
  const uint64_t e = a.e[j];
  if (e == kNo || e == kErr || e == kPartial) return true;
  if (j == 0) return a.s[0] == kNo;
  return a.s[j] != a.e[j - 1];
}

__global__ __launch_bounds__(256) void index_flag_kernel(IndexArgs a, int sst_valid) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n_chunks) return;
  a.base[j] = link_broken(a, j) ? 1 : 0;
  if (!sst_valid) a.sst[j * kSpecStarts] = kNo;
}

__global__ __launch_bounds__(256) void index_list_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < a.n_chunks && link_broken(a, j)) a.bad[a.base[j]] = j;
}

// The true start T of chunk j is one of its speculated chain's first
// kSpecStarts starts: the chain from T is the rest of it.
__device__ __forceinline__ bool take_over(const IndexArgs& a, uint64_t j, uint64_t T) {
  const uint64_t* st = a.sst + j * kSpecStarts;
  const uint64_t n = a.cnt[j] < (uint64_t)kSpecStarts ? a.cnt[j] : (uint64_t)kSpecStarts;
  for (uint64_t m = 1; m < n; ++m) {
    if (st[m] == T) {
      a.s[j] = T;
      a.cnt[j] -= m;
      return true;
    }
  }
  return false;
}

// One lane: repair the chain (see header). scal[1] = chunks in effect.
template <int P>
__global__ void index_fix_kernel(IndexArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (a.scal[18]) return;  // the exhaustive resolution set every chunk
  const uint64_t C = a.n_chunks;
  a.scal[2] = kNo;
  a.scal[1] = C;
  uint64_t T0 = a.begin, j0 = 0;
  if (a.speculative) {
    // the first chunk with a speculated start opens the range (a record may
    // cover the first chunks entirely); none at all: no record starts here
    while (j0 < C && a.s[j0] == kNo) ++j0;
    if (j0 == C) {
      a.scal[1] = 0;
      return;
    }
    T0 = a.s[j0];
    for (uint64_t i = 0; i < j0; ++i) {
      a.s[i] = T0;
      a.e[i] = T0;
      a.cnt[i] = 0;
    }
  }
  const uint64_t m = a.scal[0];
  uint64_t next = 0;  // chunks below are final
  uint8_t* scratch = a.scratch;
  for (uint64_t k = 0; k < m; ++k) {
    uint64_t j = a.bad[k];
    if (j < next || j < j0) continue;
    uint64_t T = j == 0 ? T0 : a.e[j - 1];
    for (;;) {
      const uint64_t hi = chunk_hi(a, j);
      if (T >= hi) {  // no record starts inside this chunk
        a.s[j] = T;
        a.e[j] = T;
        a.cnt[j] = 0;
        a.pf[j] = 0;
      } else if (T > a.s[j] && a.sst[j * kSpecStarts] == a.s[j] && a.e[j] != kNo &&
                 a.e[j] != kErr && a.e[j] != kPartial && take_over(a, j, T)) {
        // the speculated chain started with false records inside the record
        // ending at T; from T on it is the true chain
      } else {
        // the chain from T, until it meets the speculated one (walk_meet:
        // the lane's work is the records up to the meeting point, not the
        // chunk)
        Chain c{};
        bool met;
        walk_meet<P>(a, j, T, a.in_len, scratch, 0, c, met);
        a.s[j] = T;
        a.cnt[j] = c.count;
        a.pf[j] = 0;
        if (c.code) {
          a.e[j] = c.end;
          a.scal[1] = j + 1;
          a.scal[2] = j;
          a.scal[3] = c.count;
          a.scal[4] = c.end;
          a.res->code = c.code;
          a.res->fail_offset = c.err_off;
          return;
        }
        a.e[j] = c.end;
      }
      T = a.e[j];
      if (j + 1 < C && (a.s[j + 1] != T || a.e[j + 1] == kNo || a.e[j + 1] == kErr)) {
        ++j;
        continue;
      }
      break;
    }
    next = j + 1;
  }
}

// ---- exhaustive resolution (opt-in, TGPU_INDEX_EXHAUSTIVE) ------------------
// Built for program-less streams whose speculation leaves many links broken,
// on the premise that false chains of the general reader need not meet the
// true one inside a chunk (a false record read as a long container lands
// anywhere), so the merge rounds could not fix them and the verification lane
// would walk the stream alone (round 4: 3.8 s). Measured: with the
// speculation's reach bounded by the record length, false chains do meet and
// the merge rounds repair every link; reading every position is 20-40x
// slower, so this stays off by default. Every byte position p of chunk j is read as
// a record start (nxt(p) = its end, or a failure), and pointer jumping over
// the chunk's positions in LDS (13 rounds: 2^13 > the 4 KiB chunk) gives,
// for each position, the chain's exit past the chunk's end and its records.
// The first kXWindow entries go to tables xe / xc; one lane then follows the
// true path T_0 = begin, T_{j+1} = xe[j][T_j - lo_j] — a lookup per chunk
// where the verification walks the chunk — and sets s / e / cnt. A true entry
// past the window (a record straddling more than kXWindow bytes into a
// chunk) or a record nested past the private frames stops the lookups there
// and leaves the rest to index_fix_kernel; a record the reader rejects on
// the path ends the stream as index_fix_kernel would.
constexpr uint32_t kXChunk = 4096;  // (index_chunk_bytes' lane chunks are at most this)
constexpr uint32_t kXTerm = 0xffffffffu;
constexpr uint32_t kXFail = 0x80000000u;  // X: the chain stops at a record the reader rejects

// (each position is read from an LDS copy of the chunk and kXReach bytes past
// it: a record reaching further reads as a failure here — the path lookup
// re-reads such a record in HBM and, if it is a record, leaves the chunks
// from there to the verification walk)
constexpr uint32_t kXReach = 4096;

template <int P>
__global__ __launch_bounds__(256) void index_xtab_kernel(IndexArgs a) {
  __shared__ uint32_t T0[kXChunk], K0[kXChunk], X0[kXChunk];
  __shared__ uint32_t T1[kXChunk], K1[kXChunk], X1[kXChunk];
  __shared__ __attribute__((aligned(16))) uint8_t stage[kXChunk + kXReach + 32];
  const uint64_t rs = (a.rec_size + 15) & ~15ull;
  uint8_t* scratch = a.xscratch + ((uint64_t)blockIdx.x * 256 + threadIdx.x) * rs;
  const uint32_t root = (a.sc.s[0].size + 15) & ~15u;
  for (uint64_t j = blockIdx.x; j < a.n_chunks; j += gridDim.x) {
    const uint64_t lo = chunk_lo(a, j), hi = chunk_hi(a, j);
    const uint32_t len = (uint32_t)(hi - lo);
    const uint64_t a0 = lo & ~15ull;
    const uint64_t b1 = hi + a.x_reach < a.in_len ? hi + a.x_reach : a.in_len;
    const uint32_t nvec = (uint32_t)((b1 - a0 + 15) >> 4);
    for (uint32_t v = threadIdx.x; v < nvec; v += 256) {
      const uint64_t g = a0 + 16ull * v;
      if (g + 16 <= a.in_len) {
        *(uint4*)(stage + 16 * v) = *(const uint4*)(a.in + g);
      } else {
        for (uint32_t b = 0; b < 16; ++b) stage[16 * v + b] = g + b < a.in_len ? a.in[g + b] : 0;
      }
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < len; p += 256) {
      dev::Reader r = dev::make_reader(stage, lo + p, b1, a.string_limit, a.container_limit,
                                       a.max_depth, a.height);
      r.base = a0;
      dev::Arena A = dev::record_arena<P>(a.sc, nullptr, kDiscardArena, lo + p, scratch + root);
      dev::read_record_any<P>(r, a.sc, scratch, A);
      // (a failure, a record reaching past the copy, or one nested past the
      // private frames: the chain stops here)
      if (!r.ok()) {
        T0[p] = kXTerm;
        K0[p] = 0;
        X0[p] = kXFail | p;
      } else if (r.pos >= hi) {
        T0[p] = kXTerm;
        K0[p] = 1;
        X0[p] = (uint32_t)(r.pos - lo);
      } else {
        T0[p] = (uint32_t)(r.pos - lo);
        K0[p] = 1;
        X0[p] = 0;
      }
    }
    __syncthreads();
    uint32_t *Ta = T0, *Ka = K0, *Xa = X0, *Tb = T1, *Kb = K1, *Xb = X1;
    for (int rd = 0; rd < 13; ++rd) {
      bool open = false;
      for (uint32_t p = threadIdx.x; p < len; p += 256) {
        const uint32_t t = Ta[p];
        if (t == kXTerm) {
          Tb[p] = t;
          Kb[p] = Ka[p];
          Xb[p] = Xa[p];
        } else {
          const uint32_t t2 = Ta[t];
          Tb[p] = t2;
          Kb[p] = Ka[p] + Ka[t];
          Xb[p] = Xa[t];
          open |= t2 != kXTerm;
        }
      }
      uint32_t* sw;
      sw = Ta; Ta = Tb; Tb = sw;
      sw = Ka; Ka = Kb; Kb = sw;
      sw = Xa; Xa = Xb; Xb = sw;
      if (!__syncthreads_or(open)) break;
    }
    for (uint32_t w = threadIdx.x; w < kXWindow; w += 256) {
      uint64_t x = kNo;
      uint32_t k = 0;
      if (w < len) {
        const uint32_t v = Xa[w];
        x = (v & kXFail) ? ((1ull << 63) | (lo + (v & ~kXFail))) : lo + v;
        k = Ka[w];
      }
      a.xe[j * kXWindow + w] = x;
      a.xc[j * kXWindow + w] = k;
    }
    __syncthreads();  // (the next chunk reuses the arrays)
  }
}

// One lane: the true path through the tables (non-speculative ranges).
// scal[18] = 1: every chunk set (index_fix_kernel has nothing to do).
template <int P>
__global__ void index_xresolve_kernel(IndexArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t C = a.n_chunks;
  uint64_t T = a.begin;
  for (uint64_t j = 0; j < C; ++j) {
    const uint64_t lo = chunk_lo(a, j), hi = chunk_hi(a, j);
    if (T >= hi) {  // no record starts in this chunk
      a.s[j] = T;
      a.e[j] = T;
      a.cnt[j] = 0;
      a.pf[j] = 0;
      continue;
    }
    const uint64_t w = T - lo;
    if (w >= kXWindow) return;
    const uint64_t x = a.xe[j * kXWindow + w];
    const uint32_t k = a.xc[j * kXWindow + w];
    if (x == kNo) return;
    if (x >> 63) {
      // the chain from T stops at a record the reader rejects, k records in;
      // read it with the deep slab (a record nested past the private frames
      // is not a failure: the verification walks on from there)
      const uint64_t f = x & ~(1ull << 63);
      uint64_t q = 0;
      Chain c{};
      if (one_record<P>(a, f, a.in_len, a.scratch, 0, true, q, c) > 0) return;
      a.s[j] = T;
      a.cnt[j] = k;
      a.pf[j] = 0;
      a.e[j] = f;
      a.scal[1] = j + 1;
      a.scal[2] = j;
      a.scal[3] = k;
      a.scal[4] = f;
      a.res->code = c.code;
      a.res->fail_offset = c.err_off;
      a.scal[18] = 1;
      return;
    }
    a.s[j] = T;
    a.e[j] = x;
    a.cnt[j] = k;
    a.pf[j] = 0;
    T = x;
  }
  a.scal[1] = C;
  a.scal[2] = kNo;
  a.scal[18] = 1;
}

__global__ __launch_bounds__(256) void index_prep_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < a.n_chunks) a.base[j] = j < a.scal[1] ? a.cnt[j] : 0;
  if (j == 0) a.scal[6] = 0;  // tiles listed for the emit's re-walk (stored starts)
}

// Emit, program-only; a chain the program cannot finish is handed to
// index_emit_cont_kernel (ep = where it stopped, ec = starts written).
__global__ __launch_bounds__(256) void index_emit_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.n_chunks) return;
  a.ep[j] = kNo;
  if (j >= a.scal[1]) return;
  const uint64_t b = a.base[j];
  const uint64_t n = a.cnt[j];
  if (n == 0 || b > a.max_records) return;
  const uint64_t cap = a.max_records + 1 - b;
  uint64_t p = a.s[j];
  bool stuck = true;
  uint64_t c = 0;
  if (a.prog) c = prog_chain(a, p, kNo, n, a.offs + b, cap, stuck);
  if (c < n) {
    a.ep[j] = p;
    a.ec[j] = c;
  }
}

// Emission of chunk j's chain from where the program stopped (ep[j]) with
// the general reader; lane >= 0: deep pass (HBM skip frames).
template <int P>
__device__ __forceinline__ void emit_cont(const IndexArgs& a, uint64_t j, int lane) {
  const uint64_t b = a.base[j] + a.ec[j];
  const uint64_t n = a.cnt[j] - a.ec[j];
  if (b > a.max_records) return;
  Chain c;
  chain<P>(a, a.ep[j], kNo, false, a.scratch + j * a.rec_size, c, a.offs + b,
           a.max_records + 1 - b, n, lane);
  if (c.code == kErrDeep) {  // the deep pass re-walks the whole chain
    a.deep_chunks[atomicAdd(&a.res->n_deep_chunks, 1ull)] = j;
    return;
  }
  if (a.recs)  // fused decode: these records take the general decoder
    for (uint64_t i = 0; i < c.count && b + i < a.n_decode; ++i)
      a.irr[atomicAdd(a.nirr, 1ull)] = b + i;
}

template <int P>
__device__ __forceinline__ void index_emit_cont_one(const IndexArgs& a, uint64_t j) {
  if (a.ep[j] == kNo) return;
  emit_cont<P>(a, j, -1);
}
SCRATCH_KERNEL(index_emit_cont_kernel, index_emit_cont_one)

template <int P>
__global__ __launch_bounds__(64) void index_deep_emit_kernel(IndexArgs a) {
  const uint32_t lane = blockIdx.x * 64 + threadIdx.x;
  if (lane >= a.deep.lanes) return;
  const uint64_t m = a.res->n_deep_chunks;
  for (uint64_t k = lane; k < m; k += a.deep.lanes) emit_cont<P>(a, a.deep_chunks[k], (int)lane);
}

// Fused decode: a stream that ends (or fails) before n_decode records hands
// its first missing record to the general decoder, which reports it exactly
// (underflow, or the reader error the index stopped at).
__global__ void index_decode_tail_kernel(IndexArgs a, const unsigned long long* total_p) {
  if (threadIdx.x || blockIdx.x) return;
  const uint64_t total = *total_p;
  // decode_batch: the first missing record fails (underflow or the reader
  // error); a stream range: only a reader error's record (partially decoded
  // like the reference leaves it)
  if (total < a.n_decode && (a.decode_tail || a.scal[2] != kNo))
    a.irr[atomicAdd(a.nirr, 1ull)] = total;
}

// total records; end of the last one; status; decode padding of the index.
__global__ void index_finish_kernel(IndexArgs a, unsigned long long* total_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t ce = a.scal[1];
  uint64_t total = 0, end = a.begin;
  if (ce) {
    total = a.base[ce - 1] + a.cnt[ce - 1];
    end = a.e[ce - 1];
  }
  DevResult* res = a.res;
  res->first_start = ce ? a.s[0] : kNo;
  if (a.scal[2] != kNo && ce) {  // reader error: total = records before it
    res->first_fail = total;
    end = a.scal[4];
  } else if (!ce) {
    end = a.speculative ? kNo : a.begin;  // no record starts in the range
  }
  res->n_records = total;
  res->total_bytes = end;
  if (total <= a.max_records) a.offs[total] = end;
  *total_out = total;
}

// offs[total+1 .. fill_to] = offs[total]: records past the stream's end (or
// its first bad record) re-read that position, so the decoder reports them
// exactly (underflow / the same error) without a host round trip.
__global__ __launch_bounds__(256) void index_pad_kernel(IndexArgs a,
                                                        const unsigned long long* total_p) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t total = *total_p;
  if (i > total && i <= a.fill_to && total <= a.max_records) a.offs[i] = a.offs[total];
}

__global__ __launch_bounds__(256) void index_empty_kernel(DevResult* res, uint64_t* offs,
                                                          uint64_t pos, uint64_t fill_to) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i <= fill_to) offs[i] = pos;
  if (i == 0) {
    res->n_records = 0;
    res->total_bytes = pos;
    res->first_start = kNo;
  }
}

}  // namespace

hipError_t launch_index_empty(DevResult* res, uint64_t* offs, uint64_t pos, uint64_t fill_to,
                              hipStream_t stream) {
  hipLaunchKernelGGL(index_empty_kernel, dim3((uint32_t)((fill_to + 256) / 256)), dim3(256), 0,
                     stream, res, offs, pos, fill_to);
  return hipGetLastError();
}

uint64_t index_tile_bytes() { return kTile; }
uint64_t index_tile_lanes() { return kTileLanes; }

uint64_t index_chunk_bytes(uint64_t span, bool tiles, uint64_t mean) {
  // schemas with a program: LDS tiles once there are enough of them
  if (tiles && span >= 64ull * kTile) return kTile;
  // lane chunks: ~1k+ chunks keep the chip busy; chunks stay >= 1 KiB so a
  // chunk holds several records and speculation has a long chain to confirm
  // (about 16 records when the mean record length is known)
  uint64_t c = 4096;
  while (c > 1024 && (span / c < 4096 || (mean && c > 16 * mean))) c >>= 1;
  if (const char* v = getenv("TGPU_INDEX_CHUNK")) c = std::max(64, std::min(atoi(v), 4096));
  return c;
}

// TGPU_INDEX_TIMING=2: HIP events between the index's launches (stderr)
struct PhaseTimer {
  hipStream_t s;
  bool on;
  int n = 0;
  hipEvent_t ev[32];
  const char* name[32];
  PhaseTimer(hipStream_t st) : s(st) {
    const char* e = getenv("TGPU_INDEX_TIMING");
    on = e && e[0] == '2';
    mark("start");
  }
  void mark(const char* what) {
    if (!on || n >= 32) return;
    (void)hipEventCreate(&ev[n]);
    (void)hipEventRecord(ev[n], s);
    name[n++] = what;
  }
  ~PhaseTimer() {
    if (!on) return;
    (void)hipEventSynchronize(ev[n - 1]);
    for (int k = 1; k < n; ++k) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, ev[k - 1], ev[k]);
      fprintf(stderr, "  %-10s %.3f ms\n", name[k], ms);
    }
    for (int k = 0; k < n; ++k) (void)hipEventDestroy(ev[k]);
  }
};

// What the general-reader helpers would find after the tile speculation:
// scal[8] tiles the program left partial (index_cont), scal[9] tiles without
// a start (index_spec_fallback), scal[10] broken links (index_merge).
__global__ __launch_bounds__(256) void index_summary_kernel(IndexArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  bool partial = false, none = false, broken = false;
  if (j < a.n_chunks) {
    const uint64_t s0 = a.s[j], e0 = a.e[j];
    partial = e0 == kPartial;
    none = s0 == kNo && e0 == kNo;
    if (j > 0 && e0 != kErr && e0 != kPartial) {
      const uint64_t T = a.e[j - 1];
      broken = T != kNo && T != kErr && T != kPartial && s0 != T;
    }
  }
  const int np = __syncthreads_count(partial), nn = __syncthreads_count(none),
            nb = __syncthreads_count(broken);
  if (threadIdx.x == 0) {
    if (np) atomicAdd(&a.scal[8], (unsigned long long)np);
    if (nn) atomicAdd(&a.scal[9], (unsigned long long)nn);
    if (nb) atomicAdd(&a.scal[10], (unsigned long long)nb);
  }
}

hipError_t launch_index_stream(const IndexArgs& a, hipStream_t stream, const JitKernels* jit,
                               bool* fused, uint64_t* h_sync, const XTabAlloc* xalloc) {
  PhaseTimer pt(stream);
  {  // (merge-round counters, the exhaustive resolution's flag)
    const hipError_t e0 = hipMemsetAsync(a.scal + 16, 0, 8 * sizeof(unsigned long long), stream);
    if (e0 != hipSuccess) return e0;
  }
  // (st_decode: the caller decodes from the index; the finish keeps the tail rule)
  const bool decode = a.recs && a.prog && a.chunk == kTile && !a.st_decode;
  if (fused) *fused = decode;
  const uint64_t C = a.n_chunks;
  const dim3 g((uint32_t)((C + 255) / 256)), b(256);
  const dim3 sg((uint32_t)std::min<uint64_t>((C + 255) / 256, kScratchGrid));
  bool need_cont = true, need_fallback = true, need_merge = true;
  const bool tiles = a.prog && a.chunk == kTile;
  if (pt.on) (void)hipMemsetAsync(a.scal + 12, 0, 4 * sizeof(unsigned long long), stream);
  if (tiles) {
    if (jit) {
      const hipError_t e = jit_launch_index(jit, 0, a, C, stream);
      if (e != hipSuccess) return e;
    } else {
      hipLaunchKernelGGL(index_tile_spec_kernel, dim3((uint32_t)C), dim3(kTileLanes), 0, stream, a);
    }
  } else if (a.prog) {
    hipLaunchKernelGGL(index_spec_kernel, g, b, 0, stream, a);
  } else {
    TGPU_BY_PROTOCOL(a.protocol, hipLaunchKernelGGL(index_spec_general_kernel<P_>, g, b, 0, stream, a));
  }
  pt.mark("spec");
  if (pt.on && jit) {  // (TGPU_SPEC_CHECK builds: stuck tiles, of them with LDS != HBM, words)
    uint64_t d[4] = {};
    (void)hipMemcpyAsync(d, a.scal + 12, sizeof(d), hipMemcpyDeviceToHost, stream);
    (void)hipStreamSynchronize(stream);
    fprintf(stderr, "  spec check: threads whose staged words changed after the staging barrier %llu; stuck %llu, "
            "staged copy differs at the end %llu, words %llu\n", (unsigned long long)d[0],
            (unsigned long long)d[1], (unsigned long long)d[2], (unsigned long long)d[3]);
  }
  // what the speculation left to repair: read mid-call by blocking tile
  // calls (to skip the helpers nothing needs), kept for tgpu_index_stats
  hipError_t e = hipMemsetAsync(a.scal + 8, 0, 3 * sizeof(unsigned long long), stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(index_summary_kernel, g, b, 0, stream, a);
  if (tiles && h_sync) {
    e = hipMemcpyAsync(h_sync, a.scal + 8, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return e;
    // the fallback and the repair act on what the continuation leaves
    need_cont = h_sync[0] != 0;
    need_fallback = need_cont || h_sync[1] != 0;
    need_merge = need_fallback || h_sync[2] != 0;
    pt.mark("summary");
    if (pt.on)
      fprintf(stderr, "  tiles %llu: partial %llu, no start %llu, broken links %llu\n",
              (unsigned long long)C, (unsigned long long)h_sync[0],
              (unsigned long long)h_sync[1], (unsigned long long)h_sync[2]);
  }
  if (a.prog && need_cont)
    TGPU_BY_PROTOCOL(a.protocol, hipLaunchKernelGGL(index_cont_kernel<P_>, sg, b, 0, stream, a));
  pt.mark("cont");
  // (a speculative range opens at its first program-confirmed start: a
  // general-reader start there has no predecessor chunk to verify it)
  if (a.prog && !a.speculative && need_fallback)
    TGPU_BY_PROTOCOL(a.protocol, hipLaunchKernelGGL(index_spec_fallback_kernel<P_>, sg, b, 0, stream, a));
  pt.mark("fallback");
  if (need_merge) {
    // Jacobi rounds of the parallel repair (TGPU_MERGE_ROUNDS, default 6;
    // rounds after one that changed nothing return at once)
    int rounds = 6;
    if (const char* v = getenv("TGPU_MERGE_ROUNDS")) rounds = atoi(v);
    for (int r = 0; r < rounds; ++r) {
      hipLaunchKernelGGL(index_merge_snap_kernel, sg, b, 0, stream, a, r);
      TGPU_BY_PROTOCOL(a.protocol, hipLaunchKernelGGL(index_merge_round_kernel<P_>, sg, b, 0, stream,
                                                      a, r));
    }
  }
  // sst is written by the general speculation and the fallback only (and by
  // the fallback only when it ran: a skipped one leaves an earlier call's
  // starts in the reused workspace)
  const int sst_valid = !a.prog || (!a.speculative && need_fallback);
  pt.mark("merge");
  hipLaunchKernelGGL(index_flag_kernel, g, b, 0, stream, a, sst_valid);
  e = launch_scan_tiles(a.base, C, a.part, a.scal, nullptr, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(index_list_kernel, g, b, 0, stream, a);
  // the exhaustive resolution of a program-less stream's links (blocking
  // calls), opt-in: TGPU_INDEX_EXHAUSTIVE=1 always, =2 when more than 64
  // links are broken (the count read mid-call). Measured slower than the
  // merge rounds once the speculation's reach follows the record length
  // (1.6-3.0 s against 78 ms on the adversarial stream)
  if (h_sync && xalloc && !a.prog && !a.speculative && a.chunk <= kXChunk) {
    const char* xv = getenv("TGPU_INDEX_EXHAUSTIVE");
    const int mode = xv ? atoi(xv) : 0;
    uint64_t bad = 0;
    if (mode == 2) {
      e = hipMemcpyAsync(h_sync, a.scal, sizeof(uint64_t), hipMemcpyDeviceToHost, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      if (e != hipSuccess) return e;
      bad = h_sync[0];
    }
    if (mode == 1 || (mode == 2 && bad > 64)) {
      const uint32_t grid = (uint32_t)std::min<uint64_t>(C, 1024);
      const uint64_t rs = (a.rec_size + 15) & ~15ull;
      const uint64_t tab = C * kXWindow;
      const uint64_t bytes = tab * 8 + ((tab * 4 + 15) & ~15ull) + (uint64_t)grid * 256 * rs;
      uint8_t* w = xalloc->get(xalloc->user, bytes);
      if (w) {
        IndexArgs y = a;
        y.xe = (uint64_t*)w;
        y.xc = (uint32_t*)(w + tab * 8);
        y.xscratch = w + tab * 8 + ((tab * 4 + 15) & ~15ull);
        TGPU_BY_PROTOCOL(a.protocol, hipLaunchKernelGGL(index_xtab_kernel<P_>, dim3(grid), b, 0,
                                                        stream, y));
        TGPU_BY_PROTOCOL(a.protocol, hipLaunchKernelGGL(index_xresolve_kernel<P_>, dim3(1), dim3(64),
                                                        0, stream, y));
        pt.mark("exhaustive");
      }
    }
  }
  TGPU_BY_PROTOCOL(a.protocol, hipLaunchKernelGGL(index_fix_kernel<P_>, dim3(1), dim3(64), 0, stream, a));
  pt.mark("fix");
  hipLaunchKernelGGL(index_prep_kernel, g, b, 0, stream, a);
  e = launch_scan_tiles(a.base, C, a.part, nullptr, nullptr, stream);
  if (e != hipSuccess) return e;
  IndexArgs x = a;
  if (!decode) x.recs = nullptr;
  // stored starts: copied by a light kernel; the emit tiles re-walk only the
  // tiles it lists, a grid of at most ~6 resident workgroups per CU looping
  const bool copy = !decode && a.st16 && a.prog && a.chunk == kTile;
  if (!copy) x.st16 = nullptr;
  const uint64_t emit_grid = copy ? std::min<uint64_t>(C, 2048) : C;
  pt.mark("prep");
  if (copy)
    hipLaunchKernelGGL(index_starts_copy_kernel, dim3((uint32_t)((C + 3) / 4)), dim3(256), 0, stream,
                       x);
  pt.mark("copy");
  if (a.prog && a.chunk == kTile && jit) {
    e = jit_launch_index(jit, decode ? 2 : 1, x, decode ? C : emit_grid, stream);
    if (e != hipSuccess) return e;
  } else if (decode) {
    hipLaunchKernelGGL(index_tile_decode_kernel, dim3((uint32_t)C), dim3(kTileLanes), 0, stream, x);
  } else if (a.prog && a.chunk == kTile)
    hipLaunchKernelGGL(index_tile_emit_kernel, dim3((uint32_t)emit_grid), dim3(kTileLanes), 0,
                       stream, x);
  else
    hipLaunchKernelGGL(index_emit_kernel, g, b, 0, stream, a);
  pt.mark("emit");
  // the emit's continuation only has work where a re-walked tile stopped
  // (copied tiles never do): with host reads, the finish goes first (it does
  // not depend on it) and one read gives both the re-walk count and the total
  const bool defer = copy && h_sync;
  if (defer) {
    e = launch_index_finish(a, decode || (a.st_decode && a.recs), stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h_sync, a.scal + 6, sizeof(uint64_t),
                                            hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(h_sync + 3, a.scal + 5, sizeof(uint64_t), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return e;
    pt.mark("finish");
    if (pt.on) fprintf(stderr, "  re-walked tiles %llu\n", (unsigned long long)h_sync[0]);
  }
  if (!defer || h_sync[0]) {
    TGPU_BY_PROTOCOL(a.protocol, hipLaunchKernelGGL(index_emit_cont_kernel<P_>, sg, b, 0, stream, x));
    if (a.deep.lanes)
      TGPU_BY_PROTOCOL(a.protocol, hipLaunchKernelGGL(index_deep_emit_kernel<P_>,
                                                      dim3((a.deep.lanes + 63) / 64), dim3(64), 0,
                                                      stream, x));
    pt.mark("emit_cont");
  }
  if (defer) return hipGetLastError();
  const hipError_t fe = launch_index_finish(a, decode || (a.st_decode && a.recs), stream);
  pt.mark("cont+fin");
  return fe;
}

hipError_t launch_index_finish(const IndexArgs& a, bool decode, hipStream_t stream) {
  hipLaunchKernelGGL(index_finish_kernel, dim3(1), dim3(64), 0, stream, a, a.scal + 5);
  if (decode)
    hipLaunchKernelGGL(index_decode_tail_kernel, dim3(1), dim3(64), 0, stream, a, a.scal + 5);
  if (a.fill_to > 0)
    hipLaunchKernelGGL(index_pad_kernel, dim3((uint32_t)((a.fill_to + 256) / 256)), dim3(256), 0,
                       stream, a, a.scal + 5);
  return hipGetLastError();
}

hipError_t launch_index_onepass(const IndexArgs& a, hipStream_t stream, const JitKernels* jit,
                                bool rr) {
  const uint64_t C = a.n_chunks;
  if (!a.prog || a.chunk != kTile || C == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(index_onepass_init_kernel, dim3((uint32_t)((C + 255) / 256)), dim3(256), 0,
                     stream, a);
  const bool decode = a.recs != nullptr;
  if (rr) return jit_launch_index(jit, 5, a, C, stream);  // (the caller checked jit_has)
  if (jit) return jit_launch_index(jit, decode ? 4 : 3, a, C, stream);
  if (decode)
    hipLaunchKernelGGL(index_onepass_kernel<true>, dim3((uint32_t)C), dim3(kTileLanes), 0, stream, a);
  else
    hipLaunchKernelGGL(index_onepass_kernel<false>, dim3((uint32_t)C), dim3(kTileLanes), 0, stream,
                       a);
  return hipGetLastError();
}

}  // namespace tgpu
