// tgpu_host.cpp — the host-memory path: records and
// wire bytes that start and end in host memory, the way the reference's
// callers hold them (an IOBuf from a socket or file,
// thrift/lib/cpp2/protocol/Serializer.h:62-72,136-148). A batch is cut into
// chunks of records; three slots (stream + device buffers + result context)
// rotate so that chunk k+1's host->device copy, chunk k's kernels and chunk
// k-1's device->host copy run at the same time (the copy engines of both
// directions and the CUs all busy). The bulk rate is bounded by PCIe, not
// by the kernels: DESIGN.md §6.1 has the measured numbers.
//
// The chunk pipeline needs records of a fixed canonical Binary length (the
// fixed-layout path: BASELINE configs 1/2), where chunk boundaries are known
// without parsing. A chunk whose decode does not end exactly on its boundary
// (a non-canonical record changed the lengths, or a malformed record) is
// redone with the whole rest of the stream resident, so results and errors
// are exactly the single-call ones. Variable-length streams (no lists) take
// that resident path from the start: copy in, fused index + decode, copy out.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "tgpu_internal.h"

namespace {

constexpr int kSlots = 3;
constexpr uint64_t kDefaultChunk = 1ull << 22;  // records per chunk

// A device buffer kept by the pipe across calls, grown on demand (the
// chunk pipelines' workspaces: hipMalloc / hipFree of hundreds of MiB per
// call cost more than the copies they serve). Calls are blocking, so a
// buffer is idle whenever a call starts and may be replaced then.
struct GrowBuf {
  uint8_t* p = nullptr;
  uint64_t cap = 0;
  bool reserve(uint64_t n) {
    n = std::max<uint64_t>(n, 16);
    if (n <= cap) return true;
    release();
    if (hipMalloc(&p, n) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      return false;
    }
    cap = n;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostPipe {
  int device = 0;
  hipStream_t s[kSlots] = {};
  tgpu_context* c[kSlots] = {};
  uint8_t* d_in[kSlots] = {};
  uint8_t* d_out[kSlots] = {};
  uint64_t in_cap = 0, out_cap = 0;
  // tgpu_decode_host_chunks: the stream, records, arena, offsets; packed
  // list elements, the packing's tile sums and scan partials, totals
  GrowBuf din, drec, dar, doffs, dpk, psum, ppart, ptot;
  // tgpu_encode_host_chunks: two slots of records, strings, lists, wire
  GrowBuf erec[2], estr[2], elst[2], eout[2];
};

void pipe_free_buffers(HostPipe* p) {
  for (int k = 0; k < kSlots; ++k) {
    if (p->d_in[k]) (void)hipFree(p->d_in[k]);
    if (p->d_out[k]) (void)hipFree(p->d_out[k]);
    p->d_in[k] = p->d_out[k] = nullptr;
  }
  p->in_cap = p->out_cap = 0;
}

int pipe_reserve(HostPipe* p, uint64_t in_bytes, uint64_t out_bytes) {
  if (in_bytes <= p->in_cap && out_bytes <= p->out_cap) return TGPU_OK;
  pipe_free_buffers(p);
  for (int k = 0; k < kSlots; ++k)
    if (hipMalloc(&p->d_in[k], std::max<uint64_t>(in_bytes, 16)) != hipSuccess ||
        hipMalloc(&p->d_out[k], std::max<uint64_t>(out_bytes, 16)) != hipSuccess)
      return TGPU_ERR_HIP;
  p->in_cap = in_bytes;
  p->out_cap = out_bytes;
  return TGPU_OK;
}

// Host buffers are DMA'd directly when pinned; pageable ones are pinned in
// place for the duration of the call (hipHostRegister).
struct PinGuard {
  void* p = nullptr;
  bool registered = false;
  PinGuard(const void* ptr, uint64_t bytes) {
    if (!ptr || !bytes) return;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, ptr) == hipSuccess && at.type == hipMemoryTypeHost) return;
    (void)hipGetLastError();
    if (hipHostRegister(const_cast<void*>(ptr), bytes, hipHostRegisterDefault) == hipSuccess) {
      p = const_cast<void*>(ptr);
      registered = true;
    } else {
      (void)hipGetLastError();  // pageable copies still work, only slower
    }
  }
  ~PinGuard() {
    if (registered) (void)hipHostUnregister(p);
  }
};

void set_status(tgpu_status* st, int code, uint64_t record, uint64_t off) {
  if (!st) return;
  std::memset(st, 0, sizeof(*st));
  st->code = code;
  tgpu_code_classify(code, &st->exc_class, &st->tproto_type);
  st->record = record;
  st->byte_offset = off;
}

}  // namespace

namespace tgpu {

void* host_pipe_create() {
  auto* p = new (std::nothrow) HostPipe();
  if (!p) return nullptr;
  (void)hipGetDevice(&p->device);
  for (int k = 0; k < kSlots; ++k) {
    if (hipStreamCreateWithFlags(&p->s[k], hipStreamNonBlocking) != hipSuccess ||
        tgpu_context_create(&p->c[k]) != TGPU_OK) {
      host_pipe_destroy(p);
      return nullptr;
    }
  }
  return p;
}

void host_pipe_destroy(void* vp) {
  auto* p = (HostPipe*)vp;
  if (!p) return;
  for (int k = 0; k < kSlots; ++k) {
    if (p->s[k]) (void)hipStreamSynchronize(p->s[k]);
    if (p->c[k]) tgpu_context_destroy(p->c[k]);
    if (p->s[k]) (void)hipStreamDestroy(p->s[k]);
  }
  pipe_free_buffers(p);
  for (GrowBuf* b : {&p->din, &p->drec, &p->dar, &p->doffs, &p->dpk, &p->psum, &p->ppart, &p->ptot})
    b->release();
  for (int k = 0; k < 2; ++k)
    for (GrowBuf* b : {&p->erec[k], &p->estr[k], &p->elst[k], &p->eout[k]}) b->release();
  delete p;
}

// One direction of the pipeline over chunks of `chunk` records.
//   decode: host wire (L bytes/record) -> host records (S bytes/record)
//   encode: host records -> host wire
// Returns the first failing chunk's status (record / byte offset relative to
// the batch), or OK; *done_records / *done_bytes = what completed before it.
int host_pipeline(void* vp, const tgpu_schema* schema, int protocol, bool decode,
                  const uint8_t* h_src, uint8_t* h_dst, uint64_t n, uint64_t chunk, uint32_t L,
                  uint32_t S, const tgpu_limits* limits, tgpu_status* st, uint64_t* first_bad_chunk,
                  uint64_t* done_records) {
  auto* p = (HostPipe*)vp;
  const uint32_t in_w = decode ? L : S, out_w = decode ? S : L;
  int rc = pipe_reserve(p, chunk * in_w, chunk * out_w);
  if (rc) return rc;
  const uint64_t nchunks = (n + chunk - 1) / chunk;
  uint64_t issued = 0, waited = 0;
  *first_bad_chunk = ~0ull;
  *done_records = 0;
  int result = TGPU_OK;
  // wait for chunk w's slot and check its status; false stops the pipeline
  auto wait_chunk = [&](uint64_t w) -> bool {
    const int k = (int)(w % kSlots);
    const uint64_t r0 = w * chunk, m = std::min(chunk, n - r0);
    tgpu_status cs;
    uint64_t nd = 0, bytes = 0;
    const int code = tgpu_context_wait(p->c[k], p->s[k], &cs, &nd, &bytes);
    if (code == TGPU_OK && bytes == m * L) {  // consumed / written exactly the chunk
      *done_records = r0 + m;
      return true;
    }
    if (code == TGPU_ERR_HIP) {
      result = TGPU_ERR_HIP;
      set_status(st, TGPU_ERR_HIP, r0, 0);
      return false;
    }
    *first_bad_chunk = w;
    if (decode) {
      result = TGPU_ERR_INDEX_MISMATCH;  // caller redoes from this chunk
    } else {
      result = code;
      set_status(st, code, r0 + cs.record, r0 * L + cs.byte_offset);
    }
    return false;
  };
  bool ok = true;
  while (waited < nchunks && ok) {
    // keep kSlots chunks in flight
    while (issued < nchunks && issued - waited < (uint64_t)kSlots) {
      const int k = (int)(issued % kSlots);
      const uint64_t r0 = issued * chunk, m = std::min(chunk, n - r0);
      hipError_t e = hipMemcpyAsync(p->d_in[k], h_src + r0 * in_w, m * in_w,
                                    hipMemcpyHostToDevice, p->s[k]);
      if (e != hipSuccess) {
        set_status(st, TGPU_ERR_HIP, r0, 0);
        return TGPU_ERR_HIP;
      }
      int crc;
      if (decode)
        crc = tgpu_decode_batch(p->c[k], schema, protocol, p->d_in[k], m * L, nullptr, m,
                                p->d_out[k], nullptr, 0, limits, p->s[k], nullptr, nullptr,
                                nullptr);
      else
        crc = tgpu_encode_batch(p->c[k], schema, protocol, p->d_in[k], m, nullptr, nullptr,
                                p->d_out[k], m * L, nullptr, p->s[k], nullptr, nullptr);
      if (crc) {
        set_status(st, crc, r0, 0);
        return crc;
      }
      e = hipMemcpyAsync(h_dst + r0 * out_w, p->d_out[k], m * out_w, hipMemcpyDeviceToHost,
                         p->s[k]);
      if (e != hipSuccess) {
        set_status(st, TGPU_ERR_HIP, r0, 0);
        return TGPU_ERR_HIP;
      }
      ++issued;
    }
    ok = wait_chunk(waited++);
  }
  // drain what is still in flight after a stop
  for (uint64_t w = waited; w < issued; ++w) (void)hipStreamSynchronize(p->s[w % kSlots]);
  return result;
}

}  // namespace tgpu

using namespace tgpu;

extern "C" {

int tgpu_decode_host(tgpu_context* ctx, const tgpu_schema* schema, int protocol, const void* h_in,
                     uint64_t in_len, uint64_t n, void* h_records, uint64_t chunk_records,
                     const tgpu_limits* limits, tgpu_status* st, uint64_t* n_decoded,
                     uint64_t* consumed) {
  if (!ctx || !schema || (n && (!h_in || !h_records))) {
    set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const uint64_t L = tgpu_schema_fixed_wire_size(schema, protocol);
  const uint32_t S = tgpu_schema_record_size(schema);
  // variable-length records without lists: one resident decode (below) of
  // the whole stream; string spans index the host stream like the device's.
  // Lists would need a host list arena in the ABI: not supported here.
  if (!L && schema_has_lists(schema)) {
    set_status(st, TGPU_ERR_UNSUPPORTED, 0, 0);
    return TGPU_ERR_UNSUPPORTED;
  }
  void* pipe = context_host_pipe(ctx);
  if (!pipe) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  const uint64_t chunk = chunk_records ? chunk_records : kDefaultChunk;
  PinGuard pin_in(h_in, in_len), pin_out(h_records, n * S);
  // the pipelined part: whole records the stream holds at the canonical length
  const uint64_t fast_n = L ? std::min<uint64_t>(n, in_len / L) : 0;
  uint64_t bad = ~0ull, done = 0;
  int rc = TGPU_OK;
  if (fast_n)
    rc = host_pipeline(pipe, schema, protocol, true, (const uint8_t*)h_in, (uint8_t*)h_records,
                       fast_n, chunk, (uint32_t)L, S, limits, st, &bad, &done);
  if (rc && rc != TGPU_ERR_INDEX_MISMATCH) return rc;
  if (done == n) {
    set_status(st, TGPU_OK, n, 0);
    if (n_decoded) *n_decoded = n;
    if (consumed) *consumed = n * L;
    return TGPU_OK;
  }
  // the rest (from the first chunk that did not end on its boundary, or the
  // records past the canonical length) in one resident call: exact results
  const uint64_t r0 = done, off = done * L;
  const uint64_t rest_len = in_len - off, rest_n = n - r0;
  uint8_t *d_in = nullptr, *d_out = nullptr;
  if (hipMalloc(&d_in, std::max<uint64_t>(rest_len, 16)) != hipSuccess ||
      hipMalloc(&d_out, std::max<uint64_t>(rest_n * S, 16)) != hipSuccess) {
    if (d_in) (void)hipFree(d_in);
    set_status(st, TGPU_ERR_HIP, r0, 0);
    return TGPU_ERR_HIP;
  }
  hipStream_t s = nullptr;
  tgpu_status cs;
  uint64_t nd = 0, cons = 0;
  int code = TGPU_ERR_HIP;
  if (hipMemcpy(d_in, (const uint8_t*)h_in + off, rest_len, hipMemcpyHostToDevice) == hipSuccess) {
    code = tgpu_decode_batch(ctx, schema, protocol, d_in, rest_len, nullptr, rest_n, d_out,
                             nullptr, 0, limits, s, &cs, &nd, &cons);
    // records before the failure (and the partial failing one) go back
    const uint64_t back = std::min<uint64_t>(rest_n, nd + (code ? 1 : 0));
    if (code != TGPU_ERR_HIP &&
        hipMemcpy((uint8_t*)h_records + r0 * S, d_out, back * S, hipMemcpyDeviceToHost) !=
            hipSuccess)
      code = TGPU_ERR_HIP;
  }
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  if (code == TGPU_ERR_HIP) {
    set_status(st, TGPU_ERR_HIP, r0, 0);
    return TGPU_ERR_HIP;
  }
  if (st) {
    *st = cs;
    st->record = code ? r0 + cs.record : n;
    if (code) st->byte_offset = off + cs.byte_offset;
  }
  if (n_decoded) *n_decoded = r0 + nd;
  if (consumed) *consumed = off + cons;
  return code;
}

int tgpu_encode_host(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                     const void* h_records, uint64_t n, void* h_out, uint64_t out_capacity,
                     uint64_t chunk_records, tgpu_status* st, uint64_t* out_size) {
  if (!ctx || !schema || (n && (!h_records || !h_out))) {
    set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const uint64_t L = tgpu_schema_fixed_wire_size(schema, protocol);
  const uint32_t S = tgpu_schema_record_size(schema);
  if (!L) {
    set_status(st, TGPU_ERR_UNSUPPORTED, 0, 0);
    return TGPU_ERR_UNSUPPORTED;
  }
  void* pipe = context_host_pipe(ctx);
  if (!pipe) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  const uint64_t chunk = chunk_records ? chunk_records : kDefaultChunk;
  // records that fit the output; the first one that does not is the
  // reference's overflow point (TGPU_ERR_OUTPUT_OVERFLOW, as the device call)
  const uint64_t fit = std::min<uint64_t>(n, out_capacity / L);
  PinGuard pin_in(h_records, n * S), pin_out(h_out, fit * L);
  uint64_t bad = ~0ull, done = 0;
  int rc = TGPU_OK;
  if (fit)
    rc = host_pipeline(pipe, schema, protocol, false, (const uint8_t*)h_records, (uint8_t*)h_out,
                       fit, chunk, (uint32_t)L, S, nullptr, st, &bad, &done);
  if (rc) {
    if (out_size) *out_size = done * L;
    return rc;
  }
  if (fit < n) {
    set_status(st, TGPU_ERR_OUTPUT_OVERFLOW, fit, fit * L);
    if (out_size) *out_size = fit * L;
    return TGPU_ERR_OUTPUT_OVERFLOW;
  }
  set_status(st, TGPU_OK, n, 0);
  if (out_size) *out_size = n * L;
  return TGPU_OK;
}

// ---- any schema: one resident pass (copy in, device call, copy out) -------
namespace {
struct DevBuf {
  uint8_t* p = nullptr;
  bool alloc(uint64_t n) { return hipMalloc(&p, std::max<uint64_t>(n, 16)) == hipSuccess; }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};
}  // namespace

int tgpu_decode_host_ex(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                        const void* h_in, uint64_t in_len, uint64_t n, void* h_records,
                        void* h_arena, uint64_t arena_capacity, const tgpu_limits* limits,
                        tgpu_status* st, uint64_t* n_decoded, uint64_t* consumed) {
  if (n_decoded) *n_decoded = 0;
  if (consumed) *consumed = 0;
  if (!ctx || !schema || (n && (!h_in || !h_records)) || (arena_capacity && !h_arena)) {
    set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const uint32_t S = tgpu_schema_record_size(schema);
  PinGuard pin_in(h_in, in_len), pin_rec(h_records, n * S), pin_ar(h_arena, arena_capacity);
  DevBuf din, drec, dar;
  if (!din.alloc(in_len) || !drec.alloc(n * S) || (arena_capacity && !dar.alloc(arena_capacity))) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  tgpu_status cs{};
  uint64_t nd = 0, cons = 0;
  int code = TGPU_ERR_HIP;
  if (hipMemcpy(din.p, h_in, in_len, hipMemcpyHostToDevice) == hipSuccess) {
    code = tgpu_decode_batch(ctx, schema, protocol, din.p, in_len, nullptr, n, drec.p,
                             arena_capacity ? dar.p : nullptr, arena_capacity, limits, nullptr,
                             &cs, &nd, &cons);
    // the records before the failure and the partial failing one go back,
    // and the arena (its bytes outside the spans are unspecified)
    const uint64_t back = std::min<uint64_t>(n, nd + (code ? 1 : 0));
    if (code != TGPU_ERR_HIP &&
        (hipMemcpy(h_records, drec.p, back * S, hipMemcpyDeviceToHost) != hipSuccess ||
         (arena_capacity &&
          hipMemcpy(h_arena, dar.p, arena_capacity, hipMemcpyDeviceToHost) != hipSuccess)))
      code = TGPU_ERR_HIP;
  }
  if (code == TGPU_ERR_HIP) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  if (st) *st = cs;
  if (n_decoded) *n_decoded = nd;
  if (consumed) *consumed = cons;
  return code;
}

int tgpu_encode_host_ex(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                        const void* h_records, uint64_t n, const void* h_strings,
                        uint64_t strings_len, const void* h_lists, uint64_t lists_len,
                        void* h_out, uint64_t out_capacity, uint64_t* h_out_offsets,
                        tgpu_status* st, uint64_t* out_size) {
  if (out_size) *out_size = 0;
  if (!ctx || !schema || (n && (!h_records || !h_out)) || (strings_len && !h_strings) ||
      (lists_len && !h_lists)) {
    set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const uint32_t S = tgpu_schema_record_size(schema);
  PinGuard pin_rec(h_records, n * S), pin_s(h_strings, strings_len), pin_l(h_lists, lists_len),
      pin_out(h_out, out_capacity);
  DevBuf drec, dstr, dlist, dout, doffs;
  if (!drec.alloc(n * S) || !dstr.alloc(strings_len) || !dlist.alloc(lists_len) ||
      !dout.alloc(out_capacity) || (h_out_offsets && !doffs.alloc((n + 1) * 8))) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  if (hipMemcpy(drec.p, h_records, n * S, hipMemcpyHostToDevice) != hipSuccess ||
      (strings_len && hipMemcpy(dstr.p, h_strings, strings_len, hipMemcpyHostToDevice) != hipSuccess) ||
      (lists_len && hipMemcpy(dlist.p, h_lists, lists_len, hipMemcpyHostToDevice) != hipSuccess)) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  tgpu_status cs{};
  uint64_t size = 0;
  int code = tgpu_encode_batch(ctx, schema, protocol, drec.p, n, dstr.p, dlist.p, dout.p,
                               out_capacity, h_out_offsets ? (uint64_t*)doffs.p : nullptr,
                               nullptr, &cs, &size);
  if (code != TGPU_ERR_HIP &&
      (hipMemcpy(h_out, dout.p, std::min(size, out_capacity), hipMemcpyDeviceToHost) !=
           hipSuccess ||
       (h_out_offsets && code == TGPU_OK &&
        hipMemcpy(h_out_offsets, doffs.p, (n + 1) * 8, hipMemcpyDeviceToHost) != hipSuccess)))
    code = TGPU_ERR_HIP;
  if (code == TGPU_ERR_HIP) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  if (st) *st = cs;
  if (out_size) *out_size = size;
  return code;
}

// ---- packed list elements (tgpu_decode_host_chunks_ex, TGPU_HOST_PACK_LISTS)
// The decoded list arena follows the position rule (an element array at
// scale x its wire position), so a chunk's arena slice is as large as its
// wire (x scale) whatever share of it the elements are: config 4 sends 373 MB
// of slices back for 134 MB of elements. Packing moves a finished chunk's
// element arrays to the front of its slice (record order, no gaps) in a
// second buffer laid out like the host arena and points the records' spans
// there, so only the records and the packed bytes cross PCIe back.
namespace {
constexpr uint32_t kPackMax = 8;
struct PackSpec {
  uint32_t n;
  uint32_t member[kPackMax];
  uint32_t width[kPackMax];
};

__device__ __forceinline__ uint64_t pack_bytes(const uint8_t* rec, const PackSpec& ps) {
  uint64_t b = 0;
  for (uint32_t f = 0; f < ps.n; ++f)
    b += (uint64_t)((const tgpu_span*)(rec + ps.member[f]))->length * ps.width[f];
  return b;
}

// inclusive-scan helper of one 256-thread block: returns the exclusive prefix
// of v, *total the block's sum
__device__ __forceinline__ unsigned long long block_scan256(unsigned long long v,
                                                            unsigned long long* wsum,
                                                            unsigned long long* total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  unsigned long long before = 0, all = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    before += k < w ? wsum[k] : 0;
    all += wsum[k];
  }
  *total = all;
  return before + x - v;
}

__global__ __launch_bounds__(256) void pack_size_kernel(const uint8_t* __restrict__ recs, uint64_t n,
                                                        uint32_t S, PackSpec ps,
                                                        unsigned long long* __restrict__ sums) {
  __shared__ unsigned long long wsum[4];
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const unsigned long long b = i < n ? pack_bytes(recs + i * S, ps) : 0;
  unsigned long long total;
  (void)block_scan256(b, wsum, &total);
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// sums: the scanned tile sums. Element arrays of record i go to
// dst[base + its prefix ..), its spans are rewritten to there (one lane per
// record, word copies where both ends share an alignment).
__global__ __launch_bounds__(256) void pack_copy_kernel(uint8_t* __restrict__ recs, uint64_t n,
                                                        uint32_t S, PackSpec ps,
                                                        const unsigned long long* __restrict__ sums,
                                                        const uint8_t* __restrict__ arena,
                                                        uint8_t* __restrict__ dst, uint64_t base) {
  __shared__ unsigned long long wsum[4];
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint8_t* rec = recs + i * S;
  const unsigned long long b = i < n ? pack_bytes(rec, ps) : 0;
  unsigned long long total;
  uint64_t off = base + sums[blockIdx.x] + block_scan256(b, wsum, &total);
  if (i >= n) return;
  for (uint32_t f = 0; f < ps.n; ++f) {
    tgpu_span* sp = (tgpu_span*)(rec + ps.member[f]);
    const uint64_t bytes = (uint64_t)sp->length * ps.width[f];
    if (!bytes) continue;
    const uint8_t* src = arena + sp->offset;
    uint8_t* d = dst + off;
    // words of the widest size both ends share the alignment of (8 / 4 /
    // 2 / 1 bytes: element arrays are 8-aligned in the arena, the packed
    // offsets step by the element width), bytes up to it and after
    const uintptr_t mis = ((uintptr_t)src ^ (uintptr_t)d) | 8;
    const uint32_t wsz = (uint32_t)(mis & (~mis + 1));
    uint64_t k = 0;
    for (; k < bytes && (((uintptr_t)src + k) & (wsz - 1)); ++k) d[k] = src[k];
    if (wsz == 8) {
      for (; k + 8 <= bytes; k += 8) *(uint64_t*)(d + k) = *(const uint64_t*)(src + k);
    } else if (wsz == 4) {
      for (; k + 4 <= bytes; k += 4) *(uint32_t*)(d + k) = *(const uint32_t*)(src + k);
    } else if (wsz == 2) {
      for (; k + 2 <= bytes; k += 2) *(uint16_t*)(d + k) = *(const uint16_t*)(src + k);
    }
    for (; k < bytes; ++k) d[k] = src[k];
    sp->offset = off;
    off += bytes;
  }
}
}  // namespace

// ---- any schema, chunk-pipelined (tgpu_decode_host_chunks /
// tgpu_encode_host_chunks) ---------------------------------------------------
namespace {
constexpr uint64_t kDefaultChunkBytes = 64ull << 20;
constexpr uint64_t kDefaultChunkRecords = 1ull << 20;

struct Events {
  std::vector<hipEvent_t> ev;
  explicit Events(size_t n) : ev(n, nullptr) {
    for (auto& e : ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  }
  ~Events() {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

struct Range {
  uint64_t r0, r1;
  hipEvent_t done;
};
}  // namespace

int tgpu_decode_host_chunks(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                            const void* h_in, uint64_t in_len, uint64_t n, void* h_records,
                            void* h_arena, uint64_t arena_capacity, const tgpu_limits* limits,
                            uint64_t chunk_bytes, tgpu_chunk_fn on_chunk, void* user,
                            tgpu_status* st, uint64_t* n_decoded, uint64_t* consumed) {
  return tgpu_decode_host_chunks_ex(ctx, schema, protocol, h_in, in_len, n, h_records, h_arena,
                                    arena_capacity, limits, chunk_bytes, 0u, on_chunk, user, st,
                                    n_decoded, consumed);
}

int tgpu_decode_host_chunks_ex(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                               const void* h_in, uint64_t in_len, uint64_t n, void* h_records,
                               void* h_arena, uint64_t arena_capacity, const tgpu_limits* limits,
                               uint64_t chunk_bytes, uint32_t flags, tgpu_chunk_fn on_chunk,
                               void* user, tgpu_status* st, uint64_t* n_decoded,
                               uint64_t* consumed) {
  if (n_decoded) *n_decoded = 0;
  if (consumed) *consumed = 0;
  if (!ctx || !schema || (n && (!h_in || !h_records)) || (arena_capacity && !h_arena)) {
    set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const uint64_t C = chunk_bytes ? chunk_bytes : kDefaultChunkBytes;
  const uint32_t S = tgpu_schema_record_size(schema);
  const uint64_t scale = tgpu_schema_arena_scale(schema, protocol);
  auto resident_all = [&]() {
    tgpu_status cs{};
    uint64_t nd = 0, cons = 0;
    const int code = tgpu_decode_host_ex(ctx, schema, protocol, h_in, in_len, n, h_records,
                                         h_arena, arena_capacity, limits, &cs, &nd, &cons);
    if (on_chunk && cs.exc_class != TGPU_EXC_RUNTIME) {  // (runtime errors decode nothing)
      const uint64_t back = std::min<uint64_t>(n, nd + (code ? 1 : 0));
      if (back) on_chunk(user, 0, back);
    }
    if (st) *st = cs;
    if (n_decoded) *n_decoded = nd;
    if (consumed) *consumed = cons;
    return code;
  };
  // small batches (or no arena where one is needed): the resident pass
  if (n == 0 || in_len <= 2 * C || (scale && arena_capacity < scale * in_len)) return resident_all();
  void* vp = context_host_pipe(ctx);
  if (!vp) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  auto* p = (HostPipe*)vp;
  PinGuard pin_in(h_in, in_len), pin_rec(h_records, n * S), pin_ar(h_arena, arena_capacity);
  GrowBuf &din = p->din, &drec = p->drec, &dar = p->dar, &doffs = p->doffs;
  if (!din.reserve(in_len) || !drec.reserve(n * S) ||
      (arena_capacity && !dar.reserve(arena_capacity)) || !doffs.reserve((n + 1) * 8)) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  const uint64_t P = (in_len + C - 1) / C;
  const bool blocks = scale && arena_capacity && schema_block_rule(schema);
  // packed list elements (TGPU_HOST_PACK_LISTS; schemas whose arena holds
  // scalar list elements only): each chunk's element arrays at the front of
  // its arena slice, the records' spans pointing there; the chunk's packed
  // size is read back, then its records and packed bytes go back
  PackSpec ps{};
  if ((flags & TGPU_HOST_PACK_LISTS) && scale && arena_capacity)
    ps.n = packable_lists(schema, protocol, ps.member, ps.width, kPackMax);
  const bool pack = ps.n > 0;
  const uint64_t pnb = (n + 255) / 256 + 1;
  if (pack && (!p->dpk.reserve(arena_capacity) || !p->psum.reserve(pnb * 8) ||
               !p->ppart.reserve((scan_tiles_parts(pnb) + 1) * 8) || !p->ptot.reserve(P * 8))) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  std::vector<uint64_t> htot_v;
  uint64_t* htot = nullptr;
  if (pack) {
    if (hipHostMalloc((void**)&htot, P * 8, 0) != hipSuccess) {
      (void)hipGetLastError();
      htot_v.resize(P);
      htot = htot_v.data();
    }
  }
  struct HostFree {
    uint64_t* p;
    bool pinned;
    ~HostFree() {
      if (p && pinned) (void)hipHostFree(p);
    }
  } htot_guard{htot, pack && htot_v.empty()};
  Events evin(P), evdec(P), evout(P);
  const hipStream_t sin = p->s[0], sdec = p->s[1], sout = p->s[2];
  for (uint64_t k = 0; k < P; ++k) {
    const uint64_t b = k * C, e = std::min(in_len, b + C);
    if (hipMemcpyAsync(din.p + b, (const uint8_t*)h_in + b, e - b, hipMemcpyHostToDevice, sin) !=
            hipSuccess ||
        hipEventRecord(evin.ev[k], sin) != hipSuccess) {
      (void)hipStreamSynchronize(sin);
      set_status(st, TGPU_ERR_HIP, 0, 0);
      return TGPU_ERR_HIP;
    }
  }
  std::vector<Range> pending;
  uint64_t announced = 0;
  auto announce = [&](bool all) {
    size_t k = 0;
    for (; k < pending.size(); ++k) {
      if (!all && hipEventQuery(pending[k].done) != hipSuccess) break;
      if (all) (void)hipEventSynchronize(pending[k].done);
      if (on_chunk) on_chunk(user, pending[k].r0, pending[k].r1);
      announced = pending[k].r1;
    }
    pending.erase(pending.begin(), pending.begin() + k);
  };
  // a decoded chunk's records and arena bytes (from `abuf`, `abytes` at
  // scale * B) back to the host on sout, announced once they land
  auto send_back = [&](uint64_t kk, uint64_t rr, uint64_t nk, uint64_t bb, uint64_t abytes,
                       const uint8_t* abuf) {
    if (hipStreamWaitEvent(sout, evdec.ev[kk], 0) != hipSuccess ||
        hipMemcpyAsync((uint8_t*)h_records + rr * S, drec.p + rr * S, nk * S,
                       hipMemcpyDeviceToHost, sout) != hipSuccess ||
        (scale && abytes &&
         hipMemcpyAsync((uint8_t*)h_arena + scale * bb, abuf + scale * bb, abytes,
                        hipMemcpyDeviceToHost, sout) != hipSuccess) ||
        hipEventRecord(evout.ev[kk], sout) != hipSuccess)
      return false;
    pending.push_back(Range{rr, rr + nk, evout.ev[kk]});
    return true;
  };
  struct Staged {
    uint64_t k, r0, nk, B;
  };
  std::vector<Staged> staged;  // packed chunks whose size is not read yet
  auto flush_pending = [&]() {
    while (!staged.empty()) {
      const Staged c = staged.front();
      if (hipEventSynchronize(evdec.ev[c.k]) != hipSuccess ||
          !send_back(c.k, c.r0, c.nk, c.B, htot[c.k], p->dpk.p))
        return false;
      staged.erase(staged.begin());
    }
    return true;
  };
  uint64_t B = 0, r0 = 0, k = 0;
  bool clean = true;
  while (r0 < n && B < in_len) {
    const uint64_t end = std::min(in_len, (k + 1) * C);
    if (end <= B) {
      ++k;
      continue;
    }
    const uint64_t ap = std::min(k + 1, P - 1);  // the next piece must be resident too
    const uint64_t avail = std::min(in_len, (ap + 1) * C);
    tgpu_status cs{};
    uint64_t nk = 0, first = 0, last = 0;
    if (hipStreamWaitEvent(sdec, evin.ev[ap], 0) != hipSuccess) {
      clean = false;  // (the resident pass below reports the HIP failure)
      break;
    }
    const int rc = tgpu_decode_stream(p->c[1], schema, protocol, din.p, avail, B, end, 0,
                                      (uint64_t*)doffs.p + r0, n - r0, drec.p + r0 * S,
                                      arena_capacity ? dar.p : nullptr, arena_capacity, limits,
                                      sdec, &cs, &nk, &first, &last);
    if (rc != TGPU_OK || first != B || last < B || (nk == 0 && end < in_len)) {
      clean = false;  // a record the range cannot end cleanly on: the resident pass
      break;
    }
    if (blocks && end < in_len && r0 + nk < n && nk % kArenaBlock) {
      // the block rule: a piece hands back whole blocks of kArenaBlock
      // records (its blocks are then the resident pass's, and a fallback's
      // arena slice starts at a block), the next piece starts at the first
      // record it did not keep; a range of fewer than one block (records of
      // over piece / 256 bytes) is decoded again with the next piece added
      if (nk < kArenaBlock) {
        ++k;
        continue;
      }
      nk -= nk % kArenaBlock;
      if (hipMemcpy(&last, (uint64_t*)doffs.p + r0 + nk, 8, hipMemcpyDeviceToHost) != hipSuccess) {
        clean = false;
        break;
      }
    }
    if (nk) {
      if (pack) {
        // pack the chunk's element arrays (sdec), its packed size to htot[k]
        const uint64_t nb = (nk + 255) / 256;
        auto* sums = (unsigned long long*)p->psum.p;
        hipLaunchKernelGGL(pack_size_kernel, dim3((uint32_t)nb), dim3(256), 0, sdec,
                           drec.p + r0 * S, nk, S, ps, sums);
        hipError_t pe = hipGetLastError();
        if (pe == hipSuccess)
          pe = launch_scan_tiles(sums, nb, (unsigned long long*)p->ppart.p,
                                 (unsigned long long*)p->ptot.p + k, nullptr, sdec);
        if (pe == hipSuccess) {
          hipLaunchKernelGGL(pack_copy_kernel, dim3((uint32_t)nb), dim3(256), 0, sdec,
                             drec.p + r0 * S, nk, S, ps, sums, dar.p, p->dpk.p, scale * B);
          pe = hipGetLastError();
        }
        if (pe == hipSuccess)
          pe = hipMemcpyAsync(htot + k, (uint64_t*)p->ptot.p + k, 8, hipMemcpyDeviceToHost, sdec);
        if (pe != hipSuccess || hipEventRecord(evdec.ev[k], sdec) != hipSuccess) {
          clean = false;
          break;
        }
        // (tgpu_decode_stream above is a blocking call, so the chunk's
        // kernels are all but done: its packed size is read at once and its
        // copy back starts behind the pack)
        staged.push_back(Staged{k, r0, nk, B});
        if (!flush_pending()) {
          clean = false;
          break;
        }
      } else if (hipEventRecord(evdec.ev[k], sdec) != hipSuccess ||
                 !send_back(k, r0, nk, B, std::min(arena_capacity, scale * last) - scale * B,
                            dar.p)) {
        clean = false;
        break;
      }
    }
    announce(false);
    B = last;
    r0 += nk;
    ++k;
  }
  if (clean && !flush_pending()) clean = false;
  // the wire position of the first record not sent back (a chunk still
  // staged for packing, or the loop's end)
  const uint64_t Bsent = staged.empty() ? B : staged.front().B;
  (void)hipStreamSynchronize(sin);
  (void)hipStreamSynchronize(sdec);
  announce(true);
  if (clean && r0 == n) {
    set_status(st, TGPU_OK, n, 0);
    if (n_decoded) *n_decoded = n;
    if (consumed) *consumed = B;
    return TGPU_OK;
  }
  // a range that did not end cleanly (or the stream ended before n records):
  // the whole batch resident on the device, exact status; the records from
  // the first one not yet handed over come back
  tgpu_status cs{};
  uint64_t nd = 0, cons = 0;
  int code = tgpu_decode_batch(p->c[1], schema, protocol, din.p, in_len, nullptr, n, drec.p,
                               arena_capacity ? dar.p : nullptr, arena_capacity, limits, sdec,
                               &cs, &nd, &cons);
  if (code != TGPU_ERR_HIP) {
    const uint64_t back = std::min<uint64_t>(n, nd + (code ? 1 : 0));
    // arena bytes of the records from `announced` on: they start at the
    // wire position of record `announced`, which is Bsent (every announced
    // range ended cleanly at the next one's start)
    const uint64_t a0 = std::min(arena_capacity, scale * Bsent);
    if (code != TGPU_ERR_HIP && back > announced &&
        (hipMemcpy((uint8_t*)h_records + announced * S, drec.p + announced * S,
                   (back - announced) * S, hipMemcpyDeviceToHost) != hipSuccess ||
         (scale && hipMemcpy((uint8_t*)h_arena + a0, dar.p + a0, arena_capacity - a0,
                             hipMemcpyDeviceToHost) != hipSuccess)))
      code = TGPU_ERR_HIP;
    if (code != TGPU_ERR_HIP && on_chunk && back > announced && cs.exc_class != TGPU_EXC_RUNTIME)
      on_chunk(user, announced, back);
  }
  if (code == TGPU_ERR_HIP) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  if (st) *st = cs;
  if (n_decoded) *n_decoded = nd;
  if (consumed) *consumed = cons;
  return code;
}

int tgpu_encode_host_chunks(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                            uint64_t n, uint64_t chunk_records, tgpu_fill_fn fill,
                            tgpu_reserve_fn reserve, void* user, tgpu_status* st,
                            uint64_t* out_size) {
  return tgpu_encode_host_chunks_ex(ctx, schema, protocol, n, chunk_records, fill, reserve,
                                    nullptr, user, st, out_size);
}

int tgpu_encode_host_chunks_ex(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                               uint64_t n, uint64_t chunk_records, tgpu_fill_fn fill,
                               tgpu_reserve_fn reserve, tgpu_landed_fn landed, void* user,
                               tgpu_status* st, uint64_t* out_size) {
  if (out_size) *out_size = 0;
  if (!ctx || !schema || !fill || !reserve) {
    set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  if (n == 0) {
    set_status(st, TGPU_OK, 0, 0);
    return TGPU_OK;
  }
  void* vp = context_host_pipe(ctx);
  if (!vp) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  auto* p = (HostPipe*)vp;
  const uint64_t K = chunk_records ? chunk_records : kDefaultChunkRecords;
  const uint64_t nch = (n + K - 1) / K;
  const uint32_t S = tgpu_schema_record_size(schema);
  const hipStream_t sin = p->s[0], senc = p->s[1], sout = p->s[2];
  // two slots: chunk k's device form and output in slot k % 2
  // (device buffers: the pipe's, kept across calls)
  struct Slot {
    GrowBuf *rec, *str, *lst, *out;
    hipEvent_t in_done = nullptr, out_done = nullptr;
    uint64_t m = 0;
  } slot[2] = {{&p->erec[0], &p->estr[0], &p->elst[0], &p->eout[0]},
               {&p->erec[1], &p->estr[1], &p->elst[1], &p->eout[1]}};
  for (auto& sl : slot) {
    (void)hipEventCreateWithFlags(&sl.in_done, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&sl.out_done, hipEventDisableTiming);
  }
  struct EvFree {
    Slot* s;
    ~EvFree() {
      for (int i = 0; i < 2; ++i) {
        (void)hipEventDestroy(s[i].in_done);
        (void)hipEventDestroy(s[i].out_done);
      }
    }
  } evfree{slot};
  // upload chunk c's form into its slot (after the slot's previous output left)
  auto upload = [&](uint64_t c) -> int {
    Slot& sl = slot[c % 2];
    const uint64_t r0 = c * K, m = std::min(K, n - r0);
    tgpu_host_form f{};
    if (fill(user, r0, r0 + m, &f) != 0 || !f.records) return TGPU_ERR_INVALID_ARGUMENT;
    // (the slot's previous chunk has been encoded: its inputs are free)
    if (!sl.rec->reserve(m * S) || !sl.str->reserve(f.strings_len + 16) ||
        !sl.lst->reserve(f.lists_len + 16))
      return TGPU_ERR_HIP;
    if (hipMemcpyAsync(sl.rec->p, f.records, m * S, hipMemcpyHostToDevice, sin) != hipSuccess ||
        (f.strings_len && hipMemcpyAsync(sl.str->p, f.strings, f.strings_len,
                                         hipMemcpyHostToDevice, sin) != hipSuccess) ||
        (f.lists_len && hipMemcpyAsync(sl.lst->p, f.lists, f.lists_len, hipMemcpyHostToDevice,
                                       sin) != hipSuccess) ||
        hipEventRecord(sl.in_done, sin) != hipSuccess)
      return TGPU_ERR_HIP;
    sl.m = m;
    return TGPU_OK;
  };
  // encode chunk c (async); the output buffer grows to the chunk's size on
  // an overflow, found by the blocking size pass
  auto encode = [&](uint64_t c) -> int {
    Slot& sl = slot[c % 2];
    const uint64_t want = std::max<uint64_t>(16ull << 20, sl.m * 64);
    // (growing the wire buffer waits for its previous chunk's copy out)
    if (want > sl.out->cap &&
        (hipEventSynchronize(sl.out_done) != hipSuccess || !sl.out->reserve(want)))
      return TGPU_ERR_HIP;
    if (hipStreamWaitEvent(senc, sl.in_done, 0) != hipSuccess ||
        hipStreamWaitEvent(senc, sl.out_done, 0) != hipSuccess)
      return TGPU_ERR_HIP;
    return tgpu_encode_batch(p->c[c % 2], schema, protocol, sl.rec->p, sl.m, sl.str->p, sl.lst->p,
                             sl.out->p, sl.out->cap, nullptr, senc, nullptr, nullptr);
  };
  // chunks whose wire is on its way to the caller's memory, in order; the
  // slot's out_done event is re-recorded two chunks later, so at most the
  // previous chunk is still pending when a chunk's copy is issued
  struct Landing {
    uint64_t r0, r1;
    void* dst;
    uint64_t bytes;
    hipEvent_t done;
  };
  std::vector<Landing> landing;
  auto land = [&](bool all, uint64_t keep) {
    size_t k = 0;
    for (; k < landing.size() && landing.size() - k > keep; ++k) {
      Landing& l = landing[k];
      if (all || hipEventQuery(l.done) != hipSuccess) (void)hipEventSynchronize(l.done);
      if (landed) landed(user, l.r0, l.r1, l.dst, l.bytes);
    }
    landing.erase(landing.begin(), landing.begin() + k);
  };
  uint64_t total = 0;
  int rc = upload(0);
  if (rc == TGPU_OK) rc = encode(0);
  for (uint64_t c = 0; c < nch && rc == TGPU_OK; ++c) {
    Slot& sl = slot[c % 2];
    if (c + 1 < nch) rc = upload(c + 1);  // the host builds chunk c+1 while c encodes
    if (rc) break;
    tgpu_status cs{};
    uint64_t done = 0, bytes = 0;
    int code = tgpu_context_wait(p->c[c % 2], senc, &cs, &done, &bytes);
    if (code == TGPU_ERR_OUTPUT_OVERFLOW) {
      // the slot's output was too small for this chunk: size it exactly
      uint64_t need = 0;
      tgpu_status ss{};
      DevBuf offs;
      if (!offs.alloc((sl.m + 1) * 8)) {
        rc = TGPU_ERR_HIP;
        break;
      }
      code = tgpu_encoded_size(p->c[c % 2], schema, protocol, sl.rec->p, sl.m, sl.lst->p,
                               (uint64_t*)offs.p, senc, &ss, &need);
      if (code == TGPU_OK) {
        if (hipEventSynchronize(sl.out_done) != hipSuccess || !sl.out->reserve(need + 16)) {
          rc = TGPU_ERR_HIP;
          break;
        }
        code = tgpu_encode_batch(p->c[c % 2], schema, protocol, sl.rec->p, sl.m, sl.str->p,
                                 sl.lst->p, sl.out->p, sl.out->cap, nullptr, senc, &cs, &bytes);
      } else {
        cs = ss;
        bytes = 0;
      }
    }
    if (code == TGPU_ERR_HIP) {
      rc = TGPU_ERR_HIP;
      break;
    }
    // the chunk's wire (or, on an error, the records before it) goes out
    if (bytes) {
      land(false, 1);  // (the slot's event is re-recorded below)
      void* dst = reserve(user, bytes);
      if (!dst || hipMemcpyAsync(dst, sl.out->p, bytes, hipMemcpyDeviceToHost, sout) != hipSuccess ||
          hipEventRecord(sl.out_done, sout) != hipSuccess) {
        rc = dst ? TGPU_ERR_HIP : TGPU_ERR_OUTPUT_OVERFLOW;
        if (!dst) set_status(st, TGPU_ERR_OUTPUT_OVERFLOW, c * K, total);
        break;
      }
      landing.push_back(Landing{c * K, c * K + (code == TGPU_OK ? sl.m : cs.record), dst, bytes,
                                sl.out_done});
      total += bytes;
    }
    if (code != TGPU_OK) {
      (void)hipStreamSynchronize(sout);
      land(true, 0);
      if (st) {
        *st = cs;
        st->record = c * K + cs.record;
        st->byte_offset = total - bytes + cs.byte_offset;
      }
      if (out_size) *out_size = total;
      (void)hipStreamSynchronize(sin);
      return code;
    }
    if (c + 1 < nch) rc = encode(c + 1);
  }
  (void)hipStreamSynchronize(sin);
  (void)hipStreamSynchronize(senc);
  (void)hipStreamSynchronize(sout);
  land(true, 0);
  if (rc) {
    if (rc != TGPU_ERR_OUTPUT_OVERFLOW) set_status(st, rc, 0, 0);
    if (out_size) *out_size = total;
    return rc;
  }
  set_status(st, TGPU_OK, n, 0);
  if (out_size) *out_size = total;
  return TGPU_OK;
}

int tgpu_host_alloc(uint64_t bytes, void** out) {
  if (!out) return TGPU_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  if (hipHostMalloc(out, std::max<uint64_t>(bytes, 16), hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return TGPU_ERR_HIP;
  }
  return TGPU_OK;
}

void tgpu_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int tgpu_encoded_size_host(tgpu_context* ctx, const tgpu_schema* schema, int protocol,
                           const void* h_records, uint64_t n, const void* h_lists,
                           uint64_t lists_len, uint64_t* h_out_offsets, tgpu_status* st,
                           uint64_t* total) {
  if (total) *total = 0;
  if (!ctx || !schema || (n && !h_records) || (lists_len && !h_lists)) {
    set_status(st, TGPU_ERR_INVALID_ARGUMENT, 0, 0);
    return TGPU_ERR_INVALID_ARGUMENT;
  }
  const uint32_t S = tgpu_schema_record_size(schema);
  PinGuard pin_rec(h_records, n * S), pin_l(h_lists, lists_len);
  DevBuf drec, dlist, doffs;
  if (!drec.alloc(n * S) || !dlist.alloc(lists_len) || !doffs.alloc((n + 1) * 8)) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  if ((n && hipMemcpy(drec.p, h_records, n * S, hipMemcpyHostToDevice) != hipSuccess) ||
      (lists_len && hipMemcpy(dlist.p, h_lists, lists_len, hipMemcpyHostToDevice) != hipSuccess)) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  tgpu_status cs{};
  uint64_t size = 0;
  int code = tgpu_encoded_size(ctx, schema, protocol, drec.p, n, lists_len ? dlist.p : nullptr,
                               (uint64_t*)doffs.p, nullptr, &cs, &size);
  if (code == TGPU_OK && h_out_offsets &&
      hipMemcpy(h_out_offsets, doffs.p, (n + 1) * 8, hipMemcpyDeviceToHost) != hipSuccess)
    code = TGPU_ERR_HIP;
  if (code == TGPU_ERR_HIP) {
    set_status(st, TGPU_ERR_HIP, 0, 0);
    return TGPU_ERR_HIP;
  }
  if (st) *st = cs;
  if (total) *total = size;
  return code;
}

}  // extern "C"
