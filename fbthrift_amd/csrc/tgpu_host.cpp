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

#include "tgpu_internal.h"

namespace {

constexpr int kSlots = 3;
constexpr uint64_t kDefaultChunk = 1ull << 22;  // records per chunk

struct HostPipe {
  int device = 0;
  hipStream_t s[kSlots] = {};
  tgpu_context* c[kSlots] = {};
  uint8_t* d_in[kSlots] = {};
  uint8_t* d_out[kSlots] = {};
  uint64_t in_cap = 0, out_cap = 0;
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
