// k_skim.hip — schemaless skim of an indexed stream (tgpu_skim_batch).
//
// One lane per record walks its top-level fields exactly like the parse loop
// of protocol::parseObject (thrift/lib/cpp2/protocol/detail/Object.h:416-432):
// readFieldBegin until STOP; a bool is read (FieldMaskUtil.h:441-450), any
// other value is passed over by the protocol's skip and kept as (offset,
// length) of its encoded bytes, the masked parse's setMaskedDataFull
// (FieldMaskUtil.h:373-388). The reader, skip and limits are the decoder's
// (tgpu_device.h), so depth / size / varint / bool errors are the ones the
// decoder reports for the same bytes. The first failing record in record
// order is re-diagnosed by one lane and published like a decode result.
#include "tgpu_device.h"

namespace tgpu {
namespace {

using namespace dev;

__device__ __forceinline__ Reader skim_reader(const SkimArgs& a, uint64_t start) {
  Reader r;
  r.p = a.in;
  r.pos = start;
  r.end = a.in_len;
  r.height = (int64_t)(a.height ? a.height : a.max_depth) + 1;
  r.string_limit = a.string_limit;
  r.container_limit = a.container_limit;
  r.max_depth = a.max_depth;
  r.err = 0;
  r.err_off = 0;
  r.has_bool = false;
  r.bool_val = false;
  return r;
}

// Skims record i into its field slots; returns the reader (error latched).
template <int P>
__device__ Reader skim_one(const SkimArgs& a, uint64_t i, bool store) {
  using Pr = Proto<P>;
  const uint64_t start = a.offs[i];
  Reader r = skim_reader(a, start);
  if (start > a.in_len || a.offs[i + 1] < start) {
    r.fail(TGPU_ERR_INDEX_MISMATCH, start);
    return r;
  }
  tgpu_skim_field* out = a.fields + i * (uint64_t)a.max_fields;
  uint32_t count = 0;
  int32_t prev = 0;
  while (r.ok()) {
    uint32_t wt = 0;
    int32_t id = 0;
    if (!Pr::field_header(r, prev, wt, id)) break;  // STOP or error
    prev = id;
    const uint64_t off = r.pos;
    uint32_t flags = 0;
    if (wt == TGPU_T_BOOL) flags = TGPU_SKIM_BOOL | (Pr::read_bool(r) ? TGPU_SKIM_TRUE : 0);
    else skip<P>(r, wt, 0);
    if (!r.ok()) break;
    if (store && count < a.max_fields) {
      tgpu_skim_field f;
      f.id = (int16_t)id;
      f.ttype = (uint8_t)wt;
      f.flags = (uint8_t)flags;
      f.length = (uint32_t)(r.pos - off);
      f.offset = off;
      out[count] = f;
    }
    ++count;
  }
  if (store) a.counts[i] = count;
  if (r.ok() && r.pos != a.offs[i + 1]) r.fail(TGPU_ERR_INDEX_MISMATCH, r.pos);
  return r;
}

template <int P>
__global__ __launch_bounds__(256) void skim_kernel(SkimArgs a) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    const Reader r = skim_one<P>(a, i, true);
    if (!r.ok()) atomicMin(&a.res->first_fail, (unsigned long long)i);
  }
}

template <int P>
__global__ void skim_finish_kernel(SkimArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DevResult* res = a.res;
  const uint64_t f = res->first_fail;
  if (f < a.n) {
    const Reader r = skim_one<P>(a, f, false);
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

uint32_t skim_grid(uint64_t n) {
  const uint64_t b = (n + 255) / 256;
  return (uint32_t)(b < 8192 ? (b ? b : 1) : 8192);
}

}  // namespace

hipError_t launch_skim(const SkimArgs& a, int protocol, hipStream_t stream) {
  if (a.n)
    TGPU_BY_PROTOCOL(protocol, hipLaunchKernelGGL(skim_kernel<P_>, dim3(skim_grid(a.n)), dim3(256),
                                                  0, stream, a));
  TGPU_BY_PROTOCOL(protocol,
                   hipLaunchKernelGGL(skim_finish_kernel<P_>, dim3(1), dim3(64), 0, stream, a));
  return hipGetLastError();
}

}  // namespace tgpu
