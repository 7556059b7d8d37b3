// tgpu_internal.h — definitions shared by the C-ABI host code and the gfx950
// kernels of the bulk Thrift record codec. Not part of the public ABI.
#pragma once

#ifdef __HIPCC_RTC__
// Runtime-compiled schema kernels (tgpu_jit.cpp): hipRTC has no libc headers,
// so the fixed-width types are declared here with the host's LP64 widths.
typedef signed char int8_t;
typedef short int16_t;
typedef int int32_t;
typedef long int64_t;
typedef unsigned char uint8_t;
typedef unsigned short uint16_t;
typedef unsigned int uint32_t;
typedef unsigned long uint64_t;
typedef unsigned long uintptr_t;
#include "thrift_gpu.h"
#else
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/thrift_gpu.h"
#endif

// Runs `stmt` with the protocol as the constant P_ (a kernel template
// argument): Binary, Compact, or CompactV1.
#define TGPU_BY_PROTOCOL(proto, ...)                                    \
  do {                                                                  \
    if ((proto) == TGPU_PROTOCOL_BINARY) {                              \
      constexpr int P_ = TGPU_PROTOCOL_BINARY;                          \
      __VA_ARGS__;                                                      \
    } else if ((proto) == TGPU_PROTOCOL_COMPACT_V1) {                   \
      constexpr int P_ = TGPU_PROTOCOL_COMPACT_V1;                      \
      __VA_ARGS__;                                                      \
    } else {                                                            \
      constexpr int P_ = TGPU_PROTOCOL_COMPACT;                         \
      __VA_ARGS__;                                                      \
    }                                                                   \
  } while (0)

namespace tgpu {

// Records per workgroup tile in the fixed-layout Binary kernels. 256 records x
// any wire length L is a multiple of 16 bytes, so every tile starts on the
// same 16-byte phase as the stream base.
constexpr int kTileRecords = 256;
constexpr int kBlock = 256;
// Upper bound on the canonical wire length handled by the fixed-layout
// kernels (LDS: 256 x (L + S) bytes must fit beside a second block).
constexpr uint32_t kMaxFixedWire = 192;
constexpr uint32_t kMaxFixedRecord = 160;
constexpr int kMaxTemplateItems = 96;
// Record frames (struct / container levels) the general reader and writer
// keep per lane privately. A record nested deeper is not an error: the lane
// reports kErrDeep and the record is redone by a deep pass whose lanes keep
// their frames in HBM (DeepArgs), so records nest as deep as the data does
// (recursive schemas) up to the slab's frames.
constexpr int kPrivFrames = 8;
// HBM slab of one deep-pass lane: slab_frames skip frames (12 bytes each,
// rounded up to 16 bytes in all), then slab_frames record frames of at most
// kRecordFrameBytes (dev::ReadFrame / dev::WriteFrame).
constexpr uint64_t kSkipFrameBytes = 12;
constexpr uint64_t kRecordFrameBytes = 80;
constexpr uint64_t slab_skip_bytes(uint64_t frames) {
  return (frames * kSkipFrameBytes + 15) & ~15ull;
}
constexpr uint64_t slab_lane_bytes(uint64_t frames) {
  return slab_skip_bytes(frames) + frames * kRecordFrameBytes;
}
// Skip frames a lane keeps privately. A value nested deeper is not an error:
// the lane reports kErrDeep and its record (or index chunk) is redone by a
// deep pass whose lanes keep max_depth frames in HBM (DeepArgs), so the skip
// follows FLAGS_thrift_protocol_max_depth (Protocol.cpp:21-29) like the
// reference's recursive skip (BinaryProtocol.cpp:140-143).
constexpr int kMaxSkipDepth = 16;
constexpr int32_t kErrDeep = 0x10000;  // internal; never reaches a tgpu_status
// Frames of one deep-pass lane are capped (the reference's recursion would
// exhaust a thread stack long before): deeper -> TGPU_ERR_UNSUPPORTED.
constexpr uint64_t kMaxDeepFrames = 1ull << 22;
// The general kernels' deep passes (decode, size, write) have two tiers for
// a recursive schema when max_depth allows more than kWideFrames: the wide
// tier (up to kWideLanes lanes of kWideFrames frames, 256 MiB — a recursive
// schema's records mostly nest up to a few hundred frames: a boxed chain
// node takes 2) reads the deferred records first, and hands the ones
// nesting deeper still to list2, which the max_depth slabs' lanes (at most
// 256) read. With one tier a tree stream's deep records queued on ~60
// lanes (10 s for 1 Mi golden trees, tools/recursive_bench.py).
constexpr uint64_t kWideFrames = 256;
constexpr uint32_t kWideLanes = 16384;
struct DeepArgs {
  uint64_t* list;               // deferred records (or index chunks)
  unsigned long long* count;    // entries in list
  uint8_t* slabs;               // lanes x slab_lane_bytes(slab_frames)
  uint64_t slab_frames;
  uint32_t lanes;
  uint32_t more;                // these slabs are the wide tier's (deep_decode_kernel)
  uint8_t* wslabs;              // the wide tier: wlanes x slab_lane_bytes(kWideFrames)
  uint32_t wlanes;              // (0: one tier)
  uint32_t pad;
  uint64_t* list2;              // the wide tier's leftovers (count2 entries)
  unsigned long long* count2;
};
// arena == nullptr with this capacity: list elements are read and validated
// but not stored (the stream indexer measures records without output).
constexpr uint64_t kDiscardArena = ~0ull;
// Starts of a speculated chain kept for the repair pass (stream indexer).
constexpr int kSpecStarts = 8;

// One step of the canonical Binary wire template of a fixed-layout schema
// (every field unqualified, fixed width; nested structs flattened). The item
// covers `hdr_len` constant bytes (field header / STOP / nested header)
// followed by `width` value bytes (big-endian on the wire).
struct TemplateItem {
  uint16_t wire_off;  // offset of the first byte of the item in the record
  uint8_t hdr_len;    // 0..4 constant bytes
  uint8_t width;      // 0,1,2,4,8 value bytes
  uint32_t hdr;       // constant bytes, little-endian packed (byte 0 first)
  uint16_t member_off;
  uint8_t is_bool;    // value must be 0/1 (Binary readBool / validate_bool)
  uint8_t pad;
};

struct FixedTemplate {
  uint32_t wire_len;     // L
  uint32_t record_size;  // S
  uint32_t n_items;
  uint32_t n_isset;      // isset bytes set to 1 (all of them; unqualified)
  uint16_t isset_off[64];
  TemplateItem items[kMaxTemplateItems];
};

// The same template regrouped by output 8-byte word of the record layout
// (records with S % 8 == 0): word j = const_bits (isset bytes, zero padding)
// OR the values of items[first .. first+n) placed at byte `dst`. Items with
// width 0 (STOP, nested struct headers) ride on the last word; each item is
// owned by exactly one word, so every header byte is checked exactly once.
constexpr int kMaxPlanWords = 20;  // S <= 160
struct PlanItem {
  uint16_t wire_off;
  uint8_t hdr_len;
  uint8_t width;
  uint32_t hdr;
  uint8_t dst;  // byte offset of the value inside its 8-byte word
  uint8_t is_bool;
  uint8_t pad[2];
};
struct PlanWord {
  unsigned long long const_bits;
  uint16_t first_item;
  uint8_t n_items;
  uint8_t has_value;  // at least one item with width > 0 (encode must load it)
  uint8_t pad[4];
};
struct FixedPlan {
  uint32_t wire_len;   // L
  uint32_t n_words;    // Q = S / 8
  uint32_t n_items;
  uint32_t pad;
  PlanWord words[kMaxPlanWords];
  PlanItem items[kMaxTemplateItems];
};

// ---- compiled record programs (variable-length canonical fast path) -------
// A schema whose fields are all unqualified compiles to a straight-line
// program describing the canonical wire form of one record: the header bytes
// the generated readNoXfer expects at each step (advanceToNextField's fast
// path, BinaryProtocol-inl.h:586-621 / CompactProtocol-inl.h:811-872) and the
// value encoding that follows. Nested structs are flattened; members are at
// absolute offsets of the root record.
enum VOpKind : uint8_t {
  VOP_CONST = 1,   // hdr_len constant bytes (field header, STOP, nested header)
  VOP_FIXED = 2,   // width big-endian bytes -> member (Binary ints, doubles, floats, bytes)
  VOP_VARINT = 3,  // zigzag varint (bits 32/64) -> member of `width` bytes (Compact ints)
  VOP_STRING = 4,  // length (Binary BE i32 / Compact varint) + bytes -> tgpu_span view
  VOP_LIST = 5,    // list header + scalar elements -> arena, tgpu_span
  VOP_CBOOL = 6,   // Compact bool field: value carried in the header byte
  VOP_ISSET = 7,   // set an isset byte (after a nested struct's STOP)
  // nested programs only (build_nested_program): a list / set whose elements
  // are structs or scalar lists. Header + count, the element array from the
  // record's arena region, then the body ops (up to index hdr_len, the
  // matching VOP_SEQ_END) once per element with members relative to the
  // element slot of hdr bytes; elem_ttype / elem_ct: the wire element type.
  VOP_SEQ = 8,
  VOP_SEQ_END = 9,
  // a map whose pairs are {key (width: its ttype, bits: its slot bytes),
  // value (elem_ttype)}: header (elem_ct = Compact key/value ctypes), hdr-byte
  // pairs from the region, the body (key op at 0, the value's ops at bits)
  // once per pair, ended by VOP_SEQ_END like VOP_SEQ
  VOP_MSEQ = 10,
  // nested programs: a field header (member: the field id; hdr: its Binary
  // header; elem_ct: its Compact ctype; is_bool: a bool field; width 1: an
  // optional field, present when its header is next; isset: its isset
  // byte; bits: the value ops that follow; elem_kind 1: a terse field, read
  // like an optional one, written unless empty). Compact headers are deltas from
  // the struct's last field (VOP_SBEGIN's scope), so they are computed, not
  // constant, once fields may be absent.
  VOP_FHDR = 11,
  VOP_SBEGIN = 12,  // a struct's fields begin (hdr_len: one past its VOP_SEND;
                    // width 1: a union — one member at most, its FHDRs optional)
  VOP_SEND = 13,    // its STOP
  // a boxed struct field (cpp.ref / thrift.box): the object (hdr bytes) from
  // the record's region, read / written by the body ops (members relative to
  // it) up to its VOP_BOX_END (hdr_len: one past it); member: the field's span
  VOP_BOX = 14,
  VOP_BOX_END = 15,
  // a recursive schema's struct past the levels its nested program unrolls
  // (build_nested_program): the record is handed to the general kernels
  // when its value is read; such a program has no writer (nprog_defer)
  VOP_DEFER = 16,
};
enum VElemKind : uint8_t {
  VEL_FIXED = 1,   // big-endian fixed width (Binary ints, doubles/floats, bytes)
  VEL_VARINT = 2,  // zigzag varint (Compact i16/i32/i64)
  VEL_BOOL = 3,    // Binary: byte must be 0/1; Compact: value = (byte == 1)
  VEL_STRING = 4,  // nested programs: a string -> tgpu_span element (a view into the stream)
};
struct VOp {
  uint8_t kind;
  uint8_t hdr_len;   // CONST / CBOOL header length
  uint8_t width;     // FIXED / VARINT store width; LIST element store width
  uint8_t bits;      // VARINT / list varint element: 32 or 64
  uint32_t hdr;      // CONST / CBOOL bytes (CBOOL: low nibble of byte 0 is the value)
  uint16_t member;   // absolute member offset
  uint16_t isset;    // absolute isset offset to set after the op (0xffff: none)
  uint8_t elem_kind;  // LIST
  uint8_t elem_ttype; // LIST: TType of the elements (wire element type)
  uint8_t elem_ct;    // LIST: Compact element ctype
  uint8_t is_bool;    // FIXED: a bool (Binary: byte must be 0/1; Compact, a
                      // container element / key / value: byte == 1)
};
// CONST op flag (elem_kind): the root record's STOP, before which fields with
// ids above the schema's (member = the root's largest id; hdr bits 8..23 =
// the last root field's id, Compact's delta base) are skipped when they are
// scalars or strings — a newer writer's appended fields
// (deserialize_struct.whisker: unknown ids go to skip).
constexpr uint8_t kStopSkipsUnknown = 1;
// FIXED op / LIST op with VEL_FIXED elements (`bits`, otherwise unused
// there): the value is little-endian on the wire — CompactV1's doubles
// (CompactV1Protocol-inl.h:44-53,84: writeLE / readLE). A CompactV1
// program is Compact's (protocol COMPACT) with these ops; it lives in
// program slot kV1Slot.
constexpr uint8_t kFixedLE = 1;
constexpr int kV1Slot = 1;
constexpr int kMaxProgramOps = 128;  // flat record programs
// nested programs (op indices and value-op counts are bytes: at most 255)
constexpr int kMaxNestedOps = 255;
struct VProgram {
  uint32_t n_ops;
  uint32_t rec_size;
  uint32_t protocol;
  uint32_t has_list;
  VOp ops[kMaxNestedOps];
};

// Block rule (round 6; thrift_gpu.h tgpu_schema_arena_scale): the list / set
// element arrays of a flat-list schema (containers: lists / sets of scalars
// only, at most kPackSlots counting by-value struct members, nothing nested
// or boxed) are packed per block of kArenaBlock records: records in order, a
// record's arrays in wire order, each 8-byte aligned, from align8(scale x the
// wire start of the block's first record). Decoders write the position rule
// (scale x an array's wire position) and arena_pack_kernel (k_arena.hip)
// moves the blocks a fast path has not packed already (DecodeArgs pack_flags:
// the compiled Binary decode tile packs each wave's block and marks it).
constexpr uint32_t kArenaBlock = 64;  // (one wave's records in the decode tile)
constexpr uint32_t kPackSlots = 8;
struct ArenaPack {
  uint32_t n;      // slots (0: the schema keeps the position rule)
  uint32_t scale;  // arena bytes per wire byte (1 Binary, 8 Compact)
  uint32_t member[kPackSlots];  // span offset in the record
  uint32_t es[kPackSlots];      // element bytes
};

// Device-side result slot of a context (one per in-flight call).
struct DevResult {
  unsigned long long first_fail;       // first failing record (UINT64_MAX: none)
  unsigned long long first_irregular;  // fixed path: first non-canonical record
  int32_t code;                        // diagnosed code of first_fail
  int32_t pad;
  unsigned long long fail_offset;      // diagnosed byte offset
  unsigned long long total_bytes;      // encode: output size; decode: consumed
  unsigned long long n_records;
  unsigned long long n_irregular;      // program path: records sent to the general decoder
  unsigned long long first_start;      // stream index: first record start found
  unsigned long long n_deep;           // records deferred to the deep pass
  unsigned long long n_deep2;          // of those, left by its wide tier
  unsigned long long n_deep_chunks;    // index chunks deferred to the deep emit pass
  unsigned long long first_misfit;     // fixed path: first exception not L bytes long
  // Stream-ordered fixed path, from the first misfit m on (tail_stride 0: none):
  // record i >= m at tail_pos + (i - m) * tail_stride (record m's length);
  // tail_min: the first record the strided tail decode did not take.
  unsigned long long tail_first, tail_pos, tail_stride, tail_min;
};

struct DevSchema {
  const tgpu_struct_desc* s;
  const tgpu_field_desc* f;
  const tgpu_type_desc* t;  // nested container types (type_index k -> t[k - 1])
  uint32_t ns, nf;
  uint32_t str_elems;   // some list/set/map holds strings: arena scale 4 / 16
  uint32_t bump_scale;  // nested schema: record regions of this scale (0: position rule)
  uint32_t nest_slot;   // nested schema, measuring reads: element slot bytes per level
  uint32_t nt;          // type-table nodes
};

struct DecodeArgs {
  DevSchema sc;
  const uint8_t* in;
  uint64_t in_len;
  const uint64_t* offs;  // n+1 record starts (given or computed)
  uint64_t n;
  uint8_t* recs;
  uint8_t* arena;
  uint64_t arena_cap;
  int32_t string_limit, container_limit, max_depth, height;
  uint32_t rec_size;
  int check_index;  // offsets were supplied by the caller: verify lengths
  DevResult* res;
  uint64_t fixed_len;  // program decode of a fixed-layout stream: record i at i * fixed_len
                       // (offs unused; a non-canonical record latches first_irregular
                       // and joins the exception list exc[0 .. exc_cap))
  uint64_t* exc;
  uint64_t exc_cap;
  DeepArgs deep;
  // records actually present (device word, e.g. the stream index's total):
  // records [min(n, *n_dev), n) are left alone; nullptr: all n
  const unsigned long long* n_dev;
  // block rule (ArenaPack): a block packed by the decode tile is marked with
  // pack_epoch (nullptr: the call does not pack); pack_k = the program's list
  // ops (the compiled decode tile packs only when they are its own)
  uint32_t* pack_flags;
  uint32_t pack_epoch;
  uint32_t pack_k;
};

// Schemaless skim of an indexed stream (k_skim.hip, tgpu_skim_batch).
struct SkimArgs {
  const uint8_t* in;
  uint64_t in_len;
  const uint64_t* offs;  // n+1 record starts
  uint64_t n;
  tgpu_skim_field* fields;
  uint32_t* counts;
  uint32_t max_fields;
  int32_t string_limit, container_limit, max_depth, height;
  DevResult* res;
  int nt_stores;  // entries stored non-temporally (never re-read here)
  uint32_t max_nest;  // struct-valued fields descended into (0: top level only)
  DeepArgs deep;
};

struct EncodeArgs {
  DevSchema sc;
  const uint8_t* recs;
  uint64_t n;
  const uint8_t* sbase;
  const uint8_t* lbase;
  uint8_t* out;
  uint64_t cap;
  uint64_t* offs;  // n+1: sizes, then offsets
  unsigned long long* block_sums;
  unsigned long long* scan_part;  // scan_tiles_parts(tiles) partial sums
  uint32_t rec_size;
  DevResult* res;
  uint64_t fixed_len;  // program write of a fixed-layout schema: record i at i * fixed_len
  uint32_t recompute;  // compiled write pass sizes its records; the size pass writes tile sums only
  uint32_t out_cap;    // write pass: LDS output tile bytes (0: prog::kOutCap)
  // general encode: records nested past the private frames (kErrDeep) are
  // sized and written again by deep-pass lanes with HBM frames
  DeepArgs deep;
};

// Wire-to-wire transcoding of an indexed stream (tgpu_xcode.h,
// k_transcode.hip): d = the source (d.offs n+1 starts; d.arena the list
// workspace of a Compact source; d.recs the record workspace of the records
// the source program cannot take, which the general reader decodes), e = the
// target (e.offs: the listed records' sizes, then every output start the
// finish or the caller reads; e.recs = d.recs, e.sbase = d.in, e.lbase =
// d.arena for those records).
struct XcodeArgs {
  DecodeArgs d;
  EncodeArgs e;
  uint64_t* irr;              // records left to the general reader / writer
  unsigned long long* nirr;
  uint32_t want_offs;         // the caller asked for every output start
  uint32_t out_mean;          // estimated target bytes per record (LDS sizing; 0: unknown)
  // single pass (tgpu_xcode.h xc_one_tile): per-tile look-back status words
  // (tiles + 1, zeroed before the launch; nullptr: the two tile passes)
  unsigned long long* xstat;
  // the two-pass kernels behind a single pass run only when *gate != 0 (a
  // record left to the general reader, or a look-back past its bound);
  // nullptr: always
  const unsigned long long* gate;
};

// ---- stream indexer (k_index.hip) -------------------------------------------
// Finds the start of every record beginning in [begin, end) of an unindexed
// stream: lanes speculate record starts per chunk, a serial pass repairs the
// chunk chain where speculation was wrong, the starts are emitted in order.
struct IndexArgs {
  DevSchema sc;
  const uint8_t* in;
  uint64_t in_len;
  uint64_t begin, end;
  int32_t speculative;
  int32_t protocol;
  uint64_t chunk;      // bytes of record starts per chunk
  uint32_t window;     // candidate starts tried per chunk
  uint32_t rec_size;
  uint64_t n_chunks;
  int32_t string_limit, container_limit, max_depth, height;
  const VProgram* prog;  // canonical-form program (nullptr: general reader only)
  // per chunk: speculated/verified first start, end of the chain, record count
  uint64_t* s;
  uint64_t* e;
  uint64_t* sst;             // speculation: the chain's first kSpecStarts starts
                             // (sst[j * kSpecStarts] == s[j] when valid)
  unsigned long long* cnt;
  uint64_t* pf;              // speculation: where the program stopped (partial chain)
  uint64_t* ep;              // emit: where the program stopped (kNo: done)
  unsigned long long* ec;    // emit: starts written before it stopped
  uint32_t* lanes;           // LDS tiles: per-lane (start, count) of the speculation pass
  unsigned long long* base;  // flags, then exclusive record-count prefix
  unsigned long long* bad;   // chunks whose chain link failed (in order)
  unsigned long long* part;  // scan partials
  unsigned long long* scal;  // [0] bad count, [1] chunks in effect, [2] error chunk,
                             // [3] records before the error in it, [4] error record start,
                             // [5] total, single pass: [6] ticket, [7] failed, [8..11]
                             // look-back windows / restarts / repairs / failed tiles
  uint8_t* scratch;          // n_chunks * rec_size: general-reader output (discarded)
  uint64_t* offs;            // record starts (max_records + 1)
  uint64_t max_records;
  uint64_t fill_to;          // decode: offs[total+1 .. fill_to] = last end
  DevResult* res;
  // fused decode (index tiles decode their records as they emit the starts;
  // recs == nullptr: index only): records [0, n_decode) of stride rec_size,
  // list arena, and the list of records left to the general decoder
  uint8_t* recs;
  uint8_t* arena;
  uint64_t arena_cap;
  uint64_t n_decode;
  uint64_t* irr;
  unsigned long long* nirr;
  int32_t decode_tail;  // a stream shorter than n_decode: its first missing record fails
  int32_t pad_;
  DeepArgs deep;        // records: fused decode deferrals; chunks: deep_chunks
  uint64_t* deep_chunks;  // emit chains stopped by kErrDeep (count: res->n_deep_chunks)
  // LDS tiles: the speculation pass's record starts per tile (tile-relative,
  // st_cap per tile; valid where pf[j] == kStartsValid), so the emit pass
  // copies them instead of re-walking the tile; nullptr: off
  uint16_t* st16;
  uint32_t st_cap;
  // the records are decoded after the index by the indexed program decode
  // (launch_index) rather than in the emit tiles: emit writes starts only,
  // the finish keeps the fused decode's tail rule
  int32_t st_decode;
  // schemas without a program: the bytes a record of the root struct can
  // start with (a root field's header, or STOP), one bit each — every
  // record of a speculated chain must (the fallback pass takes any)
  uint32_t hmask[8];
  // exhaustive resolution (program-less streams whose speculation left many
  // links broken, k_index.hip index_xtab_kernel): per chunk and entry offset
  // w < kXWindow, the chain's exit (bit 63: it ends in a record the reader
  // rejects, at that position) and its records; per-lane reader scratch
  uint64_t* xe;
  uint32_t* xc;
  uint8_t* xscratch;
  // bytes a speculated chain may read past its chunk (kSpecReach default;
  // TGPU_INDEX_SPEC_REACH) and a position's record past the exhaustive
  // resolution's chunk (<= kXReach; TGPU_INDEX_XREACH)
  uint32_t spec_reach;
  uint32_t x_reach;
};
constexpr uint32_t kXWindow = 256;  // entry offsets per chunk in the exhaustive tables

// Workspace of the exhaustive resolution, allocated only when a call needs
// it (tgpu_api.cpp: the context's grow-only buffer); nullptr: unavailable.
struct XTabAlloc {
  void* user;
  uint8_t* (*get)(void* user, uint64_t bytes);
};

// Workgroups of the grid-stride kernels whose lanes run the general reader
// for the few records / chunks the fast paths hand over (k_index.hip
// SCRATCH_KERNEL): their per-lane scratch is backed per resident wave, so a
// small grid keeps that backing small.
constexpr uint32_t kScratchGrid = 64;

#ifndef __HIPCC_RTC__
// LDS of the current device (hipDeviceAttributeMaxSharedMemoryPerMultiprocessor
// / ...PerBlock, read once per process; 160 KiB / 160 KiB on gfx950, the
// values the occupancy rules below were tuned on). k_program.hip.
int64_t device_lds_per_cu();
uint32_t lds_per_block_limit();
// the transcoder's smallest useful LDS output tile (a residency that leaves
// less takes fewer workgroups per CU instead)
constexpr uint32_t kMinXcodeOut = 1024;
// Launchers (defined in the .hip files; all asynchronous on `stream`).
// `t` is the host copy (launch geometry), `d_t` the device copy the kernels read.
// Fixed-layout decodes: a record they cannot take joins the exception list
// exc[0 .. exc_cap) (count res->n_irregular, first res->first_irregular);
// launch_fixed_exceptions then reads the listed records at their stride.
hipError_t launch_fixed_binary_decode(const FixedTemplate* t, const FixedTemplate* d_t,
                                      const uint8_t* in, uint64_t n, uint8_t* out,
                                      DevResult* res, uint64_t* exc, uint64_t exc_cap,
                                      hipStream_t stream);
hipError_t launch_fixed_binary_encode(const FixedTemplate* t, const FixedTemplate* d_t,
                                      const uint8_t* recs, uint64_t n, uint8_t* out,
                                      uint64_t* offsets, DevResult* res,
                                      hipStream_t stream);
// Word-gather variants (S % 8 == 0, record buffer 8-byte aligned).
hipError_t launch_plan_binary_decode(const FixedPlan* p, const FixedPlan* d_p,
                                     const uint8_t* in, uint64_t n, uint8_t* out,
                                     DevResult* res, uint64_t* exc, uint64_t exc_cap,
                                     hipStream_t stream);
// The fixed-layout decodes' exception records read by the general reader at
// i * L: one that does not read exactly L bytes (or fails) moves
// res->first_misfit; then first_irregular = the first misfit when the list was
// complete (else it stands), n_irregular = 0. Stream-ordered, no host sync.
hipError_t launch_fixed_exceptions(const DecodeArgs& a, int protocol, uint64_t L,
                                   hipStream_t stream);
// Stream-ordered fixed-layout calls (no host status, no host round trip):
// launch_fixed_exceptions with the resolve step followed, when a record m is
// off the stride, by record m's length L2 read by the general reader
// (res->tail_*; tail_stride stays 0 when L2 > max_stride or record m fails).
// The strided tail decode (tgpu_jit_decode_tail) then takes records m.. at
// stride L2; launch_fixed_stream_finish reads its exceptions at their stride
// positions and one lane walks from the first record off either stride.
hipError_t launch_fixed_exceptions_stream(const DecodeArgs& a, int protocol, uint64_t L,
                                          uint64_t max_stride, hipStream_t stream);
hipError_t launch_fixed_stream_finish(const DecodeArgs& a, int protocol, uint64_t L,
                                      hipStream_t stream);
// The strided tail decode (J: the tolerant program's JIT_DECODE group),
// persistent, one launch; max_stride: the longest record its tile takes.
uint64_t stream_tail_max_stride(uint32_t rec_size, uint32_t L);
struct JitKernels;
hipError_t launch_stream_tail_decode(const DecodeArgs& a, uint32_t rec_size, uint32_t L,
                                     uint64_t* irr, unsigned long long* nirr, hipStream_t stream,
                                     const JitKernels* J, int device);
// Blocking fixed-layout calls: reads record 0 at offset 0 with the general
// reader; res->first_misfit = 0 when it is not L bytes long (or fails).
hipError_t launch_fixed_probe(const DecodeArgs& a, int protocol, uint64_t L, hipStream_t stream);
hipError_t launch_plan_binary_encode(const FixedPlan* p, const FixedPlan* d_p,
                                     const uint8_t* recs, uint64_t n, uint8_t* out,
                                     uint64_t* offsets, DevResult* res,
                                     hipStream_t stream);
hipError_t launch_general_decode(const DecodeArgs& a, int protocol,
                                 hipStream_t stream);
// Compiled-program fast path over an indexed stream (a.offs): canonical records
// are decoded from an LDS-staged tile; the others are appended to `irregular`
// (count in *n_irregular) and decoded by launch_general_decode_list.
// ---- schema compiler (tgpu_jit.cpp) ------------------------------------------
// Kernels generated and compiled for one program (nullptr: not compiled —
// policy or failure; the interpreting kernels run instead).
struct JitKernels;
// JIT_NESTED: the indexed decode of a nested program (VOP_SEQ), generated as
// straight-line code with one loop per container level.
// JIT_NINDEX: the stream index's speculation / emit kernels over a nested
// program's measuring walk.
// JIT_XCODE: the transcoder's program pair (tgpu_xcode.h), jit_kernels_xcode.
enum JitGroup {
  JIT_DECODE = 0,
  JIT_ENCODE = 1,
  JIT_INDEX = 2,
  JIT_NESTED = 3,
  JIT_NINDEX = 4,
  JIT_XCODE = 5
};
const JitKernels* jit_kernels(const VProgram& prog, int device, int group, uint64_t records,
                              uint64_t bytes, bool force);
// Records of at most 128 bytes, S % 8 == 0, get a second compiled decode
// that builds records in registers instead of an LDS record tile
// (decode_tile kRS, JIT_DECODE entry 2).
bool decode_regrec(uint32_t rec_size);
// only_group >= 0: that group alone
int jit_compile_check(const VProgram& P, const char* arch, char* log, uint64_t log_cap,
                      int only_group = -1);
// entry `which` of a compiled group exists (JIT_DECODE entry 1, the strided
// tail decode: tolerant programs only)
bool jit_has(const JitKernels* J, int which);
hipError_t jit_launch_decode(const JitKernels* J, const DecodeArgs& a, uint64_t grid,
                             uint32_t cap, uint32_t lds, uint64_t* irr, unsigned long long* nirr,
                             hipStream_t s, int which = 0);
// first: the group's first encode entry (JIT_NESTED: 2, its size / write)
hipError_t jit_launch_encode(const JitKernels* J, bool write, const EncodeArgs& a, uint64_t grid,
                             uint32_t lds, hipStream_t s, int first = 0);
// The transcoder's pair (source program's decode, target program's writer);
// which: 0 size, 1 write, 2 / 3 the same with records in registers.
const JitKernels* jit_kernels_xcode(const VProgram& ps, const VProgram& pd, int device,
                                    uint64_t records, bool force);
hipError_t jit_launch_xcode(const JitKernels* J, int which, const XcodeArgs& x, uint64_t grid,
                            uint32_t cap, uint32_t ocap, uint32_t lds, hipStream_t s);
int jit_compile_check_xcode(const VProgram& ps, const VProgram& pd, const char* arch, char* log,
                            uint64_t log_cap);
// Wire-to-wire transcoding of x.d's indexed stream (k_transcode.hip): the
// pair's compiled kernels (jit) or the AOT DynProg pair over d_ps / d_pd.
hipError_t launch_xcode(const XcodeArgs& x, int from, int to, const VProgram* d_ps,
                        const VProgram* d_pd, hipStream_t s, const JitKernels* jit);
// which: 0 speculation, 1 emit, 2 emit + fused decode
hipError_t jit_launch_index(const JitKernels* J, int which, const IndexArgs& a, uint64_t grid,
                            hipStream_t s);

// jit: the schema's compiled kernels (nullptr: interpret d_prog).
// VOP_LIST ops of a flat program (the compiled decode tile's block-rule
// table: prog_list_ops x 8 bytes per record).
inline uint32_t prog_list_ops(const VProgram& P) {
  uint32_t k = 0;
  for (uint32_t i = 0; i < P.n_ops; ++i) k += P.ops[i].kind == VOP_LIST ? 1u : 0u;
  return k;
}
// Block rule: blocks of records [0, m) (m from the finished call's DevResult:
// n_records, + 1 for a failing record) not marked by the decode (k_arena.hip).
hipError_t launch_arena_pack(const DecodeArgs& a, const ArenaPack& p, hipStream_t stream);
hipError_t launch_program_decode(const DecodeArgs& a, const VProgram* d_prog,
                                 uint32_t rec_size, uint64_t* irregular,
                                 unsigned long long* n_irregular, hipStream_t stream,
                                 const JitKernels* jit, uint64_t span_bytes = 0);
hipError_t launch_general_decode_list(const DecodeArgs& a, int protocol,
                                      const uint64_t* list,
                                      const unsigned long long* n_list,
                                      hipStream_t stream);
hipError_t launch_skim(const SkimArgs& a, int protocol, hipStream_t stream);
// The records deferred by kErrDeep (a.deep), redone with HBM skip frames.
hipError_t launch_deep_decode(const DecodeArgs& a, int protocol, hipStream_t stream);
// Status of a fixed-layout batch whose tail from record rec_base was indexed
// and decoded (a: the tail, indices relative to rec_base).
hipError_t launch_tail_decode_finish(const DecodeArgs& a, int protocol, uint64_t rec_base,
                                     hipStream_t stream);
hipError_t launch_decode_finish(const DecodeArgs& a, int protocol,
                                uint64_t fixed_len, hipStream_t stream);
// nj: a nested program's compiled kernels (JIT_NESTED) for the size / write
// passes instead of the general writer's (nullptr: the general writer);
// defer: its program is a recursive schema's unrolled one, whose deferred
// records the deep pass sizes and writes.
hipError_t launch_general_encode(const EncodeArgs& a, int protocol,
                                 uint64_t n_blocks, hipStream_t stream,
                                 const JitKernels* nj = nullptr, bool defer = false);
hipError_t launch_general_size(const EncodeArgs& a, int protocol,
                               uint64_t n_blocks, hipStream_t stream,
                               const JitKernels* nj = nullptr, bool defer = false);
hipError_t launch_encode_finish(const EncodeArgs& a, int protocol,
                                uint64_t fixed_len, hipStream_t stream);
hipError_t launch_result_init(DevResult* res, uint64_t n, hipStream_t stream);
// Exclusive scan of nb per-tile byte counts in place; the total goes to
// *total1 and *total2 (either may be null). `part` holds scan_tiles_parts(nb)
// entries.
hipError_t launch_scan_tiles(unsigned long long* sums, uint64_t nb, unsigned long long* part,
                             unsigned long long* total1, uint64_t* total2, hipStream_t stream);
uint64_t scan_tiles_parts(uint64_t nb);
// Compiled-program encode (all-unqualified schemas): size pass, tile scan and,
// unless size_only, the write pass. a.offs receives sizes then start offsets
// (size_only: sizes, tile sums scanned; launch_size_offsets finishes them).
bool program_encode_fits(uint32_t rec_size);
hipError_t launch_program_encode(const EncodeArgs& a, const VProgram* d_prog,
                                 unsigned long long* part, bool size_only, hipStream_t stream,
                                 const JitKernels* jit);
hipError_t launch_size_offsets(const EncodeArgs& a, uint64_t n_blocks, hipStream_t stream);
// Fixed-layout schemas through the compiled program kernels (a.fixed_len set):
// no size pass; offsets (when a.offs) are i * fixed_len.
hipError_t launch_program_write_fixed(const EncodeArgs& a, const VProgram* d_prog,
                                      hipStream_t stream, const JitKernels* jit);

// ---- host-memory pipeline (tgpu_host.cpp) -------------------------------------
void* host_pipe_create();
void host_pipe_destroy(void* pipe);
void* context_host_pipe(tgpu_context* ctx);  // created on first use, owned by ctx
// The list spans of a schema whose decoded list arena holds nothing but
// scalar list / set elements (a flat record program; no nested regions, no
// strings inside containers): their member offsets and element widths, at
// most `max` (tgpu_decode_host_chunks_ex's packing). 0: none, or not such a
// schema.
uint32_t packable_lists(const tgpu_schema* s, int protocol, uint32_t* member, uint32_t* width,
                        uint32_t max);
bool schema_has_lists(const tgpu_schema* schema);
// the schema's list arrays follow the block rule (ArenaPack n > 0)
bool schema_block_rule(const tgpu_schema* schema);

// ---- stream indexer (k_index.hip) launchers
// mean: the stream's mean record length when known (0: not), program-less
// streams only
uint64_t index_chunk_bytes(uint64_t span, bool tiles, uint64_t mean = 0);
uint64_t index_tile_bytes();
uint64_t index_tile_lanes();
// Returns (in *fused) whether the records were decoded during the index
// (a.recs set and the LDS-tile path taken); otherwise the caller decodes them
// from the index.
// h_sync (pinned, >= 4 words; nullptr: no host reads): the index may
// synchronize to read its tile summary and skip the general-reader helper
// kernels no tile needs; h_sync[3] then holds the record total (else it is
// left alone).
hipError_t launch_index_stream(const IndexArgs& a, hipStream_t stream, const JitKernels* jit,
                               bool* fused, uint64_t* h_sync = nullptr,
                               const XTabAlloc* xalloc = nullptr);
// After a fused index + decode over a stream range: re-diagnoses a record
// the index accepted but the decode could not store (list arena overflow).
hipError_t launch_stream_decode_finish(const DecodeArgs& a, int protocol, hipStream_t stream);
// The index's epilogue: total / end / status (index_finish_kernel), the
// fused decode's missing-record hand-off and the decode padding of offs.
hipError_t launch_index_finish(const IndexArgs& a, bool decode, hipStream_t stream);
// Single-pass index (+ fused decode when a.recs): LDS tiles with decoupled
// look-back; leaves a.scal[7] != 0 when some tile could not finish alone (the
// caller then runs launch_index_stream), else the index's arrays as the
// two-pass index leaves them before its epilogue (launch_index_finish).
// Program schemas with kTile chunks only.
hipError_t launch_index_onepass(const IndexArgs& a, hipStream_t stream, const JitKernels* jit,
                                bool rr = false);
// Empty range: offs[0..fill_to] = pos, no records.
hipError_t launch_index_empty(DevResult* res, uint64_t* offs, uint64_t pos, uint64_t fill_to,
                              hipStream_t stream);
#endif  // !__HIPCC_RTC__

}  // namespace tgpu

static_assert(sizeof(tgpu::FixedPlan) % 16 == 0, "FixedPlan is copied to LDS in 16-byte chunks");
