// tgpu_jit.cpp — the schema compiler: per-schema gfx950 kernels generated and
// compiled at run time (hipRTC), the device-side counterpart of the
// reference's thrift1 code generation. The reference emits one specialized
// T::readNoXfer / T::write per struct at build time
// (thrift/compiler/generate/templates/cpp2/module_types_custom_protocol_h/
// deserialize_struct.whisker:19-160, serialize_struct.whisker:40-67); a
// batch codec that receives its schema as a runtime table
// (TableBasedSerializer.h:90-118 — the tgpu_schema_create descriptor) can do
// the same once per schema: the schema's canonical program (VProgram) is
// written out as compile-time constants and the shared kernel bodies of
// tgpu_prog_kernels.h are instantiated on it, so every header byte, width,
// member offset and op dispatch folds into straight-line code.
//
// The library's own (AOT) kernels interpret the same program from device
// memory and stay the path for small batches, for schemas compiled on a
// device without hipRTC, and when TGPU_JIT=0. Policy (TGPU_JIT):
//   unset  compile when a call's batch reaches kAutoRecords records (or an
//          index call kAutoBytes bytes); use compiled kernels whenever present
//   1      compile on first use, any batch size
//   0      never compile or use them
// Compiled modules are cached per (device, program) for the process.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "tgpu_internal.h"
#include "jit_headers.inc"

namespace tgpu {

// One compiled group of kernels (JIT_DECODE: decode; JIT_ENCODE: size,
// write; JIT_INDEX: index spec, index emit, fused index emit + decode).
// Groups compile separately, on
// first need, so a decode-only caller never waits for the encoder.
struct JitKernels {
  hipModule_t mod = nullptr;
  hipFunction_t f[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  bool ok = false;
  std::string log;
};

namespace {

constexpr uint64_t kAutoRecords = 1ull << 16;
constexpr uint64_t kAutoBytes = 4ull << 20;

std::mutex g_mu;
std::map<std::string, JitKernels*>& cache() {
  static std::map<std::string, JitKernels*> m;
  return m;
}

int jit_mode() {
  const char* e = getenv("TGPU_JIT");
  if (!e || !*e) return 2;
  return atoi(e) ? 1 : 0;
}

std::string cache_key(const VProgram& P, int device, int group) {
  std::string k((const char*)&P, offsetof(VProgram, ops) + P.n_ops * sizeof(VOp));
  if (const char* v = getenv("TGPU_JIT_DEFINES")) k += v;
  k.append((const char*)&device, sizeof(device));
  k.append((const char*)&group, sizeof(group));
  return k;
}

const char* const kEntry[6][6] = {
    {"tgpu_jit_decode", "tgpu_jit_decode_tail", "tgpu_jit_decode_rr", nullptr, nullptr, nullptr},
    {"tgpu_jit_size", "tgpu_jit_write", "tgpu_jit_write_one", nullptr, nullptr, nullptr},
    {"tgpu_jit_index_spec", "tgpu_jit_index_emit", "tgpu_jit_index_decode",
     "tgpu_jit_index_onepass", "tgpu_jit_index_onepass_decode", "tgpu_jit_index_onepass_rr"},
    {"tgpu_jit_ndecode", "tgpu_jit_ndecode_hbm", "tgpu_jit_nsize", "tgpu_jit_nwrite", nullptr,
     nullptr},
    {"tgpu_jit_nindex_spec", "tgpu_jit_nindex_emit", nullptr, nullptr, nullptr, nullptr},
    {"tgpu_jit_xc_size", "tgpu_jit_xc_write", "tgpu_jit_xc_size_rr", "tgpu_jit_xc_write_rr",
     "tgpu_jit_xc_one", "tgpu_jit_xc_one_rr"}};

// The record function of a nested program (decode when !enc, the writer
// when enc): ops [k, stop) of the object at `b` (a variable name). Each
// VOP_SBEGIN opens a struct's scope with its Compact delta base `l<k>` (the
// last field id read / written), VOP_FHDR is a field header — read or
// written from the base, in a branch on presence for an optional field
// (its value ops, the next `bits` ops, inside) — VOP_SEND the struct's STOP;
// each VOP_SEQ / VOP_MSEQ a counted loop over its element slots. Leaf ops
// are the program's op helpers on the constant op.
// meas: the measuring walk of the stream index (decode form, nothing stored).
// uvar: inside a union's scope, the flag of a member taken (union_declare:
// the first present member on read — a second one fails the STOP check and
// goes to the general reader, which reports UNION_MISSING_STOP — and the
// first set one on write, serialize_union.whisker:52-66).
void gen_code(std::ostringstream& o, const VProgram& P, uint32_t k, uint32_t stop,
              const std::string& b, int indent, bool enc, std::string last, bool meas = false,
              const std::string& uvar = "") {
  const bool compact = P.protocol != TGPU_PROTOCOL_BINARY;
  const std::string ks = meas ? "<false>" : "";
  while (k < stop) {
    const std::string in(indent, ' ');
    const VOp& v = P.ops[k];
    const std::string K = std::to_string(k), op = "kOps[" + K + "]";
    if (v.kind == VOP_SBEGIN) {
      // the struct's fields up to its VOP_SEND (hdr_len: one past it)
      o << in << "{\n" << in << "  int32_t l" << K << " = 0;\n";
      if (compact) o << in << "  (void)l" << K << ";\n";
      if (v.width) o << in << "  bool u" << K << " = false;\n";
      gen_code(o, P, k + 1, v.hdr_len - 1, b, indent + 2, enc, "l" + K, meas,
               v.width ? "u" + K : std::string());
      if (enc) o << in << "  o.put(0, 1);\n";  // writeFieldStop
      else o << in << "  if (!struct_stop(src, p, end)) return false;\n";
      o << in << "}\n";
      k = v.hdr_len;
      continue;
    }
    if (v.kind == VOP_FHDR) {
      const uint32_t vend = k + 1 + v.bits;  // the field's value ops
      const bool opt = v.width != 0;
      const int32_t id = (int16_t)v.member;
      const bool cbool = compact && v.is_bool;  // the value rides in the header
      std::string hdr;
      if (enc) {
        if (cbool) {
          const VOp& cv = P.ops[k + 1];
          hdr = "put_cbool_field(o, " + std::to_string(id) + ", " + last + ", " + b + "[" +
                std::to_string(cv.member) + "])";
        } else if (compact) {
          hdr = "(put_cfield(o, " + std::to_string(id) + ", " + std::to_string(v.elem_ct) + "u, " +
                last + "), true)";
        } else {
          hdr = "(o.put(" + std::to_string(v.hdr) + "u, 3), true)";
        }
        if (!uvar.empty()) {
          o << in << "if (!" << uvar << " && " << b << "[" << v.isset << "]) {\n"
            << in << "  " << uvar << " = true;\n";
        } else if (opt && v.elem_kind) {  // terse: written unless empty
          const VOp& val = P.ops[k + 1];
          const uint32_t w = (val.kind == VOP_FIXED || val.kind == VOP_VARINT) ? val.width
                             : val.kind == VOP_CBOOL ? 1u : 0u;  // 0: a span (string, container)
          o << in << "if (!terse_leaf_empty(" << b << " + " << val.member << "u, " << w << "u)) {\n";
        } else if (opt) {
          o << in << "if (" << b << "[" << v.isset << "]) {\n";
        } else {
          o << in << "{\n";
        }
        o << in << "  if (!" << hdr << ") return false;\n";
        if (!cbool) gen_code(o, P, k + 1, vend, b, indent + 2, enc, last, meas);
        o << in << "}\n";
      } else {
        if (cbool) {
          const VOp& cv = P.ops[k + 1];
          hdr = "cbool_field" + ks + "(src, p, end, " + std::to_string(id) + ", " + last + ", " + b + " + " +
                std::to_string(cv.member) + "u, " + b + " + " + std::to_string(cv.isset) + "u)";
        } else if (compact) {
          hdr = "cfield(src, p, end, " + std::to_string(id) + ", " + std::to_string(v.elem_ct) + "u, " +
                last + ")";
        } else {
          hdr = "bfield(src, p, end, " + std::to_string(v.hdr) + "u)";
        }
        if (!uvar.empty()) {
          o << in << "if (!" << uvar << " && " << hdr << ") {\n" << in << "  " << uvar << " = true;\n";
        } else if (opt) {
          o << in << "if (" << hdr << ") {\n";
        } else {
          o << in << "if (!" << hdr << ") return false;\n" << in << "{\n";
        }
        if (!cbool) gen_code(o, P, k + 1, vend, b, indent + 2, enc, last, meas);
        o << in << "}\n";
      }
      k = vend;
      continue;
    }
    if (v.kind == VOP_SEQ || v.kind == VOP_MSEQ) {
      const std::string n = "n" + K, a = "a" + K, i = "i" + K, e = "e" + K;
      const bool seq = v.kind == VOP_SEQ;
      bool stage = false;
      o << in << "{\n";
      if (enc) {
        o << in << "  const tgpu_span s" << K << " = seq_span(" << op << ", " << b << ");\n"
          << in << "  if (!" << (seq ? "put_list_header" : "put_map_header") << "(o, " << op
          << ", kCompact, s" << K << ".length)) return false;\n"
          << in << "  const uint32_t " << n << " = s" << K << ".length;\n"
          << in << "  const uint8_t* " << a << " = lbase + s" << K << ".offset;\n"
          << in << "  for (uint32_t " << i << " = 0; " << i << " < " << n << "; ++" << i << ") {\n";
        // a small struct slot is read into registers first (its members
        // were one dependent global load each); A/B: TGPU_JIT_DEFINES
        // naming TGPU_NESTED_NOLOADSTAGE
        const char* defs = getenv("TGPU_JIT_DEFINES");
        const bool sslot = v.elem_ttype == TGPU_T_STRUCT ||
                           (v.kind == VOP_MSEQ && v.width == TGPU_T_STRUCT);
        if (sslot && v.hdr <= 64 && v.hdr % 8 == 0 &&
            !(defs && strstr(defs, "TGPU_NESTED_NOLOADSTAGE"))) {
          o << in << "    alignas(8) uint8_t " << e << "[" << v.hdr << "];\n"
            << in << "    load_slot<" << v.hdr << "u>(" << e << ", " << a << " + (uint64_t)" << i
            << " * " << v.hdr << "u);\n";
        } else {
          o << in << "    const uint8_t* " << e << " = " << a << " + (uint64_t)" << i << " * "
            << v.hdr << "u;\n";
        }
      } else {
        o << in << "  uint32_t " << n << ";\n"
          << in << "  uint8_t* " << a << ";\n"
          << in << "  if (!" << (seq ? "seq_open" : "mseq_open") << ks << "(" << op
          << ", kCompact, src, c, p, end, " << b << ", bump, " << n << ", " << a
          << ")) return false;\n"
          << in << "  for (uint32_t " << i << " = 0; " << i << " < " << n << "; ++" << i << ") {\n";
        // (a struct element / value is default-constructed first; every
        // other slot is written whole)
        const bool zero = (v.elem_ttype == TGPU_T_STRUCT ||
                           (v.kind == VOP_MSEQ && v.width == TGPU_T_STRUCT)) && !meas;
        // a small struct slot is built in registers and leaves with whole
        // 8-byte stores (written member by member into the arena it took a
        // global store per member and per isset byte)
        // (decode 3.62 -> 2.50 ms on the nested leg with the paired list
        // elements; A/B: TGPU_JIT_DEFINES naming TGPU_NESTED_NOSTAGE)
        const char* defs = getenv("TGPU_JIT_DEFINES");
        stage = zero && v.hdr <= 64 && v.hdr % 8 == 0 &&
                !(defs && strstr(defs, "TGPU_NESTED_NOSTAGE"));
        if (stage) {
          o << in << "    uint8_t* " << e << "_dst = " << a << " + (uint64_t)" << i << " * " << v.hdr
            << "u;\n"
            << in << "    alignas(8) uint8_t " << e << "[" << v.hdr << "];\n";
        } else {
          o << in << "    uint8_t* " << e << " = " << a << " + (uint64_t)" << i << " * " << v.hdr
            << "u;\n";
        }
        if (zero) o << in << "    zero_slot<" << v.hdr << "u>(" << e << ");\n";
      }
      gen_code(o, P, k + 1, v.hdr_len - 1, e, indent + 4, enc, last, meas);
      if (stage) o << in << "    copy_slot<" << v.hdr << "u>(" << e << "_dst, " << e << ");\n";
      o << in << "  }\n";
      if (!enc && !meas) o << in << "  seq_close(" << op << ", " << b << ");\n";
      o << in << "}\n";
      k = v.hdr_len;  // past the VOP_SEQ_END
      continue;
    }
    if (v.kind == VOP_BOX) {
      // a boxed struct field: its object from the record's region, zeroed
      // (make_mutable_smart_ptr), read, then the member points to it
      // (deserialize_field.whisker:21-23,49-51); written from its object, or
      // as an empty struct when null (serialize_field.whisker:44-49)
      const std::string x = "x" + K, s = "s" + K;
      o << in << "{\n";
      if (enc) {
        o << in << "  const tgpu_span " << s << " = *(const tgpu_span*)(" << b << " + " << v.member
          << "u);\n"
          << in << "  if (" << s << ".length == 0) {\n"
          << in << "    o.put(0, 1);\n"
          << in << "  } else {\n"
          << in << "    const uint8_t* " << x << " = lbase + " << s << ".offset;\n";
        gen_code(o, P, k + 1, v.hdr_len - 1, x, indent + 4, enc, last, meas);
        o << in << "  }\n";
      } else if (meas) {
        gen_code(o, P, k + 1, v.hdr_len - 1, b, indent + 2, enc, last, meas);
      } else {
        o << in << "  uint64_t a" << K << ";\n"
          << in << "  uint8_t* " << x << ";\n"
          << in << "  if (!box_open<" << v.hdr << "u>(c, bump, a" << K << ", " << x
          << ")) return false;\n";
        gen_code(o, P, k + 1, v.hdr_len - 1, x, indent + 2, enc, last, meas);
        o << in << "  *(tgpu_span*)(" << b << " + " << v.member << "u) = tgpu_span{a" << K
          << ", 1u, 0u};\n";
      }
      o << in << "}\n";
      k = v.hdr_len;  // past the VOP_BOX_END
      continue;
    }
    if (v.kind == VOP_SEQ_END || v.kind == VOP_SEND || v.kind == VOP_BOX_END) {
      ++k;
      continue;
    }
    if (v.kind == VOP_DEFER) {  // a recursive struct past the unrolled levels
      o << in << "return false;\n";
      ++k;
      continue;
    }
    if (enc) {
      if (v.kind != VOP_ISSET)
        o << in << "if (!enc_op(" << op << ", kCompact, " << b << ", sbase, lbase, o)) return false;\n";
    } else if (v.kind == VOP_LIST) {
      o << in << "if (!nlist" << ks << "(" << op << ", kCompact, src, c, p, end, " << b
        << ", bump)) return false;\n";
    } else if (v.kind != VOP_ISSET || !meas) {
      o << in << "if (!run_op<" << (meas ? "false" : "true") << ">(" << op
        << ", kCompact, src, c, p, end, " << b << ", W)) return false;\n";
    }
    ++k;
  }
}

// The generated translation unit: the program as constants + one entry point
// per kernel body.
// A program as compile-time constants: the op array `arr` and the program
// accessor `name` (tgpu_program.h's DynProg interface, kStatic).
void gen_prog(std::ostringstream& o, const VProgram& P, const char* arr, const char* name) {
  // (kLists: the block rule's table in the decode tile, decode_tile pack_tile)
  o << "__device__ constexpr tgpu::VOp " << arr << "[" << (P.n_ops ? P.n_ops : 1) << "] = {\n";
  for (uint32_t k = 0; k < P.n_ops; ++k) {
    const VOp& v = P.ops[k];
    o << "  {" << (unsigned)v.kind << ", " << (unsigned)v.hdr_len << ", " << (unsigned)v.width
      << ", " << (unsigned)v.bits << ", " << v.hdr << "u, " << v.member << ", " << v.isset << ", "
      << (unsigned)v.elem_kind << ", " << (unsigned)v.elem_ttype << ", " << (unsigned)v.elem_ct
      << ", " << (unsigned)v.is_bool << "},\n";
  }
  if (!P.n_ops) o << "  {}\n";
  o << "};\n"
       "struct "
    << name
    << " {\n"
       "  static constexpr bool kStatic = true;\n"
       "  static constexpr uint32_t kN = "
    << P.n_ops
    << ";\n"
       "  static constexpr uint32_t kLists = "
    << prog_list_ops(P)
    << ";\n"
       "  __device__ static constexpr uint32_t n_ops() { return kN; }\n"
       "  __device__ static constexpr uint32_t protocol() { return "
    << P.protocol
    << "; }\n"
       "  __device__ static constexpr bool has_lists() { return "
    << (P.has_list ? "true" : "false")
    << "; }\n"
       "  __device__ constexpr tgpu::VOp op(uint32_t k) const { return "
    << arr
    << "[k]; }\n"
       "};\n";
}

// The transcoder's pair (JIT_XCODE): the source program's decode and the
// target program's writer in the tile passes of tgpu_xcode.h — size, write
// and the single pass — with records in registers where decode_regrec
// allows (entries 2, 3, 5).
std::string gen_source_xcode(const VProgram& Ps, const VProgram& Pd) {
  std::ostringstream o;
  o << "// generated by tgpu_jit.cpp for one schema's transcoding pair\n";
  if (const char* v = getenv("TGPU_JIT_DEFINES")) o << v << "\n";
  bool tails = false;
  for (uint32_t k = 0; k < Ps.n_ops; ++k)
    tails |= Ps.ops[k].kind == VOP_CONST && Ps.ops[k].elem_kind == kStopSkipsUnknown;
  if (!tails) o << "#define TGPU_NO_TAILS 1\n";
  o << "#include \"tgpu_xcode.h\"\n"
       "namespace {\n";
  gen_prog(o, Ps, "kOps", "JP");
  gen_prog(o, Pd, "kOps2", "JQ");
  o << "constexpr uint32_t kS = " << Ps.rec_size
    << ";\n"
       "}  // namespace\n"
       "using namespace tgpu;\n";
  auto pair = [&](const char* sfx, const char* rs) {
    o << "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_xc_size" << sfx
      << "(XcodeArgs x, uint32_t cap) {\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  __shared__ unsigned long long part[4];\n"
         "  prog::xc_size_tile<JP, JQ, "
      << rs
      << ">(x, JP{}, JQ{}, kS, cap, smem, part);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_xc_write"
      << sfx
      << "(XcodeArgs x, uint32_t cap, uint32_t ocap) {\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  __shared__ prog::EncodeShared sm;\n"
         "  prog::xc_write_tile<JP, JQ, "
      << rs
      << ">(x, JP{}, JQ{}, kS, cap, ocap, smem, sm);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_xc_one"
      << sfx
      << "(XcodeArgs x, uint32_t cap, uint32_t ocap) {\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  __shared__ prog::EncodeShared sm;\n"
         "  prog::xc_one_tile<JP, JQ, "
      << rs
      << ">(x, JP{}, JQ{}, kS, cap, ocap, smem, sm);\n"
         "}\n";
  };
  pair("", "0");
  if (decode_regrec(Ps.rec_size)) pair("_rr", "kS");
  return o.str();
}

std::string gen_source(const VProgram& P, int group) {
  std::ostringstream o;
  o << "// generated by tgpu_jit.cpp for one schema program\n";
  if (const char* v = getenv("TGPU_JIT_DEFINES")) o << v << "\n";  // A/B experiments
  // a strict program (no root STOP that skips appended fields) is generated
  // without that path: left in, the dead branch cost config 4's decode 39 %
  // (1.86 -> 2.58 ms; the compiler does not fold it away)
  bool tails = false, defer = false;
  for (uint32_t k = 0; k < P.n_ops; ++k) {
    tails |= P.ops[k].kind == VOP_CONST && P.ops[k].elem_kind == kStopSkipsUnknown;
    defer |= P.ops[k].kind == VOP_DEFER;  // a recursive schema's unrolled program
  }
  if (!tails) o << "#define TGPU_NO_TAILS 1\n";
  o << "#include \"tgpu_prog_kernels.h\"\n"
       "namespace {\n";
  gen_prog(o, P, "kOps", "JP");
  o << "constexpr uint32_t kS = "
    << P.rec_size
    << ";\n"
       "}  // namespace\n"
       "using namespace tgpu;\n";
  if (group == JIT_NINDEX) {
    // the stream index over a nested program: its measuring walk (the decode
    // form with nothing stored) behind a program accessor whose ops are only
    // what the index's candidate filter reads (the first header byte, STOP)
    VOp h0{};
    h0.kind = VOP_ISSET;  // (not a constant: no first-byte filter)
    if (P.n_ops > 2 && P.ops[0].kind == VOP_SBEGIN && P.ops[1].kind == VOP_FHDR &&
        !P.ops[1].width && !(P.protocol != TGPU_PROTOCOL_BINARY && P.ops[1].is_bool)) {
      h0.kind = VOP_CONST;
      h0.hdr_len = 1;
      const int32_t id = (int16_t)P.ops[1].member;
      h0.hdr = P.protocol == TGPU_PROTOCOL_BINARY ? (P.ops[1].hdr & 0xff)
               : (id > 0 && id <= 15) ? (((uint32_t)id << 4) | P.ops[1].elem_ct)
                                      : P.ops[1].elem_ct;
    }
    o << "#include \"tgpu_nested.h\"\n"
         "namespace {\n"
         "using namespace tgpu;\n"
         "using namespace tgpu::prog;\n"
         "constexpr bool kCompact = "
      << (P.protocol == TGPU_PROTOCOL_BINARY ? "false" : "true")
      << ";\n"
         "template <class Src>\n"
         // a recursive schema's unrolled walk is called, not inlined at each
         // of its call sites (chain, 10 levels: 36 -> 6.5 s to compile; the
         // index is not these schemas' hot path)
      << (defer ? "__device__ __noinline__" : "__device__ __forceinline__")
      << " bool nmeas(const Src& src, const Ctx& c, uint32_t& p, "
         "const uint32_t end) {\n"
         "  Win W;\n"
         "  uint8_t* rec = nullptr;\n"
         "  uint64_t bump = 0;\n"
         "  (void)rec;\n"
         "  (void)bump;\n";
    gen_code(o, P, 0, P.n_ops, "rec", 2, false, "", true);
    o << "  return true;\n"
         "}\n"
         "__device__ constexpr tgpu::VOp kH0 = {"
      << (unsigned)h0.kind << ", " << (unsigned)h0.hdr_len << ", 0, 0, " << h0.hdr
      << "u, 0, 65535, 0, 0, 0, 0};\n"
         "__device__ constexpr tgpu::VOp kStop = {1, 1, 0, 0, 0u, 0, 65535, 0, 0, 0, 0};\n"
         "struct NP {\n"
         "  static constexpr bool kStatic = true;\n"
         "  static constexpr uint32_t kN = 2;\n"
         "  static constexpr uint32_t kLists = 0;\n"
         "  __device__ static constexpr uint32_t n_ops() { return kN; }\n"
         "  __device__ static constexpr uint32_t protocol() { return "
      << P.protocol
      << "; }\n"
         "  __device__ static constexpr bool has_lists() { return true; }\n"
         "  __device__ constexpr tgpu::VOp op(uint32_t k) const { return k == 0 ? kH0 : kStop; }\n"
         "};\n"
         "// the measuring walks the index kernels take (found by ADL on NP)\n"
         "__device__ __forceinline__ bool measure_lds(const NP&, const uint32_t* w32, uint32_t lim, "
         "const Ctx& c, uint32_t& pos, uint32_t end, bool& slow) {\n"
         "  bool sl = false;\n"
         "  const ClampSrc src{w32, lim, &sl};\n"
         "  uint32_t p = pos;\n"
         "  const bool ok = nmeas(src, c, p, end);\n"
         "  slow = sl;\n"
         "  if (ok && !sl) pos = p;\n"
         "  return ok;\n"
         "}\n"
         "template <bool kStore, class Src>\n"
         "__device__ __forceinline__ bool run_program(const NP&, const Src& src, const Ctx& c, "
         "uint32_t& pos, uint32_t end, uint8_t*) {\n"
         "  if (kStore) return false;  // (never a fused decode: the nested decode follows)\n"
         "  uint32_t p = pos;\n"
         "  if (!nmeas(src, c, p, end)) return false;\n"
         "  pos = p;\n"
         "  return true;\n"
         "}\n"
         "}  // namespace\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_nindex_spec(IndexArgs a) {\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];\n"
         "  __shared__ prog::IndexTileShared sm;\n"
         "  prog::index_spec_tile(a, NP{}, lds, sm);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_nindex_emit(IndexArgs a) {\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];\n"
         "  __shared__ prog::IndexTileShared sm;\n"
         "  prog::index_emit_kernel_body(a, NP{}, lds, sm);\n"
         "}\n";
    return o.str();
  }
  if (group == JIT_NESTED) {
    // a recursive schema's unrolled writer defers the records nesting past
    // its levels to the general writer's deep pass (nested_size_tile)
    if (defer) o << "#define TGPU_NESTED_DEFER 1\n";
    o << "#include \"tgpu_nested.h\"\n"
         "namespace {\n"
         "using namespace tgpu;\n"
         "using namespace tgpu::prog;\n"
         "constexpr bool kCompact = "
      << (P.protocol == TGPU_PROTOCOL_BINARY ? "false" : "true")
      << ";\n"
         "template <class Src>\n"
         "__device__ __forceinline__ bool nrec(const Src& src, const Ctx& c, uint32_t& p, "
         "const uint32_t end, uint8_t* rec, uint64_t& bump) {\n"
         "  Win W;\n";
    gen_code(o, P, 0, P.n_ops, "rec", 2, false, "");
    o << "  return true;\n"
         "}\n"
         "struct NR {\n"
         "  template <class Src>\n"
         "  __device__ __forceinline__ bool operator()(const Src& src, const Ctx& c, uint32_t& p, "
         "uint32_t end, uint8_t* rec, uint64_t& bump) const {\n"
         "    return nrec(src, c, p, end, rec, bump);\n"
         "  }\n"
         "};\n"
         "}  // namespace\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_ndecode(DecodeArgs a, "
         "uint32_t wire_cap, uint64_t* __restrict__ irr, unsigned long long* __restrict__ nirr) {\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  nested_decode_tile(a, NR{}, kS, kCompact, wire_cap, irr, nirr, smem);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_ndecode_hbm(DecodeArgs a, "
         "uint32_t wire_cap, uint64_t* __restrict__ irr, unsigned long long* __restrict__ nirr) {\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  if (wire_cap) nested_decode_tile<false>(a, NR{}, kS, kCompact, wire_cap, irr, nirr, smem);\n"
         "  else nested_decode_hbm(a, NR{}, kS, kCompact, irr, nirr);\n"
         "}\n";
    o << "namespace {\n"
         "template <class O>\n"
         "__device__ __forceinline__ bool nenc(const uint8_t* rec, const uint8_t* sbase, "
         "const uint8_t* lbase, O& o) {\n";
    gen_code(o, P, 0, P.n_ops, "rec", 2, true, "");
    o << "  return true;\n"
         "}\n"
         "struct NE {\n"
         "  template <class O>\n"
         "  __device__ __forceinline__ bool operator()(const uint8_t* rec, const uint8_t* sbase, "
         "const uint8_t* lbase, O& o) const {\n"
         "    return nenc(rec, sbase, lbase, o);\n"
         "  }\n"
         "};\n"
         "}  // namespace\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_nsize(EncodeArgs a) {\n"
         "  __shared__ unsigned long long part[4];\n"
         "  nested_size_tile(a, NE{}, part);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_nwrite(EncodeArgs a) {\n"
         "  __shared__ unsigned long long part[4];\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  nested_write_tile(a, NE{}, part, smem, a.out_cap);\n"
         "}\n";
    return o.str();
  }
  if (group == JIT_DECODE)
    o << "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_decode(DecodeArgs a, "
         "uint32_t wire_cap, uint64_t* __restrict__ irr, unsigned long long* __restrict__ nirr) "
         "{\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
      << "  prog::decode_tile(a, JP{}, kS, wire_cap, irr, nirr, smem);\n"
         "}\n";
  // the same with records built in registers (no LDS record tile): the host
  // launches it when the record tile is what limits the workgroups per CU
  if (group == JIT_DECODE && decode_regrec(P.rec_size))
    o << "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_decode_rr(DecodeArgs a, "
         "uint32_t wire_cap, uint64_t* __restrict__ irr, unsigned long long* __restrict__ nirr) "
         "{\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  prog::decode_tile<JP, false, kS>(a, JP{}, kS, wire_cap, irr, nirr, smem);\n"
         "}\n";
  // the tolerant program's persistent strided-tail decode (stream-ordered
  // fixed-layout calls, DevResult tail_*): nothing to do — every workgroup
  // returns at once — unless a record was off the stride
  if (group == JIT_DECODE && tails)
    o << "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_decode_tail(DecodeArgs a, "
         "uint32_t wire_cap, uint64_t* __restrict__ irr, unsigned long long* __restrict__ nirr) "
         "{\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  const uint64_t L2 = a.res->tail_stride;\n"
         "  if (!L2) return;\n"
         "  prog::TailStride ts{a.res->tail_first, a.res->tail_pos, L2, 0};\n"
         "  const uint64_t tiles = (a.n - ts.first + prog::kPT - 1) / prog::kPT;\n"
         "  for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {\n"
         "    ts.r0 = ts.first + t * prog::kPT;\n"
         "    prog::decode_tile<JP, true>(a, JP{}, kS, wire_cap, irr, nirr, smem, ts);\n"
         "    __syncthreads();\n"
         "  }\n"
         "}\n";
  if (group == JIT_ENCODE)
    o << "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_size(EncodeArgs a) {\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  __shared__ unsigned long long part[4];\n"
         "  prog::size_tile(a, JP{}, kS, smem, part);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_write(EncodeArgs a) {\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  __shared__ prog::EncodeShared sm;\n"
         "  prog::write_tile<JP, kS>(a, JP{}, kS, smem, sm);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_write_one("
         "EncodeArgs a) {\n"
         "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
         "  __shared__ prog::EncodeShared sm;\n"
         "  prog::write_tile_one<JP, kS>(a, JP{}, smem, sm);\n"
         "}\n";
  if (group == JIT_INDEX)
    o << "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_index_spec(IndexArgs a) "
         "{\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];\n"
         "  __shared__ prog::IndexTileShared sm;\n"
         "  prog::index_spec_tile(a, JP{}, lds, sm);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_index_emit(IndexArgs a) "
         "{\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];\n"
         "  __shared__ prog::IndexTileShared sm;\n"
         "  prog::index_emit_kernel_body(a, JP{}, lds, sm);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_index_decode(IndexArgs a) "
         "{\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t rtile[prog::kRecTileBytes + 32];\n"
         "  __shared__ prog::IndexTileShared sm;\n"
         "  prog::index_emit_tile<true>(a, JP{}, lds, sm, rtile, blockIdx.x);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_index_onepass(IndexArgs a) "
         "{\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];\n"
         "  __shared__ prog::IndexTileShared sm;\n"
         "  __shared__ prog::OnePassShared op;\n"
         "  prog::index_onepass_tile<false>(a, JP{}, lds, sm, nullptr, op);\n"
         "}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void tgpu_jit_index_onepass_decode("
         "IndexArgs a) {\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t rtile[prog::kRecTileBytes + 32];\n"
         "  __shared__ prog::IndexTileShared sm;\n"
         "  __shared__ prog::OnePassShared op;\n"
         "  prog::index_onepass_tile<true>(a, JP{}, lds, sm, rtile, op);\n"
         "}\n";
  // the one pass over the candidate-list speculation, records decoded into
  // registers (config 5: each record parsed once; index_onepass_rr_tile)
  if (group == JIT_INDEX && decode_regrec(P.rec_size))
    o << "#ifndef TGPU_OP_WAVES\n#define TGPU_OP_WAVES 7\n#endif\n"
         "extern \"C\" __global__ __launch_bounds__(256) "
         "__attribute__((amdgpu_waves_per_eu(TGPU_OP_WAVES, 8))) void tgpu_jit_index_onepass_rr("
         "IndexArgs a) {\n"
         "  __shared__ __attribute__((aligned(16))) uint8_t lds[prog::kTileLds];\n"
         "  __shared__ prog::IndexTileShared sm;\n"
         "  __shared__ prog::OnePassShared op;\n"
         "  __shared__ prog::CandResult cr;\n"
         "  // (the chain's starts in the candidates' length array: the chain\n"
         "  // writes start k after reading every length it still needs)\n"
         "  prog::index_onepass_rr_tile<JP, kS>(a, JP{}, lds, sm, op, sm.cl.len, cr);\n"
         "}\n";
  return o.str();
}

// Generated source -> code object for `arch` (a gcnArchName; with its
// feature suffix first, then the bare processor name).
bool compile_src(const std::string& src, int group, std::string arch, std::vector<char>& code,
                 std::string& log) {
  if (const char* d = getenv("TGPU_JIT_DUMP")) {  // debugging: the generated unit
    const std::string path = std::string(d) + "." + std::to_string(group) + ".hip";
    if (FILE* f = fopen(path.c_str(), "w")) {
      fputs(src.c_str(), f);
      fclose(f);
    }
  }
  for (int attempt = 0; attempt < 2 && code.empty(); ++attempt) {
    if (attempt == 1) {
      const size_t c = arch.find(':');
      if (c == std::string::npos) break;
      arch = arch.substr(0, c);
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "tgpu_schema.hip", jit_src::kCount,
                            jit_src::kTexts, jit_src::kNames) != HIPRTC_SUCCESS) {
      log = "hiprtcCreateProgram failed";
      return false;
    }
    const std::string a = "--offload-arch=" + arch;
    const char* opts[] = {a.c_str(), "-O3", "-std=c++20"};
    const hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    if (ls > 1) {
      std::string l(ls, '\0');
      hiprtcGetProgramLog(prog, &l[0]);
      log += l;
    }
    if (r == HIPRTC_SUCCESS) {
      size_t cs = 0;
      hiprtcGetCodeSize(prog, &cs);
      code.resize(cs);
      hiprtcGetCode(prog, code.data());
      if (const char* d = getenv("TGPU_JIT_DUMP")) {  // debugging: the code object
        const std::string path = std::string(d) + "." + std::to_string(group) + ".co";
        if (FILE* f = fopen(path.c_str(), "wb")) {
          fwrite(code.data(), 1, code.size(), f);
          fclose(f);
        }
      }
    }
    hiprtcDestroyProgram(&prog);
  }
  return !code.empty();
}

bool compile_code(const VProgram& P, int group, std::string arch, std::vector<char>& code,
                  std::string& log) {
  return compile_src(gen_source(P, group), group, arch, code, log);
}

bool compile_from(const std::string& src, int device, int group, JitKernels& J) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    J.log = "hipGetDeviceProperties failed";
    return false;
  }
  std::vector<char> code;
  if (!compile_src(src, group, prop.gcnArchName, code, J.log)) return false;
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (prev != device) (void)hipSetDevice(device);
  bool ok = hipModuleLoadData(&J.mod, code.data()) == hipSuccess;
  for (int k = 0; k < 6 && ok; ++k) {
    if (!kEntry[group][k]) continue;
    ok = hipModuleGetFunction(&J.f[k], J.mod, kEntry[group][k]) == hipSuccess;
    // (tolerant programs / small records; a deferring nested program's
    // writer; the register-record one pass)
    if (!ok && ((group == JIT_DECODE && (k == 1 || k == 2)) ||
                (group == JIT_INDEX && k == 5) ||
                (group == JIT_NESTED && (k == 2 || k == 3)) ||
                (group == JIT_XCODE && (k == 2 || k == 3 || k == 5)))) {
      (void)hipGetLastError();
      J.f[k] = nullptr;
      ok = true;
    }
  }
  if (prev != device) (void)hipSetDevice(prev);
  if (!ok) J.log += "\nmodule load failed";
  return ok;
}

bool compile(const VProgram& P, int device, int group, JitKernels& J) {
  return compile_from(gen_source(P, group), device, group, J);
}

hipError_t launch(hipFunction_t f, uint64_t grid, uint32_t lds, hipStream_t s, void** params) {
  if (grid == 0) return hipSuccess;
  return hipModuleLaunchKernel(f, (uint32_t)grid, 1, 1, 256, 1, 1, lds, s, params, nullptr);
}

}  // namespace

const JitKernels* jit_kernels(const VProgram& P, int device, int group, uint64_t records,
                              uint64_t bytes, bool force) {
  const int mode = jit_mode();
  if (mode == 0) return nullptr;
  const bool want = force || mode == 1 || records >= kAutoRecords || bytes >= kAutoBytes;
  const std::string key = cache_key(P, device, group);
  std::lock_guard<std::mutex> g(g_mu);
  auto it = cache().find(key);
  if (it != cache().end()) return it->second->ok ? it->second : nullptr;
  if (!want) return nullptr;
  JitKernels* J = new JitKernels();
  J->ok = compile(P, device, group, *J);
  if (!J->ok && getenv("TGPU_JIT_VERBOSE"))
    fprintf(stderr, "tgpu: schema kernels not compiled, using the interpreter:\n%s\n",
            J->log.c_str());
  cache()[key] = J;  // a failure is remembered too: never retried
  return J->ok ? J : nullptr;
}

const JitKernels* jit_kernels_xcode(const VProgram& Ps, const VProgram& Pd, int device,
                                    uint64_t records, bool force) {
  const int mode = jit_mode();
  if (mode == 0) return nullptr;
  const bool want = force || mode == 1 || records >= kAutoRecords;
  const std::string key = cache_key(Ps, device, JIT_XCODE) + "|" + cache_key(Pd, device, JIT_XCODE);
  std::lock_guard<std::mutex> g(g_mu);
  auto it = cache().find(key);
  if (it != cache().end()) return it->second->ok ? it->second : nullptr;
  if (!want) return nullptr;
  JitKernels* J = new JitKernels();
  J->ok = compile_from(gen_source_xcode(Ps, Pd), device, JIT_XCODE, *J);
  if (!J->ok && getenv("TGPU_JIT_VERBOSE"))
    fprintf(stderr, "tgpu: transcoding kernels not compiled, using the interpreter:\n%s\n",
            J->log.c_str());
  cache()[key] = J;
  return J->ok ? J : nullptr;
}

hipError_t jit_launch_xcode(const JitKernels* J, int which, const XcodeArgs& x, uint64_t grid,
                            uint32_t cap, uint32_t ocap, uint32_t lds, hipStream_t s) {
  if (!jit_has(J, which)) return hipErrorInvalidDeviceFunction;
  XcodeArgs a = x;
  void* p2[] = {&a, &cap};
  void* p3[] = {&a, &cap, &ocap};
  return launch(J->f[which], grid, lds, s, (which & 1) || which >= 4 ? p3 : p2);
}

int jit_compile_check_xcode(const VProgram& Ps, const VProgram& Pd, const char* arch, char* log,
                            uint64_t log_cap) {
  std::string l;
  bool ok;
  if (arch && !*arch) {
    ok = !gen_source_xcode(Ps, Pd).empty();
  } else {
    std::vector<char> code;
    ok = compile_src(gen_source_xcode(Ps, Pd), JIT_XCODE, arch ? arch : "gfx950", code, l);
  }
  if (log && log_cap) {
    const size_t n = l.size() < log_cap - 1 ? l.size() : (size_t)(log_cap - 1);
    memcpy(log, l.data(), n);
    log[n] = 0;
  }
  return ok ? TGPU_OK : TGPU_ERR_UNSUPPORTED;
}

bool decode_regrec(uint32_t rec_size) {
  return rec_size && rec_size <= 128 && rec_size % 8 == 0;
}

bool jit_has(const JitKernels* J, int which) { return J && which >= 0 && which < 6 && J->f[which]; }

hipError_t jit_launch_decode(const JitKernels* J, const DecodeArgs& a, uint64_t grid,
                             uint32_t cap, uint32_t lds, uint64_t* irr, unsigned long long* nirr,
                             hipStream_t s, int which) {
  if (!jit_has(J, which)) return hipErrorInvalidDeviceFunction;
  DecodeArgs x = a;
  void* p[] = {&x, &cap, &irr, &nirr};
  return launch(J->f[which], grid, lds, s, p);
}

hipError_t jit_launch_encode(const JitKernels* J, bool write, const EncodeArgs& a, uint64_t grid,
                             uint32_t lds, hipStream_t s, int first) {
  if (!jit_has(J, first + (write ? 1 : 0))) return hipErrorInvalidDeviceFunction;
  EncodeArgs x = a;
  void* p[] = {&x};
  return launch(J->f[first + (write ? 1 : 0)], grid, lds, s, p);
}

hipError_t jit_launch_index(const JitKernels* J, int which, const IndexArgs& a, uint64_t grid,
                            hipStream_t s) {
  IndexArgs x = a;
  void* p[] = {&x};
  return launch(J->f[which], grid, 0, s, p);
}

// Compile-only check of one program (no device needed): source generation
// and hipRTC for `arch`; the log (truncated to log_cap) on failure.
int jit_compile_check(const VProgram& P, const char* arch, char* log, uint64_t log_cap,
                      int only_group) {
  std::string l;
  bool ok = true;
  bool nested = false;
  for (uint32_t k = 0; k < P.n_ops; ++k)
    nested |= P.ops[k].kind >= VOP_SEQ;
  for (int group = nested ? JIT_NESTED : 0; group < (nested ? JIT_NINDEX + 1 : JIT_NESTED) && ok;
       ++group) {
    if (only_group >= 0 && group != only_group) continue;
    if (arch && !*arch) {  // generation only
      ok = !gen_source(P, group).empty();
      continue;
    }
    std::vector<char> code;
    ok = compile_code(P, group, arch ? arch : "gfx950", code, l);
  }
  if (log && log_cap) {
    const size_t n = l.size() < log_cap - 1 ? l.size() : (size_t)(log_cap - 1);
    memcpy(log, l.data(), n);
    log[n] = 0;
  }
  return ok ? TGPU_OK : TGPU_ERR_UNSUPPORTED;
}

}  // namespace tgpu
