/*
 * thrift_oracle.h — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A CPU restatement of fbthrift's Binary and Compact protocol semantics for
 * the bulk record path. It is never linked into, loaded by, or called from the
 * product library (fbthrift_amd/lib/libtgpu.so). Only tests/, the smoke check
 * in __graft_entry__.py and bench.py's cpu_baseline leg may use it.
 *
 * Parity pinning: the restatement is checked against golden vectors produced
 * by the reference's own pure-Python protocols (thrift/lib/py/protocol/
 * TBinaryProtocol.py, TCompactProtocol.py) — see tests/golden/make_golden.py —
 * and against the semantic pins of the reference's C++ tests restated in
 * tests/test_oracle_semantics.py (VarintUtilsTest, BinaryProtocolTest,
 * ProtocolTruncatedDataTest, CompactProtocolTest, ProtocolSkipTest).
 *
 * Descriptor and status types are shared with include/thrift_gpu.h so the
 * oracle and the device path can be compared byte for byte.
 */
#ifndef THRIFT_ORACLE_H_
#define THRIFT_ORACLE_H_

#include "../include/thrift_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Table-driven encode of n records (same layout/span rules as the C-ABI). */
int oracle_encode_batch_ex(const tgpu_struct_desc* structs, uint32_t n_structs,
                           const tgpu_field_desc* fields, uint32_t n_fields,
                           const tgpu_type_desc* types, uint32_t n_types, int protocol,
                           const void* records, uint64_t n_records, const void* string_base,
                           const void* list_base, void* out, uint64_t out_capacity,
                           uint64_t* out_offsets, tgpu_status* st, uint64_t* out_size);
int oracle_decode_batch_ex(const tgpu_struct_desc* structs, uint32_t n_structs,
                           const tgpu_field_desc* fields, uint32_t n_fields,
                           const tgpu_type_desc* types, uint32_t n_types, int protocol,
                           const void* in, uint64_t in_len, const uint64_t* offsets,
                           uint64_t n_records, void* records, void* list_arena,
                           uint64_t list_arena_capacity, const tgpu_limits* limits,
                           tgpu_status* st, uint64_t* n_decoded, uint64_t* consumed);
uint32_t oracle_arena_scale(const tgpu_struct_desc* structs, uint32_t n_structs,
                            const tgpu_field_desc* fields, uint32_t n_fields,
                            const tgpu_type_desc* types, uint32_t n_types, int protocol);
int oracle_encode_batch(const tgpu_struct_desc* structs, uint32_t n_structs,
                        const tgpu_field_desc* fields, uint32_t n_fields,
                        int protocol, const void* records, uint64_t n_records,
                        const void* string_base, const void* list_base,
                        void* out, uint64_t out_capacity, uint64_t* out_offsets,
                        tgpu_status* st, uint64_t* out_size);

/* Table-driven decode (repeated deserialize<T>(Cursor&) semantics). */
int oracle_decode_batch(const tgpu_struct_desc* structs, uint32_t n_structs,
                        const tgpu_field_desc* fields, uint32_t n_fields,
                        int protocol, const void* in, uint64_t in_len,
                        const uint64_t* offsets, uint64_t n_records,
                        void* records, void* list_arena,
                        uint64_t list_arena_capacity, const tgpu_limits* limits,
                        tgpu_status* st, uint64_t* n_decoded,
                        uint64_t* consumed);

/* Byte length of the record starting at in[pos] (reader.skip(T_STRUCT) with
 * reader.setHeight(height), height 0 = max_depth), or -(code) on error. */
int64_t oracle_record_length(int protocol, const void* in, uint64_t in_len,
                             uint64_t pos, int32_t max_depth, int32_t height);

/* reader.skip(ttype) at in[pos] (the protocol's own skip): bytes consumed or
 * -(code). */
int64_t oracle_skip_value(int protocol, const void* in, uint64_t in_len,
                          uint64_t pos, int ttype, int32_t max_depth,
                          int32_t height);

/* Schemaless skim (tgpu_skim_batch semantics): per record the top-level
 * fields as (id, wire type, bool flags, value offset, value length). */
int oracle_skim_batch(int protocol, const void* in, uint64_t in_len,
                      const uint64_t* offsets, uint64_t n_records,
                      tgpu_skim_field* fields, uint32_t max_fields,
                      uint32_t* field_counts, const tgpu_limits* limits,
                      tgpu_status* st, uint64_t* n_done);
/* The same descending into struct-valued fields up to max_nest levels
 * (tgpu_skim_batch_ex's pre-order entries; the recursion of parseObject). */
int oracle_skim_batch_ex(int protocol, const void* in, uint64_t in_len, const uint64_t* offsets,
                         uint64_t n_records, tgpu_skim_field* fields, uint32_t max_fields,
                         uint32_t* field_counts, uint32_t max_nest, const tgpu_limits* limits,
                         tgpu_status* st, uint64_t* n_done);

/* Varint / zigzag primitives (VarintUtils-inl.h restated) for unit tests. */
int oracle_read_varint(const void* in, uint64_t len, int bits,
                       uint64_t* value, uint64_t* consumed);
int oracle_write_varint(uint64_t value, void* out);

/* ---- codegen-equivalent paths (CPU baseline; cores = n_threads) ------ */
/* Config 1/2 record {1..8: i64}: generated readNoXfer/write restated for
 * BinaryProtocolReader/Writer. Returns 0 or a tgpu_code. */
int oracle_flat8_binary_decode(const void* in, uint64_t n_records,
                               void* records, int n_threads);
int oracle_flat8_binary_encode(const void* records, uint64_t n_records,
                               void* out, int n_threads);
/* Config 3 record {1..4: i32, 5..6: string}, Compact, with record index. */
int oracle_mixed_compact_decode(const void* in, const uint64_t* offsets,
                                uint64_t n_records, void* records,
                                int n_threads);
int oracle_mixed_compact_encode(const void* records, uint64_t n_records,
                                const void* string_base, void* out,
                                const uint64_t* offsets, int n_threads);
int oracle_mixed_compact_size(const void* records, uint64_t n_records, uint64_t* sizes,
                              int n_threads);
uint64_t oracle_mixed_compact_read_file(const void* in, uint64_t in_len, uint64_t max_records,
                                        void* records, uint64_t* offsets);
int oracle_nested_binary_size(const void* records, uint64_t n_records, uint64_t* sizes,
                              int n_threads);
int oracle_nested_binary_encode(const void* records, uint64_t n_records, const void* list_base,
                                void* out, const uint64_t* offsets, int n_threads);
int oracle_nested_binary_decode(const void* in, const uint64_t* offsets, uint64_t n_records,
                                void* records, void* arena, int n_threads);

/* ---- deterministic generators (shared spec with tests/golden) -------- */
uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t index);
/* Config 1/2 records (72-byte layout). */
void oracle_gen_flat8(uint64_t seed, uint64_t first, uint64_t n, void* records);

#ifdef __cplusplus
}
#endif

#endif /* THRIFT_ORACLE_H_ */
