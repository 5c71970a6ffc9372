/*
 * murr_oracle.h — CPU restatement of murr's row-blob codec (TEST INFRASTRUCTURE).
 *
 * This is the parity oracle and the CPU baseline ("port"), nothing else.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker.  The product path (libmurr_codec.so) never links it.
 *
 * Restated from murrdb/murr v0.2.1 (which cannot be built here: no Rust
 * toolchain), structurally faithful: a serial per-row loop with per-column
 * dispatch into append-style builders, as in src/io/row/read.rs:85-98 and
 * src/io/table/mod.rs:97-109.  Third-party semantics restated: arrow-rs 58.3.0
 * builders (PrimitiveBuilder / BooleanBuilder / StringBuilder /
 * NullBufferBuilder) and Rust core::str::from_utf8 (Unicode Table 3-7).
 * Pinned by the reference's own known-answer tests, restated as fixtures under
 * tests/golden/ (see tests/golden/make_golden.py).
 */
#ifndef MURR_ORACLE_H
#define MURR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    OC_UTF8 = 0, OC_BOOL, OC_INT8, OC_INT16, OC_INT32, OC_INT64,
    OC_UINT8, OC_UINT16, OC_UINT32, OC_UINT64, OC_FLOAT32, OC_FLOAT64
};

enum {
    OC_OK = 0, OC_E_INVALID_UTF8 = 1, OC_E_DTYPE = 2, OC_E_BAD_COLUMN = 3,
    OC_E_OFFSET_OVERFLOW = 4, OC_E_MALFORMED_ROW = 5, OC_E_ARGUMENT = 7,
    OC_E_NULL_KEY = 8, OC_E_ARROW = 11
};

typedef struct { uint32_t index, dtype, offset, size; } oc_column;
typedef struct {
    uint32_t ncols, bitset_size, capacity, _pad;
    const oc_column* cols;
} oc_segment;

/* Arrow array produced by a builder's finish() (owned; free with oc_array_free). */
typedef struct {
    uint8_t* values;
    uint8_t* validity;   /* NULL when no nulls */
    int32_t* offsets;    /* utf8 only */
    uint64_t length;
    uint64_t null_count;
    uint64_t values_len;
    uint32_t dtype;
    uint32_t _pad;
} oc_array;

/* Arrow input column (host). */
typedef struct {
    const void*    values;
    const uint8_t* validity;
    const int32_t* offsets;
    uint64_t       offset;
} oc_col_in;

typedef struct {
    int32_t  status;
    int32_t  _pad;
    uint64_t row;
    uint32_t column;
    uint32_t _pad2;
    char     message[128];
} oc_error;

int  oc_dtype_size(uint32_t dtype);
int  oc_segment_init(const uint32_t* dtypes, uint32_t n, oc_column* cols, oc_segment* seg);

/* WriteRow (src/io/row/write.rs:4-52). */
typedef struct { const oc_segment* schema; uint8_t* bytes; uint64_t len, cap; } oc_write_row;
void oc_write_row_new(oc_write_row* w, const oc_segment* s);
void oc_write_row_set_non_null(oc_write_row* w, const oc_column* c);
void oc_write_row_write_static(oc_write_row* w, const oc_column* c, const void* v, uint32_t size);
void oc_write_row_write_dynamic(oc_write_row* w, const oc_column* c, const uint8_t* v, uint64_t len);
void oc_write_row_free(oc_write_row* w);

/* ReadBatchBuilder (src/io/row/read.rs:62-110). */
typedef struct oc_builder oc_builder;
oc_builder* oc_builder_new(const oc_segment* seg, const uint32_t* proj, uint32_t nproj,
                           uint64_t capacity);
int  oc_builder_add_row(oc_builder* b, const uint8_t* bytes, uint64_t len, oc_error* err);
int  oc_builder_add_empty(oc_builder* b);
int  oc_builder_build(oc_builder* b, oc_array* outs /* nproj */, oc_error* err);
void oc_builder_free(oc_builder* b);

/* Store::read over one block of blobs (memory.rs:38-43): row i present iff
 * row_off[i+1] > row_off[i]. */
int  oc_decode_block(const oc_segment* seg, const uint32_t* proj, uint32_t nproj,
                     const uint8_t* data, const uint64_t* row_off, uint64_t n,
                     oc_array* outs, oc_error* err);

/* Table::write loop (src/io/table/mod.rs:97-109) without the store: blobs back
 * to back + row_off[n+1].  *blob is malloc'ed (free with oc_free). */
int  oc_encode_batch(const oc_segment* seg, const oc_col_in* cols, uint64_t n,
                     uint8_t** blob, uint64_t* blob_len, uint64_t* row_off, oc_error* err);

/* MemoryStore (src/io/store/memory.rs): a key -> row blob map over n keys
 * (Arrow utf8: key_data, key_off[n+1]) and their blobs (blob, row_off[n+1]);
 * a key given twice maps to its later row (HashMap::insert, memory.rs:55-57).
 * The map is FNV-1a open addressing in place of Rust's SipHash HashMap: the
 * same lookup semantics, a different hash.  The pointers are kept, not
 * copied. */
typedef struct oc_memstore oc_memstore;
oc_memstore* oc_memstore_new(const uint8_t* key_data, const int32_t* key_off, uint64_t n,
                             const uint8_t* blob, const uint64_t* row_off);
/* Store::read (memory.rs:28-45): per key add_row of its blob or add_empty,
 * then build() -> outs[nproj] (owned, oc_array_free). */
int  oc_memstore_read(const oc_memstore* m, const oc_segment* seg, const uint32_t* proj, uint32_t nproj,
                      const uint8_t* q_data, const int32_t* q_off, uint64_t nq, oc_array* outs,
                      oc_error* err);
void oc_memstore_free(oc_memstore* m);
/* core::str::from_utf8: 1 valid, 0 invalid (valid_up_to / error_len like Utf8Error). */
int  oc_utf8_valid(const uint8_t* s, uint64_t len, uint64_t* valid_up_to, int* error_len);

void oc_array_free(oc_array* a);
void oc_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
