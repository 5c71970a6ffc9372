/*
 * murr_oracle.c — CPU restatement of murr's row-blob codec (TEST INFRASTRUCTURE,
 * see murr_oracle.h).  Each function cites the reference file:line it follows
 * (murrdb/murr v0.2.1).  Keep it boring: per-row loops, dynamic dispatch into
 * append-style builders, exactly the reference's control flow.
 */
#include "murr_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---- dtype table: DType::size / DTypeName (src/core/schema.rs:6-19,
 *      src/io/codec/<dtype>.rs `fn size`) ---------------------------------- */
int oc_dtype_size(uint32_t dtype) {
    switch (dtype) {
    case OC_UTF8: return 4;                 /* utf8.rs:27-29 */
    case OC_BOOL: return 1;                 /* bool_.rs:27-29 */
    case OC_INT8: case OC_UINT8: return 1;  /* int8.rs:24-25, uint8.rs */
    case OC_INT16: case OC_UINT16: return 2;
    case OC_INT32: case OC_UINT32: case OC_FLOAT32: return 4;  /* float32.rs:17-26 */
    case OC_INT64: case OC_UINT64: case OC_FLOAT64: return 8;
    default: return -1;
    }
}

/* From<&TableSchema> for SegmentSchema (src/io/schema.rs:33-54) + SegmentSchema::new
 * (schema.rs:23-30): index = position among non-key columns, offset = running
 * sum of sizes, capacity = sum, bitset_size = ceil(n/8). */
int oc_segment_init(const uint32_t* dtypes, uint32_t n, oc_column* cols, oc_segment* seg) {
    uint32_t off = 0;
    for (uint32_t i = 0; i < n; i++) {
        int sz = oc_dtype_size(dtypes[i]);
        if (sz < 0) return OC_E_DTYPE;
        cols[i].index = i;
        cols[i].dtype = dtypes[i];
        cols[i].offset = off;
        cols[i].size = (uint32_t)sz;
        off += (uint32_t)sz;
    }
    seg->ncols = n;
    seg->bitset_size = (n + 7) / 8;
    seg->capacity = off;
    seg->_pad = 0;
    seg->cols = cols;
    return OC_OK;
}

/* ---- growable byte buffer (arrow-rs MutableBuffer / Vec<u8>) ------------- */
typedef struct { uint8_t* p; uint64_t len, cap; } vbuf;

static void vb_reserve(vbuf* b, uint64_t extra) {
    if (b->len + extra <= b->cap) return;
    uint64_t nc = b->cap ? b->cap : 64;
    while (nc < b->len + extra) nc *= 2;
    b->p = (uint8_t*)realloc(b->p, nc);
    if (!b->p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    b->cap = nc;
}
static void vb_push(vbuf* b, const void* src, uint64_t n) {
    vb_reserve(b, n);
    if (n) memcpy(b->p + b->len, src, n);
    b->len += n;
}
static void vb_zeros(vbuf* b, uint64_t n) {
    vb_reserve(b, n);
    memset(b->p + b->len, 0, n);
    b->len += n;
}

/* ---- WriteRow (src/io/row/write.rs) -------------------------------------- */

/* write.rs:20-28: zeroed bs+capacity bytes, bitset filled with 0xFF. */
void oc_write_row_new(oc_write_row* w, const oc_segment* s) {
    w->schema = s;
    w->len = (uint64_t)s->bitset_size + s->capacity;
    w->cap = w->len + 64;
    w->bytes = (uint8_t*)calloc(w->cap, 1);
    memset(w->bytes, 0xFF, s->bitset_size);
}

static void wr_grow(oc_write_row* w, uint64_t extra) {
    if (w->len + extra <= w->cap) return;
    uint64_t nc = w->cap * 2;
    while (nc < w->len + extra) nc *= 2;
    w->bytes = (uint8_t*)realloc(w->bytes, nc);
    w->cap = nc;
}

/* write.rs:30-35: clear bit index%8 of byte index/8. */
void oc_write_row_set_non_null(oc_write_row* w, const oc_column* c) {
    w->bytes[c->index / 8] &= (uint8_t)~(1u << (c->index % 8));
}

/* write.rs:37-42: set non-null, copy native LE bytes at bs+offset. */
void oc_write_row_write_static(oc_write_row* w, const oc_column* c, const void* v, uint32_t size) {
    oc_write_row_set_non_null(w, c);
    memcpy(w->bytes + w->schema->bitset_size + c->offset, v, size);
}

/* write.rs:44-52: slot <- u32 (len(bytes) - bs); append u32 len, then bytes. */
void oc_write_row_write_dynamic(oc_write_row* w, const oc_column* c, const uint8_t* v, uint64_t len) {
    oc_write_row_set_non_null(w, c);
    uint32_t payload_rel = (uint32_t)(w->len - w->schema->bitset_size);
    memcpy(w->bytes + w->schema->bitset_size + c->offset, &payload_rel, 4);
    wr_grow(w, 4 + len);
    uint32_t l32 = (uint32_t)len;
    memcpy(w->bytes + w->len, &l32, 4);
    w->len += 4;
    if (len) memcpy(w->bytes + w->len, v, len);
    w->len += len;
}

void oc_write_row_free(oc_write_row* w) { free(w->bytes); w->bytes = NULL; }

/* ---- ReadRow (src/io/row/read.rs:16-56) ---------------------------------- */
typedef struct {
    const oc_segment* schema;
    const uint8_t* bitset;
    const uint8_t* values;
    uint64_t values_len;
} rrow;

/* read.rs:23-30: split_at(bitset_size).  The reference panics when the slice
 * is shorter; the restatement reports MALFORMED instead. */
static int rrow_new(rrow* r, const oc_segment* s, const uint8_t* raw, uint64_t len) {
    if (len < s->bitset_size) return OC_E_MALFORMED_ROW;
    r->schema = s;
    r->bitset = raw;
    r->values = raw + s->bitset_size;
    r->values_len = len - s->bitset_size;
    return OC_OK;
}

/* read.rs:32-37 */
static int rrow_is_null(const rrow* r, const oc_column* c) {
    return (r->bitset[c->index / 8] >> (c->index % 8)) & 1;
}

/* read.rs:39-43: pod_read_unaligned of size bytes at values[offset..]. */
static int rrow_read_static(const rrow* r, const oc_column* c, void* out, uint32_t size) {
    if ((uint64_t)c->offset + size > r->values_len) return OC_E_MALFORMED_ROW;
    memcpy(out, r->values + c->offset, size);
    return OC_OK;
}

/* read.rs:45-55: p = u32 slot; len = u32 at values[p]; bytes values[p+4..p+4+len]. */
static int rrow_read_dynamic(const rrow* r, const oc_column* c, const uint8_t** out, uint64_t* olen) {
    uint32_t p, l;
    if ((uint64_t)c->offset + 4 > r->values_len) return OC_E_MALFORMED_ROW;
    memcpy(&p, r->values + c->offset, 4);
    if ((uint64_t)p + 4 > r->values_len) return OC_E_MALFORMED_ROW;
    memcpy(&l, r->values + p, 4);
    if ((uint64_t)p + 4 + l > r->values_len) return OC_E_MALFORMED_ROW;
    *out = r->values + p + 4;
    *olen = l;
    return OC_OK;
}

/* ---- core::str::from_utf8 (Rust core, run_utf8_validation; Unicode 3-7) --- */
static int utf8_char_width(uint8_t b) {
    if (b < 0x80) return 1;
    if (b >= 0xC2 && b <= 0xDF) return 2;
    if (b >= 0xE0 && b <= 0xEF) return 3;
    if (b >= 0xF0 && b <= 0xF4) return 4;
    return 0;
}

int oc_utf8_valid(const uint8_t* v, uint64_t len, uint64_t* valid_up_to, int* error_len) {
    uint64_t i = 0;
#define OC_ERR(el) do { if (valid_up_to) *valid_up_to = old; if (error_len) *error_len = (el); return 0; } while (0)
#define OC_NEXT() (++i >= len ? -1 : (int)v[i])
    while (i < len) {
        uint64_t old = i;
        uint8_t first = v[i];
        if (first >= 128) {
            int w = utf8_char_width(first), b;
            if (w == 2) {
                if ((b = OC_NEXT()) < 0) OC_ERR(0);
                if ((b & 0xC0) != 0x80) OC_ERR(1);
            } else if (w == 3) {
                if ((b = OC_NEXT()) < 0) OC_ERR(0);
                int ok = (first == 0xE0 && b >= 0xA0 && b <= 0xBF) ||
                         (first >= 0xE1 && first <= 0xEC && b >= 0x80 && b <= 0xBF) ||
                         (first == 0xED && b >= 0x80 && b <= 0x9F) ||
                         (first >= 0xEE && first <= 0xEF && b >= 0x80 && b <= 0xBF);
                if (!ok) OC_ERR(1);
                if ((b = OC_NEXT()) < 0) OC_ERR(0);
                if ((b & 0xC0) != 0x80) OC_ERR(2);
            } else if (w == 4) {
                if ((b = OC_NEXT()) < 0) OC_ERR(0);
                int ok = (first == 0xF0 && b >= 0x90 && b <= 0xBF) ||
                         (first >= 0xF1 && first <= 0xF3 && b >= 0x80 && b <= 0xBF) ||
                         (first == 0xF4 && b >= 0x80 && b <= 0x8F);
                if (!ok) OC_ERR(1);
                if ((b = OC_NEXT()) < 0) OC_ERR(0);
                if ((b & 0xC0) != 0x80) OC_ERR(2);
                if ((b = OC_NEXT()) < 0) OC_ERR(0);
                if ((b & 0xC0) != 0x80) OC_ERR(3);
            } else {
                OC_ERR(1);
            }
        }
        i++;
    }
#undef OC_ERR
#undef OC_NEXT
    return 1;
}

/* ---- arrow-rs 58 NullBufferBuilder: materialised lazily at the first null,
 *      previous slots set valid; finish() -> None when never materialised ---- */
typedef struct { vbuf bits; uint64_t len; uint64_t nulls; int materialized; } nullbuf;

static void bit_append(vbuf* b, uint64_t idx, int v) {
    if (idx % 8 == 0) vb_zeros(b, 1);
    if (v) b->p[idx / 8] |= (uint8_t)(1u << (idx % 8));
}
static void nb_append(nullbuf* nb, int valid) {
    if (!valid && !nb->materialized) {
        nb->materialized = 1;
        for (uint64_t i = 0; i < nb->len; i++) bit_append(&nb->bits, i, 1);
    }
    if (nb->materialized) bit_append(&nb->bits, nb->len, valid);
    if (!valid) nb->nulls++;
    nb->len++;
}

/* ---- ColumnEncoder trait (src/io/codec/mod.rs:43-47) as a C vtable -------- */
typedef struct encoder encoder;
struct encoder {
    int  (*add_row)(encoder*, const rrow*, oc_error*);
    void (*add_empty)(encoder*);
    void (*build)(encoder*, oc_array*);
    oc_column col;
    vbuf values;     /* primitive values / bool bits / utf8 bytes */
    vbuf offsets;    /* utf8 i32 offsets */
    uint64_t len;
    nullbuf nulls;
};

/* primitive::Encoder<T> (src/io/codec/primitive.rs:38-61).  append_null on a
 * PrimitiveBuilder advances the values buffer with a zeroed slot. */
static int prim_add_row(encoder* e, const rrow* r, oc_error* err) {
    (void)err;
    if (rrow_is_null(r, &e->col)) {
        vb_zeros(&e->values, e->col.size);
        nb_append(&e->nulls, 0);
    } else {
        uint8_t tmp[8];
        int st = rrow_read_static(r, &e->col, tmp, e->col.size);
        if (st) return st;
        vb_push(&e->values, tmp, e->col.size);
        nb_append(&e->nulls, 1);
    }
    e->len++;
    return OC_OK;
}
static void prim_add_empty(encoder* e) {          /* primitive.rs:53-56 */
    vb_zeros(&e->values, e->col.size);
    nb_append(&e->nulls, 0);
    e->len++;
}

/* BoolEncoder (src/io/codec/bool_.rs:85-104): read_static::<u8>() != 0. */
static int bool_add_row(encoder* e, const rrow* r, oc_error* err) {
    (void)err;
    if (rrow_is_null(r, &e->col)) {
        bit_append(&e->values, e->len, 0);
        nb_append(&e->nulls, 0);
    } else {
        uint8_t b;
        int st = rrow_read_static(r, &e->col, &b, 1);
        if (st) return st;
        bit_append(&e->values, e->len, b != 0);
        nb_append(&e->nulls, 1);
    }
    e->len++;
    return OC_OK;
}
static void bool_add_empty(encoder* e) {          /* bool_.rs:96-99 */
    bit_append(&e->values, e->len, 0);
    nb_append(&e->nulls, 0);
    e->len++;
}

/* Utf8Encoder (src/io/codec/utf8.rs:85-105): read_dynamic -> from_utf8 ->
 * append_value; StringBuilder pushes the running byte length as i32 offset
 * and panics ("byte array offset overflow") past i32::MAX. */
static int utf8_push_offset(encoder* e) {
    if (e->values.len > 0x7FFFFFFFull) return OC_E_OFFSET_OVERFLOW;
    int32_t o = (int32_t)e->values.len;
    vb_push(&e->offsets, &o, 4);
    return OC_OK;
}
static int utf8_add_row(encoder* e, const rrow* r, oc_error* err) {
    if (rrow_is_null(r, &e->col)) {
        nb_append(&e->nulls, 0);
    } else {
        const uint8_t* s; uint64_t l;
        int st = rrow_read_dynamic(r, &e->col, &s, &l);
        if (st) return st;
        uint64_t vut; int el;
        if (!oc_utf8_valid(s, l, &vut, &el)) {
            if (err) {
                if (el) snprintf(err->message, sizeof err->message,
                                 "invalid utf8: invalid utf-8 sequence of %d bytes from index %llu",
                                 el, (unsigned long long)vut);
                else snprintf(err->message, sizeof err->message,
                              "invalid utf8: incomplete utf-8 byte sequence from index %llu",
                              (unsigned long long)vut);
            }
            return OC_E_INVALID_UTF8;
        }
        vb_push(&e->values, s, l);
        nb_append(&e->nulls, 1);
    }
    e->len++;
    return utf8_push_offset(e);
}
static void utf8_add_empty(encoder* e) {           /* utf8.rs:98-101 */
    nb_append(&e->nulls, 0);
    e->len++;
    (void)utf8_push_offset(e);
}

/* finish(): hand the buffers over as an Arrow array. */
static void enc_build(encoder* e, oc_array* a) {
    memset(a, 0, sizeof *a);
    a->dtype = e->col.dtype;
    a->length = e->len;
    a->null_count = e->nulls.nulls;
    a->values_len = e->values.len;
    a->values = e->values.p ? e->values.p : (uint8_t*)calloc(1, 1);
    e->values.p = NULL;
    if (e->nulls.materialized) {
        a->validity = e->nulls.bits.p ? e->nulls.bits.p : (uint8_t*)calloc(1, 1);
        e->nulls.bits.p = NULL;
    }
    if (e->col.dtype == OC_UTF8) {
        a->offsets = (int32_t*)e->offsets.p;
        e->offsets.p = NULL;
    }
}

/* ArrowCodec::make_encoder via DTypeName::codec() (src/io/codec/mod.rs:59-76). */
static encoder* make_encoder(const oc_column* c, uint64_t rows) {
    encoder* e = (encoder*)calloc(1, sizeof *e);
    e->col = *c;
    e->build = enc_build;
    if (c->dtype == OC_UTF8) {
        e->add_row = utf8_add_row; e->add_empty = utf8_add_empty;
        vb_reserve(&e->values, rows * 16);      /* utf8.rs:36 with_capacity(rows, rows*16) */
        vb_reserve(&e->offsets, (rows + 1) * 4);
        int32_t z = 0;
        vb_push(&e->offsets, &z, 4);
    } else if (c->dtype == OC_BOOL) {
        e->add_row = bool_add_row; e->add_empty = bool_add_empty;
    } else {
        e->add_row = prim_add_row; e->add_empty = prim_add_empty;
        vb_reserve(&e->values, rows * c->size);  /* primitive.rs:30-35 with_capacity(rows) */
    }
    return e;
}

static void free_encoder(encoder* e) {
    free(e->values.p); free(e->offsets.p); free(e->nulls.bits.p); free(e);
}

/* ---- ReadBatchBuilder (src/io/row/read.rs:62-110) ------------------------ */
struct oc_builder {
    const oc_segment* seg;
    uint32_t nproj;
    encoder** enc;
};

/* read.rs:69-83: one encoder per requested column, request order. */
oc_builder* oc_builder_new(const oc_segment* seg, const uint32_t* proj, uint32_t nproj,
                           uint64_t capacity) {
    oc_builder* b = (oc_builder*)calloc(1, sizeof *b);
    b->seg = seg;
    b->nproj = nproj;
    b->enc = (encoder**)calloc(nproj ? nproj : 1, sizeof(encoder*));
    for (uint32_t p = 0; p < nproj; p++) b->enc[p] = make_encoder(&seg->cols[proj[p]], capacity);
    return b;
}

/* read.rs:85-91: ReadRow::new then every encoder's add_row, first error wins. */
int oc_builder_add_row(oc_builder* b, const uint8_t* bytes, uint64_t len, oc_error* err) {
    rrow r;
    int st = rrow_new(&r, b->seg, bytes, len);
    if (st) { if (err) { err->status = st; err->column = 0; } return st; }
    for (uint32_t p = 0; p < b->nproj; p++) {
        st = b->enc[p]->add_row(b->enc[p], &r, err);
        if (st) { if (err) { err->status = st; err->column = p; } return st; }
    }
    return OC_OK;
}

/* read.rs:93-98 */
int oc_builder_add_empty(oc_builder* b) {
    for (uint32_t p = 0; p < b->nproj; p++) b->enc[p]->add_empty(b->enc[p]);
    return OC_OK;
}

/* read.rs:100-109: build every encoder; RecordBatch::try_new rejects zero columns. */
int oc_builder_build(oc_builder* b, oc_array* outs, oc_error* err) {
    if (b->nproj == 0) {
        if (err) { err->status = OC_E_ARROW; snprintf(err->message, sizeof err->message,
                   "Arrow error: must either specify a row count or at least one column"); }
        return OC_E_ARROW;
    }
    for (uint32_t p = 0; p < b->nproj; p++) {
        if (b->enc[p]->col.dtype == OC_UTF8 && b->enc[p]->values.len > 0x7FFFFFFFull) {
            if (err) err->status = OC_E_OFFSET_OVERFLOW;
            return OC_E_OFFSET_OVERFLOW;
        }
        b->enc[p]->build(b->enc[p], &outs[p]);
    }
    return OC_OK;
}

void oc_builder_free(oc_builder* b) {
    if (!b) return;
    for (uint32_t p = 0; p < b->nproj; p++) free_encoder(b->enc[p]);
    free(b->enc);
    free(b);
}

/* MemoryStore::read feed loop (src/io/store/memory.rs:38-44) over a block. */
int oc_decode_block(const oc_segment* seg, const uint32_t* proj, uint32_t nproj,
                    const uint8_t* data, const uint64_t* row_off, uint64_t n,
                    oc_array* outs, oc_error* err) {
    oc_builder* b = oc_builder_new(seg, proj, nproj, n);
    int st = OC_OK;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t len = row_off[i + 1] - row_off[i];
        if (len) st = oc_builder_add_row(b, data + row_off[i], len, err);
        else st = oc_builder_add_empty(b);
        if (st) { if (err) err->row = i; break; }
    }
    if (!st) st = oc_builder_build(b, outs, err);
    oc_builder_free(b);
    return st;
}

/* ---- ColumnDecoder::write_to_row (write side) ---------------------------- */
static int in_is_null(const oc_col_in* c, uint64_t i) {
    if (!c->validity) return 0;
    uint64_t bit = c->offset + i;
    return !((c->validity[bit / 8] >> (bit % 8)) & 1);
}

/* primitive.rs:85-95, bool_.rs:111-117 (b as u8), utf8.rs:113-119. */
static void write_to_row(const oc_column* col, const oc_col_in* c, uint64_t i, oc_write_row* w) {
    if (in_is_null(c, i)) return;
    uint64_t e = c->offset + i;
    if (col->dtype == OC_UTF8) {
        int32_t a = c->offsets[e], z = c->offsets[e + 1];
        oc_write_row_write_dynamic(w, col, (const uint8_t*)c->values + a, (uint64_t)(z - a));
    } else if (col->dtype == OC_BOOL) {
        uint8_t v = (uint8_t)((((const uint8_t*)c->values)[e / 8] >> (e % 8)) & 1);
        oc_write_row_write_static(w, col, &v, 1);
    } else {
        oc_write_row_write_static(w, col, (const uint8_t*)c->values + e * col->size, col->size);
    }
}

/* Table::write row loop (src/io/table/mod.rs:97-109), store-free like
 * benches/write.rs:63-71: WriteRow::new, every decoder, into KeyValue. */
int oc_encode_batch(const oc_segment* seg, const oc_col_in* cols, uint64_t n,
                    uint8_t** blob, uint64_t* blob_len, uint64_t* row_off, oc_error* err) {
    (void)err;
    vbuf out = {0, 0, 0};
    row_off[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        oc_write_row w;
        oc_write_row_new(&w, seg);
        for (uint32_t c = 0; c < seg->ncols; c++) write_to_row(&seg->cols[c], &cols[c], i, &w);
        vb_push(&out, w.bytes, w.len);
        oc_write_row_free(&w);
        row_off[i + 1] = out.len;
    }
    *blob = out.p ? out.p : (uint8_t*)calloc(1, 1);
    *blob_len = out.len;
    return OC_OK;
}

/* ---- MemoryStore restatement (src/io/store/memory.rs) ---------------------- */
struct oc_memstore {
    const uint8_t* key_data;
    const int32_t* key_off;
    const uint8_t* blob;
    const uint64_t* row_off;
    uint64_t* slot;  /* row + 1, 0 = empty */
    uint64_t mask;
};

static uint64_t oc_fnv1a(const uint8_t* p, uint64_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (uint64_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

oc_memstore* oc_memstore_new(const uint8_t* key_data, const int32_t* key_off, uint64_t n,
                             const uint8_t* blob, const uint64_t* row_off) {
    oc_memstore* m = (oc_memstore*)calloc(1, sizeof *m);
    if (!m) return NULL;
    uint64_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    m->slot = (uint64_t*)calloc(cap, sizeof(uint64_t));
    if (!m->slot) {
        free(m);
        return NULL;
    }
    m->key_data = key_data, m->key_off = key_off, m->blob = blob, m->row_off = row_off, m->mask = cap - 1;
    for (uint64_t r = 0; r < n; r++) {  /* entries.insert(key, value): a later key replaces */
        const uint8_t* k = key_data + key_off[r];
        const uint64_t len = (uint64_t)(key_off[r + 1] - key_off[r]);
        for (uint64_t s = oc_fnv1a(k, len) & m->mask;; s = (s + 1) & m->mask) {
            const uint64_t e = m->slot[s];
            if (!e) {
                m->slot[s] = r + 1;
                break;
            }
            const uint64_t o = e - 1, olen = (uint64_t)(key_off[o + 1] - key_off[o]);
            if (olen == len && memcmp(key_data + key_off[o], k, len) == 0) {
                m->slot[s] = r + 1;
                break;
            }
        }
    }
    return m;
}

int oc_memstore_read(const oc_memstore* m, const oc_segment* seg, const uint32_t* proj, uint32_t nproj,
                     const uint8_t* q_data, const int32_t* q_off, uint64_t nq, oc_array* outs, oc_error* err) {
    oc_builder* b = oc_builder_new(seg, proj, nproj, nq);
    if (!b) return OC_E_ARGUMENT;
    for (uint64_t i = 0; i < nq; i++) {  /* memory.rs:38-43 */
        const uint8_t* k = q_data + q_off[i];
        const uint64_t len = (uint64_t)(q_off[i + 1] - q_off[i]);
        uint64_t row = ~0ull;
        for (uint64_t s = oc_fnv1a(k, len) & m->mask; m->slot[s]; s = (s + 1) & m->mask) {
            const uint64_t o = m->slot[s] - 1, olen = (uint64_t)(m->key_off[o + 1] - m->key_off[o]);
            if (olen == len && memcmp(m->key_data + m->key_off[o], k, len) == 0) {
                row = o;
                break;
            }
        }
        int st;
        if (row == ~0ull) st = oc_builder_add_empty(b);
        else st = oc_builder_add_row(b, m->blob + m->row_off[row], m->row_off[row + 1] - m->row_off[row], err);
        if (st) {
            oc_builder_free(b);
            return st;
        }
    }
    const int st = oc_builder_build(b, outs, err);
    oc_builder_free(b);
    return st;
}

void oc_memstore_free(oc_memstore* m) {
    if (!m) return;
    free(m->slot);
    free(m);
}

void oc_array_free(oc_array* a) {
    if (!a) return;
    free(a->values); free(a->validity); free(a->offsets);
    memset(a, 0, sizeof *a);
}

void oc_free(void* p) { free(p); }
