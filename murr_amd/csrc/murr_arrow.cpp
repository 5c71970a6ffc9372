// murr_arrow.cpp — host Arrow arrays (murr_host_array_t, what a read's build()
// leaves in pinned memory) exported through the Arrow C Data Interface
// (arrow/c/abi.h): one struct array = the RecordBatch that
// ReadBatchBuilder::build returns (src/io/row/read.rs:100-110), imported by
// arrow-rs (`arrow::ffi::from_ffi`) or pyarrow (`RecordBatch._import_from_c`)
// in one call, instead of one Array::from_buffers per column.  The export owns
// a compacted copy of the arrays' bytes (the pinned region is reused by the
// next read): one allocation for the array side, one for the schema side, each
// freed by its release callback.  Host code only: no device calls.
#include <cstdlib>
#include <cstring>
#include <new>

#include "murr_internal.h"

namespace {

// Arrow C format strings of the reference's dtypes (src/io/codec/*.rs: the
// Arrow type each ColumnEncoder builds; fields are nullable, read.rs:105).
const char* arrow_format(uint32_t dtype) {
    switch (dtype) {
        case MURR_UTF8: return "u";
        case MURR_BOOL: return "b";
        case MURR_INT8: return "c";
        case MURR_INT16: return "s";
        case MURR_INT32: return "i";
        case MURR_INT64: return "l";
        case MURR_UINT8: return "C";
        case MURR_UINT16: return "S";
        case MURR_UINT32: return "I";
        case MURR_UINT64: return "L";
        case MURR_FLOAT32: return "f";
        case MURR_FLOAT64: return "g";
        default: return nullptr;
    }
}

constexpr int64_t kNullable = 2;  // ARROW_FLAG_NULLABLE

uint64_t align64(uint64_t x) { return (x + 63) & ~(uint64_t)63; }

// Array side: [header][child ArrowArray x n][child pointers][buffer pointer
// triples][parent buffer slot][data, 64-B aligned].
struct ArrHeader {
    uint32_t n;
};

void release_child_array(ArrowArray* a) { a->release = nullptr; }

void release_array(ArrowArray* a) {
    if (!a || !a->release) return;
    for (int64_t i = 0; i < a->n_children; i++)
        if (a->children[i] && a->children[i]->release) a->children[i]->release(a->children[i]);
    std::free(a->private_data);
    a->release = nullptr;
}

void release_child_schema(ArrowSchema* s) { s->release = nullptr; }

void release_schema(ArrowSchema* s) {
    if (!s || !s->release) return;
    for (int64_t i = 0; i < s->n_children; i++)
        if (s->children[i] && s->children[i]->release) s->children[i]->release(s->children[i]);
    std::free(s->private_data);
    s->release = nullptr;
}

}  // namespace

extern "C" {

int murr_arrow_export(const murr_host_array_t* arrays, uint32_t n, const char* const* names, ArrowArray* out_array,
                      ArrowSchema* out_schema) {
    if (!out_array || (n && (!arrays || !names))) return MURR_E_ARGUMENT;
    std::memset(out_array, 0, sizeof *out_array);
    if (out_schema) std::memset(out_schema, 0, sizeof *out_schema);
    uint64_t length = n ? arrays[0].length : 0;
    for (uint32_t i = 0; i < n; i++)
        if (arrays[i].length != length || !arrow_format(arrays[i].dtype) || !names[i]) return MURR_E_ARGUMENT;
    // ---- array side: one allocation, the bytes compacted into it
    uint64_t data = 0;
    for (uint32_t i = 0; i < n; i++) {
        const murr_host_array_t& h = arrays[i];
        if (h.validity) data += align64((h.length + 7) / 8);
        if (h.dtype == MURR_UTF8) data += align64((h.length + 1) * 4);
        data += align64(h.values_len);
    }
    const uint64_t o_children = align64(sizeof(ArrHeader)), o_ptrs = o_children + sizeof(ArrowArray) * n,
                   o_bufs = o_ptrs + sizeof(ArrowArray*) * n, o_pbuf = o_bufs + sizeof(void*) * 3 * n,
                   o_data = align64(o_pbuf + sizeof(void*));
    uint8_t* A = (uint8_t*)std::aligned_alloc(64, align64(o_data + data + 64));
    if (!A) return MURR_E_INTERNAL;
    ((ArrHeader*)A)->n = n;
    ArrowArray* kids = (ArrowArray*)(A + o_children);
    ArrowArray** kidp = (ArrowArray**)(A + o_ptrs);
    const void** bufs = (const void**)(A + o_bufs);
    const void** pbuf = (const void**)(A + o_pbuf);
    uint8_t* d = A + o_data;
    auto put = [&](const void* src, uint64_t bytes) -> const void* {
        if (!bytes) return d;  // (a zero-length buffer: any non-null address)
        std::memcpy(d, src, bytes);
        const void* at = d;
        d += align64(bytes);
        return at;
    };
    for (uint32_t i = 0; i < n; i++) {
        const murr_host_array_t& h = arrays[i];
        ArrowArray& c = kids[i];
        std::memset(&c, 0, sizeof c);
        c.length = (int64_t)h.length;
        c.null_count = (int64_t)h.null_count;
        c.offset = 0;
        c.buffers = bufs + 3 * i;
        c.buffers[0] = h.validity && h.null_count ? put(h.validity, (h.length + 7) / 8) : nullptr;
        if (h.dtype == MURR_UTF8) {
            c.n_buffers = 3;
            static const int32_t zero = 0;
            c.buffers[1] = put(h.offsets ? (const void*)h.offsets : (const void*)&zero, (h.length + 1) * 4);
            c.buffers[2] = put(h.values, h.values_len);
        } else {
            c.n_buffers = 2;
            c.buffers[1] = put(h.values, h.values_len);
        }
        c.release = release_child_array;
        kidp[i] = &c;
    }
    pbuf[0] = nullptr;
    out_array->length = (int64_t)length;
    out_array->null_count = 0;
    out_array->offset = 0;
    out_array->n_buffers = 1;  // struct: validity only (none)
    out_array->n_children = n;
    out_array->buffers = pbuf;
    out_array->children = kidp;
    out_array->dictionary = nullptr;
    out_array->release = release_array;
    out_array->private_data = A;
    // ---- schema side: "+s" with one nullable field per column (unless the
    // caller keeps the schema of an earlier export)
    if (!out_schema) return MURR_OK;
    uint64_t names_len = 0;
    for (uint32_t i = 0; i < n; i++) names_len += std::strlen(names[i]) + 1;
    const uint64_t s_kids = 0, s_ptrs = s_kids + sizeof(ArrowSchema) * n, s_names = s_ptrs + sizeof(ArrowSchema*) * n;
    uint8_t* S = (uint8_t*)std::malloc(s_names + names_len + 1);
    if (!S) {
        out_array->release(out_array);
        return MURR_E_INTERNAL;
    }
    ArrowSchema* sk = (ArrowSchema*)(S + s_kids);
    ArrowSchema** skp = (ArrowSchema**)(S + s_ptrs);
    char* nm = (char*)(S + s_names);
    for (uint32_t i = 0; i < n; i++) {
        ArrowSchema& f = sk[i];
        std::memset(&f, 0, sizeof f);
        f.format = arrow_format(arrays[i].dtype);
        const size_t l = std::strlen(names[i]) + 1;
        std::memcpy(nm, names[i], l);
        f.name = nm;
        nm += l;
        f.flags = kNullable;
        f.release = release_child_schema;
        skp[i] = &f;
    }
    out_schema->format = "+s";
    out_schema->name = "";
    out_schema->metadata = nullptr;
    out_schema->flags = 0;
    out_schema->n_children = n;
    out_schema->children = skp;
    out_schema->dictionary = nullptr;
    out_schema->release = release_schema;
    out_schema->private_data = S;
    return MURR_OK;
}

}  // extern "C"
