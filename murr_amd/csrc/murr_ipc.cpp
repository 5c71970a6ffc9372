// murr_ipc.cpp — Arrow IPC framing of decode outputs.
//
// The read path ends in arrow-rs's IPC writers: the HTTP fetch handler writes
// the batch with `StreamWriter` (src/api/http/handlers.rs:93-101: schema
// message, one record-batch message, end-of-stream marker) and Flight's DoGet
// with `FlightDataEncoderBuilder` (src/api/flight/mod.rs:85-87, the same
// schema/record-batch messages split into FlightData header + body).  This file
// writes those messages' metadata itself -- a minimal forward flatbuffer writer
// for Message / Schema / RecordBatch (Arrow format, MetadataVersion V5) -- and
// plans the body so the device can pack a whole message with one kernel
// (murr_ipc.hip) and hand it to the host with one D2H copy.
//
// Layout rules (arrow-rs 58 `IpcWriteOptions::default()`, `write_message`):
//   encapsulated message = 0xFFFFFFFF, int32 metadata size, flatbuffer padded so
//   that 8 + size is a multiple of `alignment`, then the body; every body
//   buffer starts at a multiple of `alignment` and its padding bytes are zero;
//   a column without nulls has a zero-length validity buffer.  Buffers per
//   field in schema order: utf8 (validity, offsets, data), bool and fixed width
//   (validity, values).  Fields are `nullable = true`, no metadata
//   (src/io/row/read.rs:105).
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/murr_codec.h"
#include "murr_internal.h"

namespace murr {

namespace {

// Forward flatbuffer writer: a parent is written before its children, so every
// uoffset points forward (flatbuffers' uoffset_t is unsigned).  A vtable sits
// right before its table (the table's soffset is table - vtable).
struct FB {
    std::vector<uint8_t> b;
    size_t pos() const { return b.size(); }
    void pad_to(size_t a, size_t r = 0) {
        while (b.size() % a != r) b.push_back(0);
    }
    template <class T>
    size_t put(T v) {
        size_t p = b.size();
        b.resize(p + sizeof v);
        std::memcpy(&b[p], &v, sizeof v);
        return p;
    }
    template <class T>
    void set(size_t p, T v) {
        std::memcpy(&b[p], &v, sizeof v);
    }
    void link(size_t slot, size_t target) { set<uint32_t>(slot, (uint32_t)(target - slot)); }
};

struct TF {          // one table field
    uint16_t id;     // field id in the schema (.fbs declaration order; a union takes two)
    uint8_t size;    // 1, 2, 4 or 8 bytes; refs are 4-byte uoffsets
    uint64_t val;
    bool ref;
};

// Writes vtable + table; returns the table position.  `slots` receives the
// positions of the ref fields, in the order they appear in `fs`.
size_t table(FB& f, const std::vector<TF>& fs, std::vector<size_t>* slots) {
    uint16_t nf = 0;
    for (const TF& x : fs) nf = std::max<uint16_t>(nf, (uint16_t)(x.id + 1));
    f.pad_to(2);
    size_t vt = f.pos();
    for (int i = 0; i < 2 + nf; i++) f.put<uint16_t>(0);
    f.pad_to(8, 4);  // soffset at 4 mod 8: the first field after it is 8-aligned
    size_t t = f.pos();
    f.put<int32_t>((int32_t)(t - vt));
    std::vector<size_t> at(fs.size());
    for (uint8_t sz : {8, 4, 2, 1}) {  // widest first keeps every field aligned
        for (size_t i = 0; i < fs.size(); i++) {
            if (fs[i].size != sz) continue;
            size_t p = f.pos();
            switch (sz) {
                case 8: f.put<uint64_t>(fs[i].val); break;
                case 4: f.put<uint32_t>((uint32_t)fs[i].val); break;
                case 2: f.put<uint16_t>((uint16_t)fs[i].val); break;
                default: f.put<uint8_t>((uint8_t)fs[i].val); break;
            }
            f.set<uint16_t>(vt + 4 + 2 * fs[i].id, (uint16_t)(p - t));
            at[i] = p;
        }
    }
    f.pad_to(4);
    f.set<uint16_t>(vt, (uint16_t)(4 + 2 * nf));
    f.set<uint16_t>(vt + 2, (uint16_t)(f.pos() - t));
    if (slots) {
        slots->clear();
        for (size_t i = 0; i < fs.size(); i++)
            if (fs[i].ref) slots->push_back(at[i]);
    }
    return t;
}

// Vector of 16-byte structs {int64, int64} (FieldNode, Buffer): elements 8-aligned.
size_t vec_pairs(FB& f, const std::vector<uint64_t>& ab) {
    f.pad_to(8, 4);
    size_t v = f.put<uint32_t>((uint32_t)(ab.size() / 2));
    for (uint64_t x : ab) f.put<uint64_t>(x);
    return v;
}

size_t str(FB& f, const char* s) {
    size_t n = s ? std::strlen(s) : 0;
    f.pad_to(4);
    size_t p = f.put<uint32_t>((uint32_t)n);
    for (size_t i = 0; i < n; i++) f.b.push_back((uint8_t)s[i]);
    f.b.push_back(0);
    return p;
}

// Vector of tables: returns the vector position; slots[i] = element i's uoffset.
size_t vec_tables(FB& f, size_t n, std::vector<size_t>* slots) {
    f.pad_to(4);
    size_t v = f.put<uint32_t>((uint32_t)n);
    slots->resize(n);
    for (size_t i = 0; i < n; i++) (*slots)[i] = f.put<uint32_t>(0);
    return v;
}

enum : uint8_t { kHdrSchema = 1, kHdrRecordBatch = 3 };          // MessageHeader union
enum : uint8_t { kTInt = 2, kTFloat = 3, kTUtf8 = 5, kTBool = 6 };  // Type union
constexpr uint16_t kV5 = 4;                                       // MetadataVersion.V5

// Message {version, header_type, header, bodyLength}; returns the header slot.
size_t message(FB& f, uint8_t hdr, uint64_t body_len) {
    size_t root = f.put<uint32_t>(0);
    std::vector<size_t> s;
    size_t m = table(f, {{0, 2, kV5, false}, {1, 1, hdr, false}, {2, 4, 0, true}, {3, 8, body_len, false}}, &s);
    f.link(root, m);
    return s[0];
}

// Type union tag of one murr dtype (src/core/schema.rs DTypeName -> arrow DataType).
uint8_t type_tag(uint32_t dt) {
    switch (dt) {
        case MURR_UTF8: return kTUtf8;
        case MURR_BOOL: return kTBool;
        case MURR_FLOAT32:
        case MURR_FLOAT64: return kTFloat;
        default: return kTInt;
    }
}

// The type table: Int {bitWidth, is_signed}, FloatingPoint {precision}, Utf8 {}, Bool {}.
size_t type_table(FB& f, uint32_t dt) {
    static const uint8_t bits[MURR_NUM_DTYPES] = {0, 0, 8, 16, 32, 64, 8, 16, 32, 64, 0, 0};
    switch (type_tag(dt)) {
        case kTUtf8:
        case kTBool: return table(f, {}, nullptr);
        case kTFloat: return table(f, {{0, 2, dt == MURR_FLOAT32 ? 1u : 2u, false}}, nullptr);  // SINGLE / DOUBLE
        default: break;
    }
    bool is_signed = dt >= MURR_INT8 && dt <= MURR_INT64;
    return table(f, {{0, 4, bits[dt], false}, {1, 1, is_signed ? 1u : 0u, false}}, nullptr);
}

// Prefix + padding around a finished flatbuffer.
void encapsulate(const FB& f, uint32_t align, std::vector<uint8_t>* out) {
    uint64_t total = (8 + f.b.size() + align - 1) / align * align;
    out->assign(total, 0);
    uint32_t cont = 0xFFFFFFFFu;
    int32_t size = (int32_t)(total - 8);
    std::memcpy(out->data(), &cont, 4);
    std::memcpy(out->data() + 4, &size, 4);
    std::memcpy(out->data() + 8, f.b.data(), f.b.size());
}

}  // namespace

bool ipc_align_ok(uint32_t a) { return a >= 8 && a <= 4096 && (a & (a - 1)) == 0; }

int ipc_schema(const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj, const char* const* names,
               uint32_t align, std::vector<uint8_t>* out) {
    FB f;
    size_t hslot = message(f, kHdrSchema, 0);
    std::vector<size_t> s;
    size_t sch = table(f, {{0, 2, 0, false}, {1, 4, 0, true}}, &s);  // endianness Little, fields
    f.link(hslot, sch);
    std::vector<size_t> fslots;
    f.link(s[0], vec_tables(f, nproj, &fslots));
    for (uint32_t p = 0; p < nproj; p++) {
        uint32_t dt = seg->cols[proj[p]].dtype;
        std::vector<size_t> r;
        // Field {name, nullable, type_type, type, dictionary (absent), children}
        size_t fld = table(f, {{0, 4, 0, true}, {1, 1, 1, false}, {2, 1, type_tag(dt), false}, {3, 4, 0, true},
                               {5, 4, 0, true}},
                           &r);
        f.link(fslots[p], fld);
        f.link(r[0], str(f, names ? names[p] : ""));
        f.link(r[1], type_table(f, dt));
        std::vector<size_t> none;
        f.link(r[2], vec_tables(f, 0, &none));
    }
    encapsulate(f, align, out);
    return MURR_OK;
}

// Body layout of one record batch: IPC buffers in order, offsets relative to
// the body start.  len[i] == 0 for a validity buffer of a column without nulls.
int ipc_batch_plan(const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj, uint64_t n,
                   const uint64_t* null_counts, const uint64_t* data_lens, uint32_t align, IpcPlan* plan) {
    plan->buf_off.clear();
    plan->buf_len.clear();
    plan->buf_field.clear();
    plan->buf_kind.clear();
    uint64_t at = 0, bm = (n + 7) / 8;
    std::vector<uint64_t> nodes, bufs;
    auto add = [&](uint32_t p, uint32_t kind, uint64_t len) {
        plan->buf_off.push_back(at);
        plan->buf_len.push_back(len);
        plan->buf_field.push_back(p);
        plan->buf_kind.push_back(kind);
        bufs.push_back(at);
        bufs.push_back(len);
        at += (len + align - 1) / align * align;
    };
    for (uint32_t p = 0; p < nproj; p++) {
        uint32_t dt = seg->cols[proj[p]].dtype;
        nodes.push_back(n);
        nodes.push_back(null_counts[p]);
        add(p, kIpcValidity, null_counts[p] ? bm : 0);
        if (dt == MURR_UTF8) {
            add(p, kIpcOffsets, 4 * (n + 1));
            add(p, kIpcValues, data_lens[p]);
        } else if (dt == MURR_BOOL) {
            add(p, kIpcValues, bm);
        } else {
            add(p, kIpcValues, n * (uint64_t)seg->cols[proj[p]].size);
        }
    }
    plan->body_len = at;
    FB f;
    size_t hslot = message(f, kHdrRecordBatch, at);
    std::vector<size_t> s;
    // RecordBatch {length, nodes, buffers}
    size_t rb = table(f, {{0, 8, n, false}, {1, 4, 0, true}, {2, 4, 0, true}}, &s);
    f.link(hslot, rb);
    f.link(s[0], vec_pairs(f, nodes));
    f.link(s[1], vec_pairs(f, bufs));
    encapsulate(f, align, &plan->meta);
    return MURR_OK;
}

}  // namespace murr

using namespace murr;

namespace {

bool proj_ok(const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj) {
    if (!seg || (seg->ncols && !seg->cols) || (nproj && !proj)) return false;
    for (uint32_t p = 0; p < nproj; p++)
        if (proj[p] >= seg->ncols || seg->cols[proj[p]].dtype >= MURR_NUM_DTYPES) return false;
    return true;
}

int emit(const std::vector<uint8_t>& m, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    *out_len = m.size();
    if (!out) return MURR_OK;
    if (cap < m.size()) return MURR_E_CAPACITY;
    std::memcpy(out, m.data(), m.size());
    return MURR_OK;
}

}  // namespace

extern "C" {

int murr_ipc_schema(const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj, const char* const* names,
                    uint32_t alignment, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    if (!out_len || !ipc_align_ok(alignment) || !proj_ok(seg, proj, nproj)) return MURR_E_ARGUMENT;
    std::vector<uint8_t> m;
    ipc_schema(seg, proj, nproj, names, alignment, &m);
    return emit(m, out, cap, out_len);
}

int murr_ipc_batch_host(const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj,
                        const murr_host_array_t* arrays, uint64_t n_rows, uint32_t alignment, uint8_t* out,
                        uint64_t cap, uint64_t* out_len) {
    if (!out_len || !ipc_align_ok(alignment) || !proj_ok(seg, proj, nproj) || (nproj && !arrays))
        return MURR_E_ARGUMENT;
    if (!nproj) return MURR_E_ARROW;  // RecordBatch without columns (src/io/row/read.rs:106-108)
    std::vector<uint64_t> nulls(nproj), lens(nproj);
    for (uint32_t p = 0; p < nproj; p++) {
        if (arrays[p].dtype != seg->cols[proj[p]].dtype) return MURR_E_DTYPE;
        if (arrays[p].length != n_rows) return MURR_E_ARGUMENT;
        nulls[p] = arrays[p].null_count;
        lens[p] = arrays[p].values_len;
    }
    IpcPlan plan;
    ipc_batch_plan(seg, proj, nproj, n_rows, nulls.data(), lens.data(), alignment, &plan);
    uint64_t total = plan.meta.size() + plan.body_len;
    *out_len = total;
    if (!out) return MURR_OK;
    if (cap < total) return MURR_E_CAPACITY;
    std::memcpy(out, plan.meta.data(), plan.meta.size());
    uint8_t* body = out + plan.meta.size();
    std::memset(body, 0, plan.body_len);
    for (size_t i = 0; i < plan.buf_off.size(); i++) {
        uint64_t len = plan.buf_len[i];
        if (!len) continue;
        const murr_host_array_t& a = arrays[plan.buf_field[i]];
        const void* src = plan.buf_kind[i] == kIpcValidity  ? (const void*)a.validity
                          : plan.buf_kind[i] == kIpcOffsets ? (const void*)a.offsets
                                                            : (const void*)a.values;
        if (!src) return MURR_E_ARGUMENT;
        std::memcpy(body + plan.buf_off[i], src, len);
    }
    return MURR_OK;
}

uint64_t murr_ipc_eos(uint8_t* out) {
    static const uint8_t eos[8] = {0xFF, 0xFF, 0xFF, 0xFF, 0, 0, 0, 0};
    if (out) std::memcpy(out, eos, 8);
    return 8;
}

}  // extern "C"
