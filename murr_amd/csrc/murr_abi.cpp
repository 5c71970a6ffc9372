// murr_abi.cpp — host side of the C ABI declared in include/murr_codec.h.
//
// Owns the per-context HIP stream, events and a grow-only device workspace
// (zeroed counters + look-back granules + descriptor tables), validates
// arguments the way the reference does, launches the kernels in
// murr_kernels.hip and turns the packed device error word back into the
// reference's first error.  No exceptions cross the boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <random>
#include <atomic>
#include <map>
#include <mutex>
#include <set>
#include <chrono>
#include <condition_variable>
#include <thread>
#include <unordered_map>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <memory>
#include <vector>

#include "../../include/murr_codec.h"
#include "murr_internal.h"

using namespace murr;

namespace {

constexpr uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

int dtype_size(uint32_t d) {
    static const int sz[MURR_NUM_DTYPES] = {4, 1, 1, 2, 4, 8, 1, 2, 4, 8, 4, 8};
    return d < MURR_NUM_DTYPES ? sz[d] : -1;
}

int set_err(murr_error_t* err, int status, int hip = 0) {
    if (err) {
        std::memset(err, 0, sizeof *err);
        err->status = status;
        err->hip_error = hip;
    }
    return status;
}

bool valid_segment(const murr_segment_t* s) {
    if (!s || (s->ncols && !s->cols)) return false;
    uint32_t off = 0;
    for (uint32_t i = 0; i < s->ncols; i++) {
        const murr_column_t& c = s->cols[i];
        if (dtype_size(c.dtype) < 0 || (int)c.size != dtype_size(c.dtype) || c.index >= s->ncols)
            return false;
        off = std::max(off, c.offset + c.size);
    }
    return s->bitset_size == (s->ncols + 7) / 8 && off <= s->capacity;
}

}  // namespace

struct murr_ctx {
    // Library-allocated outputs handed to the caller (murr_sst_decode's
    // entries) that came back through murr_dev_free / murr_sst_result_free,
    // kept for reuse (size -> pointer), so a repeated call does not pay six
    // hipMallocs (~0.1 ms); released at context destroy, or past
    // kDevCacheMax bytes.  Which pointers are such outputs: g_dcached.
    std::multimap<uint64_t, void*> dfree;
    uint64_t dfree_bytes = 0;
    // some buffer entered dfree since the last device synchronisation: work
    // queued before its free (on any stream of the device: another context's
    // scan reading an adopted SST arena, the caller's own) may still read it,
    // so the next reuse first waits for the device, as the hipFree it
    // replaces did
    bool dfree_unsynced = false;
    int device = 0;
    int cus = 256;
    int enc_grid_per_cu = 1;
    hipStream_t stream = nullptr;
    hipEvent_t k0 = nullptr, k1 = nullptr;
    hipEvent_t lk0 = nullptr, lk1 = nullptr;  // a prepared run's events, when it was the last timed op
    bool timed = false;
    uint8_t* ws = nullptr;  // device workspace
    uint64_t ws_cap = 0;
    uint8_t* hs = nullptr;  // pinned host scratch
    uint64_t hs_cap = 0;
    // pending decode
    bool pending = false;
    murr_array_t* outs = nullptr;
    std::vector<uint64_t> n_rows;
    std::vector<uint32_t> dtypes;  // per projected column
    uint32_t nblocks = 0, nproj = 0;
    uint64_t rb_off = 0;           // readback offset in hs
    // a stream-mode JIT launch, re-run in local mode if its look-back timed out
    bool retry_local = false;
    std::vector<murr_column_t> r_cols;
    murr_segment_t r_seg{};
    std::vector<uint32_t> r_proj;
    std::vector<murr_block_t> r_blocks;
    double r_est = 0;
    int pending_status = MURR_OK;
    const char* last_kernel = "";  // kernel of the last decode launch
    murr_opts_t opts{};            // kernel selection (murr_ctx_set_opts)
    murr_ctx_stats_t stats{};
#ifdef MURR_TUNING
    uint64_t tl_off = 0;  // stamped builds, verbose: per-workgroup timeline in ws (0 = none)
    uint64_t tl_n = 0;
#endif
    // Staging buffers of freed builders, reused by the next ones (a read builds
    // a ReadBatchBuilder per batch, src/io/row/read.rs:69-83; pinned and device
    // allocations cost far more than the batch itself).
    struct Buf {
        uint8_t* p;
        uint64_t cap;
        bool pinned;
    };
    std::vector<Buf> pool;
    std::vector<hipEvent_t> event_pool;
    uint64_t* aux = nullptr;  // device scratch of the gather scan (group sums)
    uint64_t aux_cap = 0;     // entries
    unsigned long long* glb = nullptr;  // the fused small gather's two look-back word sets
    uint32_t glb_set = 0;               // the set the next launch uses (zeroed by the one before)
    hipEvent_t xev = nullptr; // multi-GPU reads: this stream's work, awaited by the home stream
    hipEvent_t hev = nullptr; // multi-GPU reads (as home): the work queued before a read, awaited by the shards
    // Fused transfers (the streaming host decode, murr_hstream): the next
    // decode enqueue uploads its descriptors in one segment-copy kernel with
    // the batch's input (`xin`), and reads its counters back in one with the
    // decoded buffers (`xout`), instead of two hipMemcpyAsync; with `xtimed`
    // the caller's events xe[0..3] bracket the two copies (and k0/k1 the decode).
    bool xfer = false, xtimed = false;
    std::vector<CopySeg> xin, xout;
    hipEvent_t xe[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t mk[4] = {nullptr, nullptr, nullptr, nullptr};  // murr_ctx_mark: caller's timing marks
};

// Device key index (murr_index.hip): the keys' own copy and the slot table.
struct murr_index {
    int device = 0;
    uint8_t* key_data = nullptr;    // the keys, back to back (grows by doubling)
    int32_t* key_off = nullptr;     // n + 1 offsets into key_data (grows by doubling)
    uint64_t* slots = nullptr;
    uint64_t* loc = nullptr;
    uint64_t* kp = nullptr;         // per slot: the key's first 16 bytes
    uint64_t* rc = nullptr;         // slot cache: per slot {row offset, row bytes} (murr_index_cache_rows)
    uint32_t* ru = nullptr;         //   and the row's utf8 string bytes [rc_nu]
    uint32_t rc_nu = 0;
    uint64_t cached = 0;            // rows [0, cached) are in the slot cache (0 after a rehash)
    unsigned long long* err = nullptr;
    uint64_t n = 0, mask = 0;
    uint64_t key_bytes = 0, key_cap = 0, off_cap = 0;
};

namespace {

int hip_fail(murr_error_t* err, hipError_t e) { return set_err(err, MURR_E_HIP, (int)e); }

uint32_t nutf8_of(const murr_segment_t* seg) {
    uint32_t n = 0;
    for (uint32_t i = 0; i < seg->ncols; i++) n += seg->cols[i].dtype == MURR_UTF8;
    return n;
}

#define HIPC(expr)                                          \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return hip_fail(err, _e);     \
    } while (0)

// Caller-owned device outputs through the context's reuse cache: a freed
// buffer of at least `bytes` (and at most twice that plus one granule) comes
// back instead of a new hipMalloc; new ones are rounded to the granule: 1 MiB,
// or 4 KiB below 1 MiB (a small SST file's arena stays small).  hipSuccess or
// the allocation's error (the cache is released and the call retried once).
constexpr uint64_t kDevCacheMax = 1ull << 30;
// process-wide: every buffer dev_alloc_cached made, with its context and size
// (a pointer freed through another context, or re-allocated by a plain
// hipMalloc after a direct hipFree, is dropped from it, never reused stale)
std::mutex g_dc_mu;
std::unordered_map<void*, std::pair<murr_ctx*, uint64_t>> g_dcached;
hipError_t dev_alloc_cached(murr_ctx* c, uint64_t bytes, void** out) {
    std::lock_guard<std::mutex> lk(g_dc_mu);
    const uint64_t gran = bytes < (1u << 20) ? 4096u : (1u << 20);
    auto it = c->dfree.lower_bound(bytes);
    if (it != c->dfree.end() && it->first <= 2 * bytes + gran) {
        if (c->dfree_unsynced) {
            // every buffer freed so far: its readers queued before the free are done
            const hipError_t se = hipDeviceSynchronize();
            if (se != hipSuccess) return se;
            c->dfree_unsynced = false;
        }
        *out = it->second;
        c->dfree_bytes -= it->first;
        c->dfree.erase(it);
        return hipSuccess;
    }
    const uint64_t sz = std::max<uint64_t>((bytes + gran - 1) & ~(gran - 1), gran);
    hipError_t e = hipMalloc(out, sz);
    if (e != hipSuccess && !c->dfree.empty()) {
        (void)hipGetLastError();
        for (const auto& f : c->dfree) {
            g_dcached.erase(f.second);
            (void)hipFree(f.second);
        }
        c->dfree.clear();
        c->dfree_bytes = 0;
        e = hipMalloc(out, sz);
    }
    if (e == hipSuccess) g_dcached[*out] = {c, sz};
    return e;
}
// A buffer dev_alloc_cached handed out goes back to the cache (true); any
// other pointer is the caller's to hipFree (false).
bool dev_free_cached(murr_ctx* c, void* p) {
    std::lock_guard<std::mutex> lk(g_dc_mu);
    auto it = g_dcached.find(p);
    if (it == g_dcached.end()) return false;
    if (it->second.first != c) {  // another context's: released, not cached here
        g_dcached.erase(it);
        return false;
    }
    c->dfree.emplace(it->second.second, p);
    c->dfree_bytes += it->second.second;
    c->dfree_unsynced = true;
    while (c->dfree_bytes > kDevCacheMax && !c->dfree.empty()) {  // the largest go first
        auto last = std::prev(c->dfree.end());
        c->dfree_bytes -= last->first;
        g_dcached.erase(last->second);
        (void)hipFree(last->second);
        c->dfree.erase(last);
    }
    return true;
}
// A plain allocation at `p` (hipMalloc handed the address out again): drop
// any stale record of it.
void dev_forget(void* p) {
    std::lock_guard<std::mutex> lk(g_dc_mu);
    g_dcached.erase(p);
}

// Grow a device buffer to at least `need` bytes (doubling), keeping `keep` bytes.
template <class T>
int grow(murr_ctx* c, T** p, uint64_t* cap, uint64_t need, uint64_t keep, murr_error_t* err) {
    if (need <= *cap && *p) return MURR_OK;
    uint64_t ncap = std::max<uint64_t>(std::max<uint64_t>(need, 2 * *cap), 256);
    T* q = nullptr;
    HIPC(hipMalloc(&q, ncap));
    if (keep && *p) HIPC(hipMemcpyAsync(q, *p, keep, hipMemcpyDeviceToDevice, c->stream));
    if (*p) {
        HIPC(hipStreamSynchronize(c->stream));
        HIPC(hipFree(*p));
    }
    *p = q;
    *cap = ncap;
    return MURR_OK;
}

int ensure_ws(murr_ctx* c, uint64_t bytes, murr_error_t* err) {
    if (bytes <= c->ws_cap) return MURR_OK;
    if (c->ws) HIPC(hipFree(c->ws));
    c->ws = nullptr;
    uint64_t cap = std::max<uint64_t>(round_up(bytes, 1 << 20), 4 << 20);
    HIPC(hipMalloc(&c->ws, cap));
    c->ws_cap = cap;
    return MURR_OK;
}

int ensure_hs(murr_ctx* c, uint64_t bytes, murr_error_t* err) {
    if (bytes <= c->hs_cap) return MURR_OK;
    if (c->hs) HIPC(hipHostFree(c->hs));
    c->hs = nullptr;
    uint64_t cap = std::max<uint64_t>(round_up(bytes, 1 << 16), 1 << 20);
    HIPC(hipHostMalloc(&c->hs, cap, hipHostMallocDefault));
    c->hs_cap = cap;
    return MURR_OK;
}

// Decode the packed device error word into murr_error_t.
#ifdef MURR_TUNING
// Tuning builds (make tuning): the MURR_* tuning variables of earlier rounds'
// tools, read once per context.  Release builds never read them.
void opts_from_env(murr_opts_t* o) {
    auto num = [](const char* n, uint32_t* v) {
        if (const char* e = std::getenv(n)) *v = (uint32_t)std::atoll(e);
    };
    if (const char* e = std::getenv("MURR_DECODE_JIT")) o->kernel = std::atoi(e) == 0 ? 2u : 1u;
    if (const char* e = std::getenv("MURR_ENCODE_JIT")) o->encode_kernel = std::atoi(e) == 0 ? 2u : 1u;
    if (const char* e = std::getenv("MURR_JIT_MODE")) o->mode = std::string(e) == "local" ? 1u : 2u;
    if (std::getenv("MURR_JIT_CUT")) o->mode = 3;
    if (const char* e = std::getenv("MURR_JIT_SHAPE")) std::sscanf(e, "%ux%u", &o->shape_nw, &o->shape_r);
    num("MURR_JIT_SEGTILES", &o->seg_tiles);
    num("MURR_JIT_VROWS", &o->vrows);
    num("MURR_JIT_LDS", &o->lds_budget);
    num("MURR_JIT_STAGE", &o->stage);
    if (std::getenv("MURR_DECODE_VERBOSE")) o->verbose = 1;
}
#endif

#ifdef MURR_TUNING
// Per-workgroup timeline of an MJ_TIMELINE JIT launch, in microseconds
// from the first workgroup's start: percentiles of the start, of the wait for
// the first tile, of the end; tiles per workgroup; the end by tile count and
// by XCD.
void print_timeline(murr_ctx* c) {
    std::vector<uint64_t> t(4 * c->tl_n);
    if (hipMemcpy(t.data(), c->ws + c->tl_off, 8 * t.size(), hipMemcpyDeviceToHost) != hipSuccess) return;
    uint64_t t0 = ~0ull;
    for (uint64_t g = 0; g < c->tl_n; g++)
        if (t[4 * g]) t0 = std::min(t0, t[4 * g]);
    std::vector<double> st, b0, en, dur;
    std::map<uint32_t, std::pair<double, int>> by_tiles, by_xcc;
    std::map<uint32_t, std::vector<double>> by_simd;  // decode wave 0's SIMD: durations
    FILE* dump = nullptr;
    if (const char* e = std::getenv("MURR_TIMELINE_DUMP")) dump = std::fopen(e, "a");
    for (uint64_t g = 0; g < c->tl_n; g++) {
        if (!t[4 * g]) continue;
        const double s0 = (t[4 * g] - t0) * 0.01, s1 = (t[4 * g + 1] - t0) * 0.01, s2 = (t[4 * g + 2] - t0) * 0.01;
        st.push_back(s0), b0.push_back(s1 - s0), en.push_back(s2), dur.push_back(s2 - s0);
        const uint64_t w = t[4 * g + 3];
        const uint32_t tiles = (uint32_t)(w & 0xFFFF), xcc = (uint32_t)(w >> 48) & 0xF;
        const uint32_t hwid = (uint32_t)(w >> 16);  // HW_ID: simd [5:4], cu [11:8], sh [12], se [15:13]
        auto& a = by_tiles[tiles];
        a.first = std::max(a.first, s2), a.second++;
        auto& x = by_xcc[xcc];
        x.first = std::max(x.first, s2), x.second++;
        by_simd[(hwid >> 4) & 3].push_back(s2 - s0);
        if (dump)
            std::fprintf(dump, "%llu,%.2f,%.2f,%.2f,%u,%u,%u,%u,%u,%u\n", (unsigned long long)g, s0, s1, s2, tiles, xcc,
                         (hwid >> 13) & 7, (hwid >> 12) & 1, (hwid >> 8) & 15, (hwid >> 4) & 3);
    }
    if (dump) std::fclose(dump);
    auto pct = [](std::vector<double> v, const char* name) {
        std::sort(v.begin(), v.end());
        if (v.empty()) return;
        auto q = [&](double f) { return v[(size_t)std::min<double>(v.size() - 1, f * (v.size() - 1))]; };
        std::fprintf(stderr, "  %-10s p0 %7.2f p10 %7.2f p50 %7.2f p90 %7.2f p99 %7.2f max %7.2f us\n", name, q(0), q(0.1),
                     q(0.5), q(0.9), q(0.99), q(1));
    };
    std::fprintf(stderr, "timeline (%zu workgroups):\n", st.size());
    pct(st, "start");
    pct(b0, "first tile");
    pct(dur, "duration");
    pct(en, "end");
    for (auto& kv : by_tiles) std::fprintf(stderr, "  tiles %u: %d workgroups, last end %.2f us\n", kv.first, kv.second.second, kv.second.first);
    for (auto& kv : by_xcc) std::fprintf(stderr, "  xcc %u: %d workgroups, last end %.2f us\n", kv.first, kv.second.second, kv.second.first);
    for (auto& kv : by_simd) {
        char nm[32];
        std::snprintf(nm, sizeof nm, "dur simd%u", kv.first);
        pct(kv.second, nm);
    }
}
#endif

int unpack_err(unsigned long long word, murr_error_t* err) {
    if (!word) return MURR_OK;
    uint64_t key = ~(uint64_t)word;
    int st = (int)(key & 0xF);
    if (err) {
        err->status = st;
        err->block = (uint32_t)(key >> 46);
        err->row = (key >> 14) & 0xFFFFFFFFull;
        err->column = (uint32_t)((key >> 4) & 0x3FF);
    }
    return st;
}

}  // namespace

extern "C" {

// ---- device key index ------------------------------------------------------

void murr_index_free(murr_index_t* x) {
    if (!x) return;
    (void)hipSetDevice(x->device);
    for (void* p : {(void*)x->key_data, (void*)x->key_off, (void*)x->slots, (void*)x->loc, (void*)x->kp,
                    (void*)x->rc, (void*)x->ru, (void*)x->err})
        if (p) (void)hipFree(p);
    delete x;
}

int murr_index_build(murr_ctx_t* c, const uint8_t* key_data, const int32_t* key_offsets, uint64_t key_offset,
                     uint64_t n, murr_index_t** out, murr_error_t* err) {
    if (!c || !out || c->pending || (n && (!key_data || !key_offsets)) || n >= kMissing)
        return set_err(err, MURR_E_ARGUMENT);
    *out = nullptr;
    HIPC(hipSetDevice(c->device));
    std::unique_ptr<murr_index, void (*)(murr_index*)> x(new murr_index, murr_index_free);
    x->device = c->device;
    HIPC(hipMalloc(&x->err, 8));
    HIPC(hipMemsetAsync(x->err, 0, 8, c->stream));
    const int st = murr_index_append(c, x.get(), key_data, key_offsets, key_offset, n, err);
    if (st) return st;
    *out = x.release();
    return MURR_OK;
}


int murr_index_append(murr_ctx_t* c, murr_index_t* x, const uint8_t* key_data, const int32_t* key_offsets,
                      uint64_t key_offset, uint64_t n, murr_error_t* err) {
    if (!c || !x || x->device != c->device || c->pending || (n && (!key_data || !key_offsets)) ||
        x->n + n >= kMissing)
        return set_err(err, MURR_E_ARGUMENT);
    HIPC(hipSetDevice(c->device));
    // the appended keys' byte range [first, last) in key_data
    int32_t ends[2] = {0, 0};
    if (n) {
        HIPC(hipMemcpyAsync(&ends[0], key_offsets + key_offset, 4, hipMemcpyDeviceToHost, c->stream));
        HIPC(hipMemcpyAsync(&ends[1], key_offsets + key_offset + n, 4, hipMemcpyDeviceToHost, c->stream));
        HIPC(hipStreamSynchronize(c->stream));
        if (ends[0] < 0 || ends[1] < ends[0]) return set_err(err, MURR_E_ARGUMENT);
    }
    const uint64_t bytes = (uint64_t)(ends[1] - ends[0]);
    if (x->key_bytes + bytes > 0x7FFFFFFFull) return set_err(err, MURR_E_OFFSET_OVERFLOW);
    int st = grow(c, &x->key_data, &x->key_cap, x->key_bytes + bytes + 16, x->key_bytes, err);
    if (!st) st = grow(c, &x->key_off, &x->off_cap, 4 * (x->n + n + 1), 4 * (x->n + 1), err);
    if (st) return st;
    if (x->n == 0) HIPC(hipMemsetAsync(x->key_off, 0, 4, c->stream));
    if (bytes) HIPC(hipMemcpyAsync(x->key_data + x->key_bytes, key_data + ends[0], bytes, hipMemcpyDeviceToDevice, c->stream));
    // offsets of keys n_old + 1 .. n_old + n, rebased onto the key copy
    HIPC(launch_offsets_rebase(x->key_off + x->n + 1, key_offsets + key_offset + 1, n,
                               (int64_t)x->key_bytes - ends[0], c->stream));
    const uint64_t n0 = x->n, total = x->n + n;
    IndexArgs a{};
    a.key_data = x->key_data;
    a.key_off = x->key_off;
    a.err = x->err;
    uint64_t slots = x->mask + 1;
    // slots per key at least: load factor <= 1/3.  At 1/2 (round 5) a
    // config C table sat at 0.48 and every 64-key group of a read walked a
    // 6-9 slot chain for its slowest key; at 1/3 (0.24 there) its reads took
    // 28.7-29.5 us instead of 31.2-33.2 (tools/r06/EXPERIMENTS.md #34).
    uint64_t spread = 3;
#ifdef MURR_TUNING
    if (const char* v = std::getenv("MURR_INDEX_SPREAD")) spread = std::max<uint64_t>(2, std::strtoull(v, nullptr, 10));  // (A/B)
#endif
    if (!x->slots || spread * total > slots) {
        // rehash: a table of >= spread * total slots, every key inserted again
        slots = 64;
        while (slots < spread * total) slots <<= 1;
        for (void** p : {(void**)&x->slots, (void**)&x->loc, (void**)&x->kp, (void**)&x->rc, (void**)&x->ru}) {
            if (*p) HIPC(hipFree(*p));
            *p = nullptr;
        }
        x->cached = 0;  // (the slot cache is rebuilt over the new table by the next murr_index_cache_rows)
        HIPC(hipMalloc(&x->slots, 8 * slots));
        HIPC(hipMalloc(&x->loc, 8 * slots));
        HIPC(hipMalloc(&x->kp, 16 * slots));
        HIPC(hipMemsetAsync(x->slots, 0xFF, 8 * slots, c->stream));
        x->mask = slots - 1;
        a.base = 0;
        a.n = total;
    } else {
        a.base = n0;
        a.n = n;
    }
    a.slots = x->slots;
    a.loc = x->loc;
    a.kp = x->kp;
    a.mask = x->mask;
    HIPC(launch_index_insert(a, c->stream));
    unsigned long long word = 0;
    HIPC(hipMemcpyAsync(&word, x->err, 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    if (word) return set_err(err, MURR_E_INTERNAL);
    x->n = total;
    x->key_bytes += bytes;
    return MURR_OK;
}

int murr_index_prefer_seq(murr_ctx_t* c, murr_index_t* x, const uint64_t* seqs, murr_error_t* err) {
    if (!c || !x || x->device != c->device || c->pending || (x->n && !seqs)) return set_err(err, MURR_E_ARGUMENT);
    if (!x->n) return MURR_OK;
    HIPC(hipSetDevice(c->device));
    const uint64_t slots = x->mask + 1;
    unsigned long long* tmp = nullptr;  // best seq, then winning row + 1, per slot
    HIPC(hipMalloc(&tmp, 16 * slots));
    std::unique_ptr<unsigned long long, hipError_t (*)(void*)> hold(tmp, hipFree);
    HIPC(hipMemsetAsync(tmp, 0, 16 * slots, c->stream));
    IndexArgs a{};
    a.key_data = x->key_data;
    a.key_off = x->key_off;
    a.slots = x->slots;
    a.loc = x->loc;
    a.mask = x->mask;
    a.n = x->n;
    a.err = x->err;
    HIPC(launch_index_seq(a, seqs, tmp, tmp + slots, c->stream));
    x->cached = 0;  // (rows moved between slots)
    unsigned long long word = 0;
    HIPC(hipMemcpyAsync(&word, x->err, 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    if (word) return set_err(err, MURR_E_INTERNAL);
    return MURR_OK;
}

int murr_index_cache_rows(murr_ctx_t* c, murr_index_t* x, const uint64_t* row_off, const uint32_t* row_ulen,
                          uint32_t nutf8, murr_error_t* err) {
    if (!c || !x || x->device != c->device || c->pending || (x->n && !row_off) || (nutf8 && !row_ulen) ||
        nutf8 > kGatherMaxU)
        return set_err(err, MURR_E_ARGUMENT);
    if (!x->n) return MURR_OK;
    HIPC(hipSetDevice(c->device));
    const uint64_t slots = x->mask + 1;
    if (!x->rc || nutf8 != x->rc_nu) {
        if (x->rc) HIPC(hipFree(x->rc));
        if (x->ru) HIPC(hipFree(x->ru));
        x->rc = nullptr;
        x->ru = nullptr;
        HIPC(hipMalloc(&x->rc, 16 * slots));
        if (nutf8) HIPC(hipMalloc(&x->ru, 4ull * nutf8 * slots));
        x->rc_nu = nutf8;
        x->cached = 0;
    }
    IndexArgs a{};
    a.key_data = x->key_data;
    a.key_off = x->key_off;
    a.slots = x->slots;
    a.loc = x->loc;
    a.mask = x->mask;
    a.n = x->n;
    a.rc = x->rc;
    a.ru = x->ru;
    a.nu_rc = nutf8;
    HIPC(launch_index_cache_rows(a, row_off, row_ulen, x->cached, c->stream));
    x->cached = x->n;
    return MURR_OK;
}

int murr_index_info(const murr_index_t* x, uint64_t* n, uint64_t* slots) {
    if (!x) return MURR_E_ARGUMENT;
    if (n) *n = x->n;
    if (slots) *slots = x->mask + 1;
    return MURR_OK;
}

namespace {
// Device scratch of the gather scans (group sums, rows): at least `need` u64.
int ensure_aux(murr_ctx* c, uint64_t need, murr_error_t* err) {
    if (need <= c->aux_cap) return MURR_OK;
    if (c->aux) HIPC(hipFree(c->aux));
    c->aux = nullptr;
    c->aux_cap = 0;
    const uint64_t cap = std::max<uint64_t>(need, 1 << 16);
    HIPC(hipMalloc(&c->aux, 8 * cap));
    c->aux_cap = cap;
    return MURR_OK;
}

// The fused small gather's words (gather_fused, murr_index.hip): two sets,
// both zeroed once here; launches alternate between them and each zeroes the
// other for the next (launches on one context's stream run in order).
int small_gather_words(murr_ctx* c, IndexArgs* a, murr_error_t* err) {
    a->lb = a->lb_other = nullptr;
    if (a->nq == 0 || a->nq > 64 * kGatherGroups) return MURR_OK;
    if (!c->glb) {
        void* p = nullptr;
        HIPC(hipMalloc(&p, 16 * kGatherWords));
        HIPC(hipMemsetAsync(p, 0, 16 * kGatherWords, c->stream));
        c->glb = (unsigned long long*)p;
    }
    a->lb = c->glb + kGatherWords * c->glb_set;
    c->glb_set ^= 1u;
    a->lb_other = c->glb + kGatherWords * c->glb_set;
    return MURR_OK;
}

IndexArgs index_args(const murr_index_t* x, const uint8_t* q_data, const int32_t* q_offsets, uint64_t nq) {
    IndexArgs a{};
    a.key_data = x->key_data;
    a.key_off = x->key_off;
    a.slots = x->slots;
    a.loc = x->loc;
    a.mask = x->mask;
    a.n = x->n;
    a.q_data = q_data;
    a.q_off = q_offsets;
    a.nq = nq;
    return a;
}
}  // namespace

int murr_index_lookup(murr_ctx_t* c, const murr_index_t* x, const uint8_t* q_data, const int32_t* q_offsets,
                      uint64_t nq, uint32_t* rows) {
    murr_error_t* err = nullptr;
    if (!c || !x || x->device != c->device || c->pending || (nq && (!q_data || !q_offsets || !rows)))
        return MURR_E_ARGUMENT;
    HIPC(hipSetDevice(c->device));
    IndexArgs a = index_args(x, q_data, q_offsets, nq);
    a.rows = rows;
    HIPC(launch_index_probe(a, c->stream));
    return MURR_OK;
}

int murr_index_gather(murr_ctx_t* c, const murr_index_t* x, const uint8_t* q_data, const int32_t* q_offsets,
                      uint64_t nq, const uint8_t* blob, const uint64_t* row_off, uint8_t* out_data,
                      uint64_t out_cap, uint64_t* out_row_off, uint32_t* rows, uint64_t* needed) {
    murr_error_t* err = nullptr;
    // out_data == NULL: the first phase of a two-phase gather (lookup, sizes
    // and their scan; offsets unclamped, *needed exact), rows required
    const bool scan_only = out_data == nullptr;
    if (!c || !x || x->device != c->device || c->pending || !out_row_off ||
        (nq && (!q_data || !q_offsets || !row_off || (x->n && !blob))) || (scan_only && nq && (!rows || !needed)))
        return MURR_E_ARGUMENT;
    if (nq >= kMissing || ((uintptr_t)out_data & 15)) return MURR_E_ARGUMENT;
    HIPC(hipSetDevice(c->device));
    // scratch: the scan's group sums, then the rows when the caller wants none
    const uint64_t words = gather_scratch_words(nq);
    const uint64_t need = words + (rows ? 0 : (nq + 1) / 2);
    if (const int st = ensure_aux(c, need, err)) return st;
    IndexArgs a = index_args(x, q_data, q_offsets, nq);
    a.rows = rows ? rows : (uint32_t*)(c->aux + words);
    a.blob = blob;
    a.row_off = row_off;
    a.sizes = out_row_off;
    a.out = out_data;
    a.out_cap = out_cap;
    a.needed = needed;
    a.scratch = c->aux;
    if (const int st = scan_only ? MURR_OK : small_gather_words(c, &a, err)) return st;
    if (scan_only) {
        a.out_cap = ~0ull;
        HIPC(launch_gather_scan(a, c->stream));
    } else {
        HIPC(launch_gather(a, c->stream));  // probe included
    }
    return MURR_OK;
}

namespace {
// Peer access dev -> peer (kernels on dev dereference peer's memory over
// xGMI), enabled once per pair.
int enable_peer(int dev, int peer, murr_error_t* err) {
    if (dev == peer) return MURR_OK;
    static std::mutex mu;
    static std::set<std::pair<int, int>> done;
    std::lock_guard<std::mutex> g(mu);
    if (done.count({dev, peer})) return MURR_OK;
    HIPC(hipSetDevice(dev));
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
    else if (e != hipSuccess) return hip_fail(err, e);
    done.insert({dev, peer});
    return MURR_OK;
}

int multi_tab(murr_ctx_t* home, const murr_shard_read_t* shards, uint32_t nshards, uint64_t nq, MultiTab* t,
              murr_error_t* err) {
    if (!home || !shards || !nshards || nshards > kMaxShards || home->pending) return set_err(err, MURR_E_ARGUMENT);
    t->n = nshards;
    uint64_t prev = 0;
    for (uint32_t s = 0; s < nshards; s++) {
        const murr_shard_read_t& sh = shards[s];
        if (!sh.ctx || sh.q_end < prev || sh.q_end > nq || sh.ctx->pending ||
            (sh.index && (sh.index->device != sh.ctx->device || (sh.index->n && (!sh.arena || !sh.row_off)))))
            return set_err(err, MURR_E_ARGUMENT);
        t->arena[s] = sh.arena;
        t->row_off[s] = sh.row_off;
        t->q_end[s] = sh.q_end;
        prev = sh.q_end;
    }
    if (prev != nq) return set_err(err, MURR_E_ARGUMENT);
    return MURR_OK;
}
}  // namespace

int murr_multi_gather(murr_ctx_t* home, const murr_shard_read_t* shards, uint32_t nshards, const uint8_t* q_data,
                      const int32_t* q_offsets, const uint32_t* src, uint64_t nq, uint32_t* rows,
                      uint64_t* out_row_off, uint8_t* out_data, uint64_t out_cap, uint64_t* needed,
                      murr_error_t* err) {
    MultiTab t{};
    int st = multi_tab(home, shards, nshards, nq, &t, err);
    if (st) return st;
    if (!out_row_off || (nq && (!q_data || !q_offsets || !src || !rows)) || (!out_data && !needed) ||
        nq >= kMissing || ((uintptr_t)out_data & 15))
        return set_err(err, MURR_E_ARGUMENT);
    // 0. the lookups read q_data / q_offsets / src and write `rows`, all in
    //    home memory: a shard stream other than home's first waits for what
    //    the caller queued on the home stream before this call (the call is
    //    ordered on the home stream, as the header promises)
    bool home_marked = false;
    // 1. every shard looks up its queries on its own stream (all concurrently);
    //    the home stream waits for each shard's lookup, never the host
    uint64_t q0 = 0;
    for (uint32_t s = 0; s < nshards; s++) {
        const murr_shard_read_t& sh = shards[s];
        const uint64_t n = sh.q_end - q0;
        murr_ctx* sc = sh.ctx;
        if (n && sh.index && sh.index->n) {
            if ((st = enable_peer(sc->device, home->device, err))) return st;
            if (sc != home && !home_marked) {
                HIPC(hipSetDevice(home->device));
                if (!home->hev) HIPC(hipEventCreateWithFlags(&home->hev, hipEventDisableTiming));
                HIPC(hipEventRecord(home->hev, home->stream));
                home_marked = true;
            }
            HIPC(hipSetDevice(sc->device));
            if (sc != home) HIPC(hipStreamWaitEvent(sc->stream, home->hev, 0));
            IndexArgs a = index_args(sh.index, q_data, q_offsets + q0, n);
            a.rows = rows + q0;
            HIPC(launch_index_probe(a, sc->stream));
            if (sc != home) {
                if (!sc->xev) HIPC(hipEventCreateWithFlags(&sc->xev, hipEventDisableTiming));
                HIPC(hipEventRecord(sc->xev, sc->stream));
                HIPC(hipSetDevice(home->device));
                HIPC(hipStreamWaitEvent(home->stream, sc->xev, 0));
            }
        } else if (n) {  // nothing written to this shard yet: every key is missing
            HIPC(hipSetDevice(home->device));
            HIPC(hipMemsetAsync(rows + q0, 0xFF, 4 * n, home->stream));
        }
        q0 = sh.q_end;
    }
    // 2. on home: sizes in caller order, their scan, the rows copied from the
    //    shards' arenas (peer reads)
    for (uint32_t s = 0; s < nshards; s++)
        if ((st = enable_peer(home->device, shards[s].ctx->device, err))) return st;
    HIPC(hipSetDevice(home->device));
    if ((st = ensure_aux(home, gather_scan_groups(nq) + 1, err))) return st;
    IndexArgs a{};
    a.nq = nq;
    a.src = src;
    a.rows = rows;
    a.sizes = out_row_off;
    a.out = out_data;
    a.out_cap = out_data ? out_cap : ~0ull;
    a.needed = needed;
    a.scratch = home->aux;
    if (nq) HIPC(launch_multi_gather(a, t, out_data != nullptr, home->stream));
    else HIPC(hipMemsetAsync(out_row_off, 0, 8, home->stream));
    if (!nq && needed) HIPC(hipMemsetAsync(needed, 0, 8, home->stream));
    return MURR_OK;
}

int murr_multi_gather_copy(murr_ctx_t* home, const murr_shard_read_t* shards, uint32_t nshards, const uint32_t* src,
                           uint64_t nq, const uint32_t* rows, const uint64_t* out_row_off, uint8_t* out_data,
                           murr_error_t* err) {
    MultiTab t{};
    int st = multi_tab(home, shards, nshards, nq, &t, err);
    if (st) return st;
    if (nq && (!src || !rows || !out_row_off || !out_data || ((uintptr_t)out_data & 15)))
        return set_err(err, MURR_E_ARGUMENT);
    HIPC(hipSetDevice(home->device));
    IndexArgs a{};
    a.nq = nq;
    a.src = src;
    a.rows = const_cast<uint32_t*>(rows);
    a.sizes = const_cast<uint64_t*>(out_row_off);
    a.out = out_data;
    HIPC(launch_multi_copy(a, t, home->stream));
    return MURR_OK;
}

int murr_index_gather_copy(murr_ctx_t* c, const uint32_t* rows, uint64_t nq, const uint8_t* blob,
                           const uint64_t* row_off, const uint64_t* out_row_off, uint8_t* out_data) {
    murr_error_t* err = nullptr;
    if (!c || c->pending || (nq && (!rows || !row_off || !out_row_off || !out_data)) || nq >= kMissing ||
        ((uintptr_t)out_data & 15))
        return MURR_E_ARGUMENT;
    HIPC(hipSetDevice(c->device));
    IndexArgs a{};
    a.nq = nq;
    a.rows = const_cast<uint32_t*>(rows);
    a.blob = blob;
    a.row_off = row_off;
    a.sizes = const_cast<uint64_t*>(out_row_off);
    a.out = out_data;
    a.out_cap = ~0ull;
    HIPC(launch_gather_copy(a, c->stream));
    return MURR_OK;
}

uint32_t murr_abi_version(void) { return MURR_ABI_VERSION; }

const char* murr_status_str(int s) {
    switch (s) {
    case MURR_OK: return "ok";
    case MURR_E_INVALID_UTF8: return "invalid utf8";
    case MURR_E_DTYPE: return "dtype mismatch";
    case MURR_E_BAD_COLUMN: return "column not found";
    case MURR_E_OFFSET_OVERFLOW: return "byte array offset overflow";
    case MURR_E_MALFORMED_ROW: return "malformed row blob";
    case MURR_E_CAPACITY: return "output capacity too small";
    case MURR_E_ARGUMENT: return "invalid argument";
    case MURR_E_NULL_KEY: return "null in key column";
    case MURR_E_HIP: return "HIP runtime error";
    case MURR_E_INTERNAL: return "device protocol failure";
    case MURR_E_ARROW: return "arrow error";
    case MURR_E_NO_DEVICE: return "no HIP device";
    default: return "unknown";
    }
}

int murr_dtype_size(uint32_t dtype) { return dtype_size(dtype); }

int murr_segment_init(const uint32_t* dtypes, uint32_t ncols, murr_column_t* cols_out,
                      murr_segment_t* seg_out) {
    if ((ncols && (!dtypes || !cols_out)) || !seg_out) return MURR_E_ARGUMENT;
    uint32_t off = 0;
    for (uint32_t i = 0; i < ncols; i++) {
        int sz = dtype_size(dtypes[i]);
        if (sz < 0) return MURR_E_DTYPE;
        cols_out[i] = murr_column_t{i, dtypes[i], off, (uint32_t)sz};
        off += (uint32_t)sz;
    }
    seg_out->ncols = ncols;
    seg_out->bitset_size = (ncols + 7) / 8;
    seg_out->capacity = off;
    seg_out->_pad = 0;
    seg_out->cols = cols_out;
    return MURR_OK;
}

uint64_t murr_bitmap_bytes(uint64_t n) { return round_up((n + 7) / 8, 8); }

int murr_device_count(int* n) {
    int k = 0;
    hipError_t e = hipGetDeviceCount(&k);
    if (n) *n = (e == hipSuccess) ? k : 0;
    return e == hipSuccess ? MURR_OK : MURR_E_NO_DEVICE;
}

int murr_ctx_create(int device, murr_ctx_t** out) {
    if (!out) return MURR_E_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return MURR_E_NO_DEVICE;
    if (device < 0 || device >= n) return MURR_E_ARGUMENT;
    murr_ctx* c = new (std::nothrow) murr_ctx();
    if (!c) return MURR_E_INTERNAL;
    c->device = device;
    murr_error_t* err = nullptr;
    HIPC(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPC(hipGetDeviceProperties(&prop, device));
    c->cus = prop.multiProcessorCount;
    // Persistent grid: blocks that are certainly co-resident (one below the
    // occupancy answer: MI355X_MICROARCH.md "Residency"), at least one per CU.
    c->enc_grid_per_cu = std::max(1, std::min(8, encode_blocks_per_cu()) - 1);
#ifdef MURR_TUNING
    opts_from_env(&c->opts);  // tuning builds only: once, at creation
#endif
    HIPC(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPC(hipEventCreate(&c->k0));
    HIPC(hipEventCreate(&c->k1));
    *out = c;
    return MURR_OK;
}

void murr_ctx_destroy(murr_ctx_t* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    {
        std::lock_guard<std::mutex> lk(g_dc_mu);
        for (const auto& f : c->dfree) (void)hipFree(f.second);
        for (auto it = g_dcached.begin(); it != g_dcached.end();)  // (outstanding ones: plain buffers from now on)
            it = it->second.first == c ? g_dcached.erase(it) : std::next(it);
    }
    if (c->ws) (void)hipFree(c->ws);
    if (c->aux) (void)hipFree(c->aux);
    if (c->glb) (void)hipFree(c->glb);
    if (c->hs) (void)hipHostFree(c->hs);
    for (const auto& b : c->pool) (void)(b.pinned ? hipHostFree(b.p) : hipFree(b.p));
    for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
    if (c->xev) (void)hipEventDestroy(c->xev);
    if (c->hev) (void)hipEventDestroy(c->hev);
    if (c->k0) (void)hipEventDestroy(c->k0);
    if (c->k1) (void)hipEventDestroy(c->k1);
    for (hipEvent_t e : c->mk)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

void* murr_ctx_stream(murr_ctx_t* c) { return c ? (void*)c->stream : nullptr; }

int murr_ctx_last_kernel_ms(murr_ctx_t* c, float* ms) {
    murr_error_t* err = nullptr;
    if (!c || !ms) return MURR_E_ARGUMENT;
    if (!c->timed) { *ms = 0.f; return MURR_OK; }
    hipEvent_t e0 = c->lk0 ? c->lk0 : c->k0, e1 = c->lk1 ? c->lk1 : c->k1;
    HIPC(hipEventSynchronize(e1));
    HIPC(hipEventElapsedTime(ms, e0, e1));
    return MURR_OK;
}

const char* murr_ctx_last_kernel(murr_ctx_t* c) { return c ? c->last_kernel : ""; }

int murr_ctx_mark(murr_ctx_t* c, uint32_t which) {
    murr_error_t* err = nullptr;
    if (!c || which >= 4) return MURR_E_ARGUMENT;
    HIPC(hipSetDevice(c->device));
    if (!c->mk[which]) HIPC(hipEventCreate(&c->mk[which]));
    HIPC(hipEventRecord(c->mk[which], c->stream));
    return MURR_OK;
}

int murr_ctx_mark_ms(murr_ctx_t* ca, uint32_t a, murr_ctx_t* cb, uint32_t b, float* ms) {
    murr_error_t* err = nullptr;
    if (!ca || !cb || !ms || a >= 4 || b >= 4 || !ca->mk[a] || !cb->mk[b] || ca->device != cb->device)
        return MURR_E_ARGUMENT;
    HIPC(hipEventSynchronize(cb->mk[b]));
    HIPC(hipEventElapsedTime(ms, ca->mk[a], cb->mk[b]));
    return MURR_OK;
}

int murr_ctx_set_opts(murr_ctx_t* c, const murr_opts_t* o) {
    if (!c || !o || o->kernel > 2 || o->mode > 3 || o->encode_kernel > 2 || (!o->shape_nw) != (!o->shape_r) ||
        o->reserved)
        return MURR_E_ARGUMENT;
    c->opts = *o;
    return MURR_OK;
}

int murr_ctx_get_opts(murr_ctx_t* c, murr_opts_t* o) {
    if (!c || !o) return MURR_E_ARGUMENT;
    *o = c->opts;
    return MURR_OK;
}

int murr_jit_cache_limit(uint32_t max_layouts, uint32_t* limit, uint32_t* cached) {
    const size_t l = jit_layout_limit(max_layouts);
    if (limit) *limit = (uint32_t)l;
    if (cached) *cached = (uint32_t)jit_layout_cached();
    return MURR_OK;
}

int murr_ctx_stats(murr_ctx_t* c, murr_ctx_stats_t* out) {
    if (!c || !out) return MURR_E_ARGUMENT;
    *out = c->stats;
    return MURR_OK;
}

int murr_dev_alloc(murr_ctx_t* c, uint64_t bytes, void** p) {
    murr_error_t* err = nullptr;
    if (!c || !p) return MURR_E_ARGUMENT;
    HIPC(hipSetDevice(c->device));
    // Rounded up and padded so 16-B staging loads of the last chunk stay inside.
    HIPC(hipMalloc(p, round_up(bytes ? bytes : 1, 16) + 16));
    dev_forget(*p);
    return MURR_OK;
}

int murr_dev_free(murr_ctx_t* c, void* p) {
    murr_error_t* err = nullptr;
    if (!c) return MURR_E_ARGUMENT;
    if (p && !dev_free_cached(c, p)) HIPC(hipFree(p));
    return MURR_OK;
}

int murr_host_alloc(murr_ctx_t* c, uint64_t bytes, void** p) {
    murr_error_t* err = nullptr;
    if (!c || !p) return MURR_E_ARGUMENT;
    HIPC(hipHostMalloc(p, round_up(bytes ? bytes : 1, 16) + 16, hipHostMallocDefault));
    return MURR_OK;
}

int murr_host_free(murr_ctx_t* c, void* p) {
    murr_error_t* err = nullptr;
    (void)c;
    if (p) HIPC(hipHostFree(p));
    return MURR_OK;
}

int murr_memcpy_h2d(murr_ctx_t* c, void* dst, const void* src, uint64_t n) {
    murr_error_t* err = nullptr;
    if (!c) return MURR_E_ARGUMENT;
    if (!n) return MURR_OK;
    HIPC(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return MURR_OK;
}

int murr_memcpy_d2h(murr_ctx_t* c, void* dst, const void* src, uint64_t n) {
    murr_error_t* err = nullptr;
    if (!c) return MURR_E_ARGUMENT;
    if (!n) return MURR_OK;
    HIPC(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return MURR_OK;
}

int murr_memcpy_d2d(murr_ctx_t* c, void* dst, const void* src, uint64_t n) {
    murr_error_t* err = nullptr;
    if (!c) return MURR_E_ARGUMENT;
    if (!n) return MURR_OK;
    HIPC(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return MURR_OK;
}

int murr_row_off_narrow(murr_ctx_t* c, const uint64_t* row_off, uint64_t n_rows, uint32_t* out) {
    murr_error_t* err = nullptr;
    if (!c || !row_off || !out || ((uintptr_t)out & 3) || c->pending) return MURR_E_ARGUMENT;
    HIPC(hipSetDevice(c->device));
    // the kernel checks every offset (a malformed block's interior
    // offset past 2^32 or below its predecessor is an error, never truncated);
    // its flag word comes back with one 4-byte read-back
    int st = ensure_ws(c, 64, err);
    if (st) return st;
    st = ensure_hs(c, 64, err);
    if (st) return st;
    unsigned int* bad = (unsigned int*)c->ws;
    HIPC(hipMemsetAsync(bad, 0, 4, c->stream));
    HIPC(launch_row_off_narrow(row_off, out, n_rows + 1, bad, c->stream));
    HIPC(hipMemcpyAsync(c->hs, bad, 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    const unsigned int f = *(const volatile unsigned int*)c->hs;
    if (f & 1u) return MURR_E_OFFSET_OVERFLOW;
    if (f & 2u) return MURR_E_MALFORMED_ROW;
    return MURR_OK;
}

int murr_memcpy_peer(murr_ctx_t* c, void* dst, const void* src, int src_device, uint64_t n) {
    murr_error_t* err = nullptr;
    if (!c) return MURR_E_ARGUMENT;
    if (!n) return MURR_OK;
    HIPC(hipSetDevice(c->device));
    if (src_device == c->device) HIPC(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, c->stream));
    else HIPC(hipMemcpyPeerAsync(dst, c->device, src, src_device, n, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return MURR_OK;
}

int murr_shard_of(const uint8_t* key_data, const int32_t* key_offsets, uint64_t key_offset, uint64_t n,
                  uint32_t nshards, uint32_t* out) {
    if (!nshards || (n && (!key_offsets || !out))) return MURR_E_ARGUMENT;
    for (uint64_t i = 0; i < n; i++) {
        const int32_t a = key_offsets[key_offset + i], b = key_offsets[key_offset + i + 1];
        if (b < a || (b > a && !key_data)) return MURR_E_ARGUMENT;
        uint64_t h = 0xcbf29ce484222325ull;
        for (int32_t k = a; k < b; k++) h = (h ^ key_data[k]) * 0x100000001b3ull;
        h ^= h >> 33;
        h *= 0xff51afd7ed558ccdull;
        h ^= h >> 33;
        h *= 0xc4ceb9fe1a85ec53ull;
        h ^= h >> 33;
        out[i] = (uint32_t)(h % nshards);
    }
    return MURR_OK;
}

int murr_memset_dev(murr_ctx_t* c, void* dst, int v, uint64_t n) {
    murr_error_t* err = nullptr;
    if (!c) return MURR_E_ARGUMENT;
    if (!n) return MURR_OK;
    HIPC(hipMemsetAsync(dst, v, n, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return MURR_OK;
}

int murr_sync(murr_ctx_t* c) {
    murr_error_t* err = nullptr;
    if (!c) return MURR_E_ARGUMENT;
    HIPC(hipStreamSynchronize(c->stream));
    return MURR_OK;
}

// ---- decode ------------------------------------------------------------------

namespace {
// Copy-kernel grids: reads from pinned host memory saturate PCIe with 64
// workgroups (more queue up behind the link), writes with 128.
#ifdef MURR_TUNING
uint32_t copy_grid(const char* name, uint32_t dflt) {
    const char* e = std::getenv(name);
    return e ? (uint32_t)std::max(1, std::atoi(e)) : dflt;
}
const uint32_t kCopyGridIn = copy_grid("MURR_COPY_GRID_IN", 64), kCopyGridOut = copy_grid("MURR_COPY_GRID_OUT", 128);
#else
constexpr uint32_t kCopyGridIn = 64, kCopyGridOut = 128;
#endif

// A decode's descriptor upload (c->hs -> dst): one hipMemcpyAsync, or (fused
// transfers) one segment-copy kernel together with the batch's input.
hipError_t upload_desc(murr_ctx* c, uint8_t* dst, uint64_t bytes) {
    if (!c->xfer) return hipMemcpyAsync(dst, c->hs, bytes, hipMemcpyHostToDevice, c->stream);
    c->xin.push_back(CopySeg{c->hs, dst, bytes, nullptr});
    hipError_t e = c->xtimed ? hipEventRecord(c->xe[0], c->stream) : hipSuccess;
    if (e == hipSuccess) e = launch_copy_segs(c->xin.data(), (uint32_t)c->xin.size(), kCopyGridIn, c->stream);
    if (e == hipSuccess && c->xtimed) e = hipEventRecord(c->xe[1], c->stream);
    c->xin.clear();
    return e;
}
// Its counter read-back (c->ws -> c->hs + rb): one hipMemcpyAsync, or (fused
// transfers) one segment-copy kernel together with the decoded buffers.
hipError_t read_back(murr_ctx* c, uint64_t rb, uint64_t bytes) {
    if (!c->xfer) return hipMemcpyAsync(c->hs + rb, c->ws, bytes, hipMemcpyDeviceToHost, c->stream);
    c->xout.insert(c->xout.begin(), CopySeg{c->ws, c->hs + rb, bytes, nullptr});
    hipError_t e = c->xtimed ? hipEventRecord(c->xe[2], c->stream) : hipSuccess;
    if (e == hipSuccess) e = launch_copy_segs(c->xout.data(), (uint32_t)c->xout.size(), kCopyGridOut, c->stream);
    if (e == hipSuccess && c->xtimed) e = hipEventRecord(c->xe[3], c->stream);
    c->xout.clear();
    return e;
}
// Kernel timing events: always, except untimed fused-transfer batches.
bool kernel_events(const murr_ctx* c) { return !c->xfer || c->xtimed; }
}  // namespace

namespace {

// After an enqueue: what murr_decode_wait needs to fill the counts.
int pending_set(murr_ctx* c, murr_array_t* outs, const murr_block_t* blocks, uint32_t nblocks, uint32_t nproj,
                const std::vector<DecProj>& dp, uint64_t rb) {
    c->pending = true;
    c->outs = outs;
    c->nblocks = nblocks;
    c->nproj = nproj;
    c->rb_off = rb;
    c->n_rows.resize(nblocks);
    for (uint32_t b = 0; b < nblocks; b++) c->n_rows[b] = blocks[b].n_rows;
    c->dtypes.resize(nproj);
    for (uint32_t p = 0; p < nproj; p++) c->dtypes[p] = dp[p].dtype;
    return MURR_OK;
}

// A utf8 index stride: a power of two in [64, 2^30].
bool stride_ok(uint64_t s) { return s >= 64 && s <= (1ull << 30) && (s & (s - 1)) == 0; }

// A prepared launch of the specialised decode (murr_decode_plan): its own
// device workspace holding the descriptors (uploaded once), the kernel
// arguments per projection round, and a pinned readback buffer.  A run zeroes
// the counters, launches, reads back the counts: no host-side preparation and
// no descriptor upload per launch.
constexpr uint64_t kTimeEvery = MURR_PLAN_TIME_EVERY;  // prepared plans: one timed run in four

struct JitReplay {
    uint8_t* dws = nullptr;        // device workspace: [counter set 0 | descriptors | sink]
    uint8_t* zb2 = nullptr;        // counter set 1 (runs alternate; each launch zeroes the other set)
    uint8_t* hrb = nullptr;        // pinned readback (z_lb bytes) + done flag
    uint8_t* hrb_dev = nullptr;    // its device address
    uint64_t zbytes = 0, z_lb = 0;
    uint64_t runs = 0, timed_runs = 0;
    std::vector<std::vector<uint8_t>> kargs[2];  // per counter set: per projection round
    JitShapeK K{};
    bool split = false, emit = false;
    uint32_t grid = 0, lds = 0, mode = 0;
    std::vector<int32_t*> empty_offsets;  // utf8 offsets of empty blocks: [0] = 0 per run
    // Timing: every kTimeEvery-th run (the first included) is bracketed by
    // e0/t1, the others end with e1 only -- an event recorded between
    // back-to-back launches costs ~4 us of GPU time (D shard: 0.0810 vs
    // 0.0766 ms per run, profiles/r04/probes/ab40.txt).
    hipEvent_t e0 = nullptr, t1 = nullptr, e1 = nullptr;
    hipEvent_t end = nullptr;               // the in-flight run's last event (t1 or e1)
    bool inflight = false;                  // murr_decode_run_async issued, murr_decode_run_wait not yet
    int set = 0;                            // the in-flight run's counter set
    void release() {
        if (dws) (void)hipFree(dws);
        if (zb2) (void)hipFree(zb2);
        if (hrb) (void)hipHostFree(hrb);
        if (e0) (void)hipEventDestroy(e0);
        if (t1) (void)hipEventDestroy(t1);
        if (e1) (void)hipEventDestroy(e1);
        dws = zb2 = hrb = nullptr;
        e0 = t1 = e1 = end = nullptr;
    }
};

// The layout-specialised decode (murr_jit_kernel.hip).  Tile shape from the
// mean row size.  Local mode (a workgroup owns whole blocks) when the blocks
// fill the co-resident grid; or, when every block can be cut (it has a utf8
// index, or the layout has no utf8 column), local mode over virtual blocks
// of a few tiles, each starting at its index entry; else split mode
// (segments, two passes, decoupled look-back).  A projection naming a column
// twice runs one launch per occurrence round (the later rounds only fill the
// duplicate outputs, so they report no errors).
int decode_enqueue_jit(murr_ctx* c, const murr_segment_t* seg, const JitLayout* jl, const uint32_t* proj,
                       uint32_t nproj, const murr_block_t* blocks, uint32_t nblocks, murr_array_t* outs,
                       const std::vector<DecProj>& dp, double est_row, bool force_local = false,
                       const uint64_t* const* uidx = nullptr, uint32_t stride = 0, JitReplay* rep = nullptr) {
    murr_error_t* err = nullptr;
    const murr_opts_t& O = c->opts;
    const bool verbose = O.verbose != 0;
    uint32_t nu_layout = 0;
    for (uint32_t i = 0; i < seg->ncols; i++) nu_layout += seg->cols[i].dtype == MURR_UTF8;
    const uint32_t nu = std::max<uint32_t>(nu_layout, 1);
    // Shape: 5 waves x 3 chunks (768 rows) when its two LDS slots fit 40 KiB
    // with 15 % slack over the mean row (four workgroups per CU; config B 0.62
    // -> 0.65 against 5 x 2: the per-tile overheads spread over more rows);
    // else 5 x 2 (512 rows) within the same 40 KiB; else 3 x 1 (128 rows)
    // when that fits 40 KiB with 8 % slack (four or five per CU: config C
    // 0.51 -> 0.54 against 5 x 1 at two per CU); else 5 x 1 (256 rows) within
    // 64 KiB; else 3 x 1.
    auto lds_for = [&](uint32_t s, double slack) {
        const JitShapeK& k = jl->shapes[s];
        const uint32_t st = (uint32_t)round_up((uint64_t)(k.tr * est_row * slack) + 64, 1024);
        return jit_lds_bytes(k.nw, k.r, k.nslot, st, nu_layout);
    };
    uint32_t si = 2;
    double slack = 1.08;
    uint32_t budget = 65536;
    if (lds_for(3, 1.15) <= 40960) { si = 3; slack = 1.15; budget = 40960; }
    else if (lds_for(0, 1.15) <= 40960) { si = 0; slack = 1.15; budget = 40960; }
    else if (lds_for(2, 1.08) <= 40960) { si = 2; budget = 40960; }
    else if (lds_for(1, 1.08) <= 65536) si = 1;
    if (O.shape_nw)
        for (uint32_t s = 0; s < kJitShapes; s++)
            if (jl->shapes[s].nw == O.shape_nw && jl->shapes[s].r == O.shape_r) si = s;
    if (O.lds_budget) budget = O.lds_budget;
    const JitShapeK& K = jl->shapes[si];
    const uint32_t smax = std::max<uint32_t>(
        1024, ((budget - std::min(budget, jit_lds_bytes(K.nw, K.r, K.nslot, 0, nu_layout))) / K.nslot) & ~1023u);
    uint32_t stage = (uint32_t)std::min<uint64_t>(round_up((uint64_t)(K.tr * est_row * slack) + 64, 1024), smax);
    if (O.stage) stage = (uint32_t)round_up(O.stage, 1024);
    const uint32_t lds = jit_lds_bytes(K.nw, K.r, K.nslot, stage, nu_layout);

    // Workgroups per CU: the occupancy answer, never above the LDS bound.
    // Stream mode needs the whole grid resident at once (workgroups wait on
    // each other's tiles), and the API over-counts when SGPRs bind, so its
    // grid also respects a worst-case register bound: 106 SGPRs allow 6 waves
    // per SIMD (MI355X_MICROARCH.md, residency), the VGPR count allows
    // 512 / alloc, and a 5-wave workgroup may put 2 waves on one SIMD.
    // (the occupancy and register queries are cached per kernel and LDS size:
    // each is a runtime call that costs microseconds on every launch)
    // (keyed on the shape's uid: a module the JIT cache unloaded may leave its
    // function address to a later one, which must not inherit its answers)
    auto occupancy = [&](hipFunction_t fn, bool split) {
        static std::mutex mu;
        static std::map<std::pair<uint64_t, uint32_t>, int> cache;
        const std::pair<uint64_t, uint32_t> key{2 * K.uid + (split ? 1 : 0), lds};
        int n = 0;
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = cache.find(key);
            if (it != cache.end()) n = it->second;
        }
        if (!n) {
            if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 64 * K.nw, lds) != hipSuccess || n < 1) n = 1;
            std::lock_guard<std::mutex> g(mu);
            cache[key] = n;
        }
        return std::min<int>(n, std::max<int>(1, (int)(163840 / std::max<uint32_t>(lds, 1))));
    };
    const int bpc = occupancy(K.fn, false);
    int bpc_safe = occupancy(K.fn_split, true);
    {
        static std::mutex mu;
        static std::map<uint64_t, int> regs;
        int vgprs = 0;
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = regs.find(K.uid);
            if (it != regs.end()) vgprs = it->second;
        }
        if (!vgprs) {
            if (hipFuncGetAttribute(&vgprs, HIP_FUNC_ATTRIBUTE_NUM_REGS, K.fn_split) != hipSuccess || vgprs < 1) vgprs = 128;
            std::lock_guard<std::mutex> g(mu);
            regs[K.uid] = vgprs;
        }
        const int alloc = (vgprs + 7) / 8 * 8;
        const int per_simd = std::min(std::min(8, 512 / alloc), 6);
        const int waves_per_simd_per_wg = (int)(K.nw + 3) / 4;
        bpc_safe = std::max(1, std::min(bpc_safe, per_simd / waves_per_simd_per_wg));
    }
    const uint64_t G = (uint64_t)c->cus * bpc;

    std::vector<DecBlock> db(nblocks);
    uint64_t tiles = 0, nonempty = 0, total_rows = 0;
    bool cuttable = true;  // every block can be cut into virtual blocks
    for (uint32_t b = 0; b < nblocks; b++) {
        const uint64_t* ux = uidx ? uidx[b] : nullptr;
        db[b] = dec_block(blocks[b], tiles, ux);
        tiles += (blocks[b].n_rows + K.tr - 1) / K.tr;
        nonempty += blocks[b].n_rows != 0;
        total_rows += blocks[b].n_rows;
        cuttable &= nu_layout == 0 || ux != nullptr || blocks[b].n_rows == 0;
    }
    // local mode when whole blocks keep >= 75 % of the grid busy
    bool local = false, cut = false;
    if (nonempty) {
        const uint64_t rounds = (nonempty + G - 1) / G;
        local = nonempty * 4 >= rounds * G * 3;
        if (!local && cuttable && stride_ok(nu_layout ? stride : 64)) local = cut = true;
        // mode 3: cut whenever possible (whole blocks may leave workgroup slots idle)
        if (O.mode == 3 && cuttable && stride_ok(nu_layout ? stride : 64)) local = cut = true;
    }
    if (O.mode == 1 || O.mode == 2) {
        local = O.mode == 1;
        cut = cut && local;
    }
    if (force_local) local = true;
    // (virtual) blocks of local mode: whole blocks, or cuts every V rows (a
    // multiple of the index stride, about 8 per workgroup for balance)
    std::vector<JitSeg> lsegs;
    uint64_t vrows = 0;  // rows per virtual block (cut mode)
    if (local) {
        const uint64_t S = nu_layout ? std::max<uint32_t>(stride, 1) : K.tr;  // (stride checked when cut)
        uint64_t V = std::max<uint64_t>(K.tr, (total_rows + 8 * G - 1) / (8 * G));
        V = (V + S - 1) / S * S;
        if (O.vrows) V = std::max<uint64_t>(S, (uint64_t)O.vrows / S * S);
        vrows = V;
        for (uint32_t b = 0; b < nblocks; b++) {
            const uint64_t n = blocks[b].n_rows;
            if (!n) continue;
            if (!cut) lsegs.push_back(JitSeg{b, 0, 0, n});
            else
                for (uint64_t r = 0; r < n; r += V) lsegs.push_back(JitSeg{b, 0, r, std::min(n, r + V)});
        }
    }
    // Split mode: segments of seg_tiles tiles dealt round-robin over a
    // co-resident grid; a grid round of segments (the distance between a
    // segment's two passes) is kept near 96 MiB so the second pass still
    // finds it in the Infinity Cache.
    const uint64_t G_split = (uint64_t)c->cus * bpc_safe;
    // segment tiles: the launch's tiles over whole grid rounds of <= 96 MiB
    const double tile_in = K.tr * (est_row + 8.0);
    const uint64_t grid_rounds = std::max<uint64_t>(1, (uint64_t)std::ceil(tiles * tile_in / 100663296.0));
    uint64_t seg_tiles = std::max<uint64_t>(1, (tiles + grid_rounds * G_split - 1) / (grid_rounds * G_split));
    if (O.seg_tiles) seg_tiles = O.seg_tiles;
    std::vector<JitSeg> jsegs;
    if (!local) {
        for (uint32_t b = 0; b < nblocks; b++) {
            const uint64_t n = blocks[b].n_rows, seg_rows = seg_tiles * K.tr;
            const uint32_t first = (uint32_t)jsegs.size();
            for (uint64_t r = 0; r < n; r += seg_rows) jsegs.push_back(JitSeg{b, first, r, std::min(n, r + seg_rows)});
        }
    }
    const uint64_t nseg = jsegs.size();
    // Local mode: the co-resident grid walks the (virtual) blocks g, g + G, ...;
    // opts.grid ~0 launches one workgroup per (virtual) block instead, so the
    // hardware hands the next one to whichever CU frees a slot first.
    uint64_t grid_local = std::min<uint64_t>(G, lsegs.size());
    if (O.grid == 0xFFFFFFFFu) grid_local = lsegs.size();
    else if (O.grid) grid_local = std::min<uint64_t>(O.grid, lsegs.size());
    const uint64_t grid = std::max<uint64_t>(1, local ? grid_local : std::min<uint64_t>(G_split, nseg));
    // Cut mode: neighbouring virtual blocks share output lines (a 128-row
    // piece of a validity bitmap is 16 B of a 128-B line, a string run's ends
    // are partial lines).  Dealt g, g + G, ... in index order, the eight
    // pieces of a line came from eight XCDs (workgroup g runs on XCD g % 8),
    // each L2 writing its piece back as a partial line.  Runs of eight
    // consecutive virtual blocks go to workgroups of one XCD instead, so a
    // line's pieces meet in one L2.
    uint32_t xorder = cut && grid % 8 == 0 && lsegs.size() >= 64 && vrows < 1024 ? 1u : 0u;
#ifdef MURR_TUNING
    // 0 index order, 1 runs of 8 round-robin over the XCDs, 2 the same runs
    // with each 8 runs' XCDs in a pseudo-random order
    if (const char* e = std::getenv("MURR_XORDER")) xorder = xorder ? (uint32_t)std::atoi(e) : 0u;
#endif
    uint64_t xrun = 8;  // virtual blocks per run
#ifdef MURR_TUNING
    if (const char* e = std::getenv("MURR_XRUN")) xrun = std::max(1, std::atoi(e));
#endif
    if (xorder) {
        const uint64_t nv = lsegs.size();
        std::vector<std::vector<uint64_t>> pos(8), vb(8);
        for (uint64_t p = 0; p < nv; p++) pos[(p % grid) % 8].push_back(p);
        uint32_t perm[8] = {0, 1, 2, 3, 4, 5, 6, 7};
        for (uint64_t k = 0; k < nv; k++) {
            const uint64_t m = k / xrun;
            if (xorder == 2 && k % (8 * xrun) == 0) {
                std::mt19937 rng((uint32_t)(m * 2654435761u + 12345u));
                std::shuffle(perm, perm + 8, rng);
            }
            vb[xorder == 2 ? perm[m % 8] : m % 8].push_back(k);
        }
        std::vector<JitSeg> out(nv);
        std::vector<uint64_t> free_pos, free_vb;
        for (uint32_t x = 0; x < 8; x++) {
            const size_t m = std::min(pos[x].size(), vb[x].size());
            for (size_t i = 0; i < m; i++) out[pos[x][i]] = lsegs[vb[x][i]];
            free_pos.insert(free_pos.end(), pos[x].begin() + m, pos[x].end());
            free_vb.insert(free_vb.end(), vb[x].begin() + m, vb[x].end());
        }
        std::sort(free_pos.begin(), free_pos.end());
        std::sort(free_vb.begin(), free_vb.end());
        for (size_t i = 0; i < free_pos.size(); i++) out[free_pos[i]] = lsegs[free_vb[i]];
        lsegs.swap(out);
    }
    bool emit = false;
    for (uint32_t p = 0; p < nproj; p++) emit |= dp[p].is_utf8;

    // projection rounds: round r decodes the r-th occurrence of every column
    std::vector<std::vector<uint32_t>> occ(seg->ncols);
    for (uint32_t p = 0; p < nproj; p++) occ[proj[p]].push_back(p);
    uint32_t rounds = 1;
    for (const auto& v : occ) rounds = std::max<uint32_t>(rounds, (uint32_t)v.size());
    const uint32_t ncols = seg->ncols, npad = (ncols + 1) & ~1u;

    std::vector<DecOut> dout((uint64_t)nblocks * nproj);
    for (uint64_t i = 0; i < dout.size(); i++)
        dout[i] = DecOut{(uint8_t*)outs[i].values, outs[i].validity, outs[i].offsets, outs[i].values_cap};

    const uint64_t nbp = (uint64_t)nblocks * nproj;
    // granules per projection round, then the round's segment claim word
    const uint64_t flag_bytes = local || !emit ? 0 : round_up(8 * nu * nseg + 8, 16);
    const uint64_t z_err = 0, z_nulls = kErrBytes, z_lens = z_nulls + 8 * nbp, z_flags = round_up(z_lens + 8 * nbp, 16);
    const uint64_t zbytes = round_up(z_flags + flag_bytes * rounds, 16);
    const uint64_t d_blocks = zbytes;
    const uint64_t d_outs = round_up(d_blocks + sizeof(DecBlock) * nblocks, 16);
    const std::vector<JitSeg>& segs_out = local ? lsegs : jsegs;
    const uint64_t d_segs = round_up(d_outs + sizeof(DecOut) * dout.size(), 16);
    const uint64_t d_slots = round_up(d_segs + sizeof(JitSeg) * segs_out.size(), 16);
    const uint64_t d_projc = round_up(d_slots + 2 * (uint64_t)npad * rounds, 16);
    const uint64_t d_sink = round_up(d_projc + 2 * (uint64_t)nproj, 256);
#ifdef MURR_TUNING
    const uint64_t tl_bytes = 32 * grid;  // a stamped build's timeline (MJ_TIMELINE writes it to the sink)
#else
    const uint64_t tl_bytes = 0;
#endif
    const uint64_t dend = d_sink + std::max<uint64_t>(1024, tl_bytes);
    int st = MURR_OK;
    uint8_t* ws = nullptr;
    if (rep) {
        HIPC(hipMalloc(&rep->dws, dend));
        HIPC(hipMalloc(&rep->zb2, zbytes));
        HIPC(hipMemsetAsync(rep->zb2, 0, zbytes, c->stream));
        // read-back + done flag, written by the kernel's epilogue: coherent
        // (fine-grained) pinned memory the device writes over PCIe
        HIPC(hipHostMalloc(&rep->hrb, round_up(z_flags, 64) + 64, hipHostMallocMapped | hipHostMallocCoherent));
        HIPC(hipHostGetDevicePointer((void**)&rep->hrb_dev, rep->hrb, 0));
        ws = rep->dws;
    } else {
        st = ensure_ws(c, dend, err);
        if (st) return st;
        ws = c->ws;
    }
    const uint64_t z_lb = z_flags;  // readback: error word, stamps, nulls, lens
    const uint64_t hz = zbytes <= 65536 ? zbytes : 0;
    const uint64_t hdesc = d_sink - zbytes, rb = round_up(hz + hdesc, 64);
    st = ensure_hs(c, rb + z_lb, err);
    if (st) return st;
    uint8_t* hd = c->hs + hz;
    if (hz) std::memset(c->hs, 0, hz);
    std::memcpy(hd + (d_blocks - zbytes), db.data(), sizeof(DecBlock) * nblocks);
    std::memcpy(hd + (d_outs - zbytes), dout.data(), sizeof(DecOut) * dout.size());
    if (!segs_out.empty()) std::memcpy(hd + (d_segs - zbytes), segs_out.data(), sizeof(JitSeg) * segs_out.size());
    std::vector<uint16_t> slots((uint64_t)npad * rounds, 0xFFFF);
    for (uint32_t col = 0; col < ncols; col++)
        for (uint32_t r = 0; r < occ[col].size(); r++) slots[(uint64_t)r * npad + col] = (uint16_t)occ[col][r];
    std::memcpy(hd + (d_slots - zbytes), slots.data(), 2 * slots.size());
    for (uint32_t p = 0; p < nproj; p++) ((uint16_t*)(hd + (d_projc - zbytes)))[p] = (uint16_t)proj[p];

    if (!hz) HIPC(hipMemsetAsync(ws, 0, zbytes, c->stream));
    if (rep) {
        HIPC(hipMemcpyAsync(ws + zbytes - hz, c->hs, hz + hdesc, hipMemcpyHostToDevice, c->stream));
        HIPC(hipStreamSynchronize(c->stream));  // c->hs is reused by the next call
    } else {
        HIPC(upload_desc(c, ws + zbytes - hz, hz + hdesc));
    }
    // Empty blocks: utf8 offsets = [0] (StringBuilder starts with offset 0).
    for (uint32_t b = 0; b < nblocks; b++)
        if (blocks[b].n_rows == 0)
            for (uint32_t p = 0; p < nproj; p++)
                if (dp[p].is_utf8 && outs[(uint64_t)b * nproj + p].offsets) {
                    if (rep) rep->empty_offsets.push_back(outs[(uint64_t)b * nproj + p].offsets);
                    else HIPC(hipMemsetAsync(outs[(uint64_t)b * nproj + p].offsets, 0, 4, c->stream));
                }

    std::vector<uint8_t> karg(round_up(sizeof(JitArgsHead) + 2 * (uint64_t)npad, 8), 0);
    JitArgsHead h{};
    h.blocks = (const DecBlock*)(ws + d_blocks);
    h.outs = (const DecOut*)(ws + d_outs);
    h.order = nullptr;
    h.segs = (const JitSeg*)(ws + d_segs);
    h.projcols = (const uint16_t*)(ws + d_projc);
    h.nulls = (unsigned long long*)(ws + z_nulls);
    h.lens = (unsigned long long*)(ws + z_lens);
    h.err = (unsigned long long*)(ws + z_err);
    h.sink = ws + d_sink;
    h.nseg = nseg;
    h.emit = emit;
    h.nblocks = nblocks;
    h.nproj = nproj;
    h.norder = (uint32_t)lsegs.size();
    h.ulog = cut && nu_layout ? (uint32_t)__builtin_ctzll(stride) : 0;
    h.mode = local ? 0 : 1;
    h.stage = stage;
    h.fast = cut || !local ? 1u : 0u;
    if (verbose)
        std::fprintf(stderr, "decode launch (jit %ux%us%u): %s grid %llu (%d/CU, %d split) blocks %llu tiles %llu segments %llu (%llu tiles) rows/tile %u stage %u lds %u rounds %u fast %u\n",
                     K.nw, K.r, K.nslot, cut ? "local-cut" : local ? "local" : "split", (unsigned long long)grid, bpc, bpc_safe,
                     (unsigned long long)(local ? lsegs.size() : nonempty),
                     (unsigned long long)tiles, (unsigned long long)nseg, (unsigned long long)seg_tiles, K.tr, stage, lds, rounds,
                     h.fast);
#ifdef MURR_TUNING
    c->tl_off = rep ? 0 : d_sink;
    c->tl_n = grid;
    if (tl_bytes) HIPC(hipMemsetAsync(ws + d_sink, 0, tl_bytes, c->stream));
#endif
    if (rep) {
        rep->zbytes = zbytes;
        rep->z_lb = z_lb;
        rep->K = K;
        rep->split = !local;
        rep->emit = emit;
        rep->grid = (uint32_t)grid;
        rep->lds = lds;
        rep->mode = cut ? 2u : local ? 1u : 3u;
    } else if (kernel_events(c)) {
        HIPC(hipEventRecord(c->k0, c->stream));
    }
    if (tiles) {
        for (uint32_t r = 0; r < rounds; r++) {
            h.slot_tab = (const uint16_t*)(ws + d_slots + 2 * (uint64_t)npad * r);
            h.abort_word = local || !emit ? nullptr : (unsigned int*)(ws + 8);  // read back beside the error word
            h.flags = (unsigned long long*)(ws + z_flags + flag_bytes * r);
            h.report = r == 0;
            std::memcpy(karg.data(), &h, sizeof h);
            std::memcpy(karg.data() + sizeof h, slots.data() + (uint64_t)npad * r, 2 * (uint64_t)npad);
            if (rep) {
                // counter set 0 (in ws) zeroes set 1 after the last round, and
                // the other way round; rounds before the last zero nothing
                for (int set = 0; set < 2; set++) {
                    JitArgsHead hs = h;
                    uint8_t* zb = set ? rep->zb2 : ws;
                    hs.nulls = (unsigned long long*)(zb + z_nulls);
                    hs.lens = (unsigned long long*)(zb + z_lens);
                    hs.err = (unsigned long long*)(zb + z_err);
                    hs.flags = (unsigned long long*)(zb + z_flags + flag_bytes * r);
                    hs.abort_word = h.abort_word ? (unsigned int*)(zb + 8) : nullptr;
                    hs.zero_next = r + 1 == rounds ? (unsigned int*)(set ? ws : rep->zb2) : nullptr;
                    hs.zero_words = (uint32_t)(zbytes / 4);
                    // the last round's epilogue hands the counters to the host
                    hs.ticket = (unsigned int*)(zb + 12);
                    hs.rb_words = (uint32_t)(z_lb / 8);
                    hs.rb_host = r + 1 == rounds ? (unsigned long long*)rep->hrb_dev : nullptr;
                    std::vector<uint8_t> ka = karg;
                    std::memcpy(ka.data(), &hs, sizeof hs);
                    rep->kargs[set].push_back(ka);
                }
            } else {
                HIPC(jit_decode_launch(K, !local, karg.data(), karg.size(), (uint32_t)grid, lds, c->stream));
            }
        }
        if (!rep) c->last_kernel = "murr_jit_decode";
    }
    if (rep) return MURR_OK;
    c->stats.last_mode = cut ? 2u : local ? 1u : 3u;
    c->stats.last_grid = (uint32_t)grid;
    c->stats.last_shape_nw = K.nw;
    c->stats.last_shape_r = K.r;
    if (kernel_events(c)) HIPC(hipEventRecord(c->k1, c->stream));
    c->timed = kernel_events(c);
    c->lk0 = c->lk1 = nullptr;
    HIPC(read_back(c, rb, z_lb));
    c->retry_local = !local && emit && tiles;
    if (c->retry_local) {
        c->r_cols.assign(seg->cols, seg->cols + seg->ncols);
        c->r_seg = *seg;
        c->r_seg.cols = c->r_cols.data();
        c->r_proj.assign(proj, proj + nproj);
        c->r_blocks.assign(blocks, blocks + nblocks);
        c->r_est = est_row;
    }
    return pending_set(c, outs, blocks, nblocks, nproj, dp, rb);
}

}  // namespace


int murr_segment_prepare(murr_ctx_t* c, const murr_segment_t* seg) {
    murr_error_t* err = nullptr;
    if (!c || !valid_segment(seg)) return MURR_E_ARGUMENT;
    HIPC(hipSetDevice(c->device));
    std::string why;
    if (seg->ncols && !jit_layout(c->device, seg, &why)) {
        std::fprintf(stderr, "murr: JIT decode unavailable: %s\n", why.c_str());
        return MURR_E_INTERNAL;
    }
    std::vector<EncCol> ec(seg->ncols);
    for (uint32_t i = 0; i < seg->ncols; i++) {
        const murr_column_t& col = seg->cols[i];
        ec[i] = EncCol{nullptr, nullptr, nullptr, 0, col.dtype, col.index, col.offset, col.size};
    }
    if (seg->ncols &&
        !jit_encode_kernel(c->device, seg->bitset_size, seg->capacity, ec.data(), seg->ncols, 32768, 256,
                           jit_encode_sbw(0, 0, seg->bitset_size + seg->capacity, nutf8_of(seg)), &why)) {
        std::fprintf(stderr, "murr: JIT encode unavailable: %s\n", why.c_str());
        return MURR_E_INTERNAL;
    }
    return MURR_OK;
}

int murr_decode_enqueue(murr_ctx_t* c, const murr_segment_t* seg, const uint32_t* proj,
                        uint32_t nproj, const murr_block_t* blocks, uint32_t nblocks,
                        murr_array_t* outs) {
    return murr_decode_enqueue_ix(c, seg, proj, nproj, blocks, nblocks, nullptr, 0, outs);
}

namespace {
// Argument checks of a decode (the reference's errors first: zero columns is
// ArrowError, an unknown column SegmentError) and its per-projection
// descriptors and mean row size.
int decode_prep(murr_ctx* c, const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj,
                const murr_block_t* blocks, uint32_t nblocks, const uint64_t* const* uidx, uint32_t stride,
                const murr_array_t* outs, std::vector<DecProj>& dp, double& est_row) {
    murr_error_t* err = nullptr;
    if (!c || !valid_segment(seg) || (nblocks && (!blocks || !outs)) || (nproj && !proj) ||
        c->pending)
        return MURR_E_ARGUMENT;
    if (uidx && !stride_ok(stride)) return MURR_E_ARGUMENT;
    if (nproj == 0) return MURR_E_ARROW;  // RecordBatch::try_new, read.rs:106-108
    if (nproj > kMaxProj || nblocks > 0x3FFFF) return MURR_E_ARGUMENT;
    for (uint32_t p = 0; p < nproj; p++)
        if (proj[p] >= seg->ncols) return MURR_E_BAD_COLUMN;
    HIPC(hipSetDevice(c->device));

    dp.assign(nproj, DecProj{});
    uint32_t nutf8 = 0;
    for (uint32_t p = 0; p < nproj; p++) {
        const murr_column_t& col = seg->cols[proj[p]];
        dp[p] = DecProj{col.dtype, col.index, col.offset, col.size, col.dtype == MURR_UTF8, 0};
        if (col.dtype == MURR_UTF8) dp[p].uslot = nutf8++;
    }
    for (uint32_t b = 0; b < nblocks; b++) {
        const murr_block_t& bl = blocks[b];
        if (bl.n_rows && (!bl.data || (!bl.row_off && !bl.row_off32) || ((uintptr_t)bl.data & 15) ||
                          ((uintptr_t)bl.row_off32 & 3)))
            return MURR_E_ARGUMENT;
        for (uint32_t p = 0; p < nproj; p++) {
            const murr_array_t& o = outs[(uint64_t)b * nproj + p];
            if (bl.n_rows && (!o.validity || !o.values || (dp[p].is_utf8 && !o.offsets)))
                return MURR_E_ARGUMENT;
            if (dp[p].is_utf8 && !o.offsets) return MURR_E_ARGUMENT;
            if (((uintptr_t)o.validity & 7) || (dp[p].dtype == MURR_BOOL && ((uintptr_t)o.values & 7)) ||
                (!dp[p].is_utf8 && ((uintptr_t)o.values & (dp[p].width - 1))))
                return MURR_E_ARGUMENT;
        }
    }
    // Tile shape: NW waves x KC 64-row chunks per wave.  The largest tile whose
    // two LDS buffers (row-offset slice + blob stage, +25 % for row-size
    // variance) fit the per-workgroup budget, from the data_bytes hints (or a
    // schema estimate); a tile that still outgrows its stage is decoded from HBM.
    uint64_t hint_bytes = 0, hint_rows = 0;
    bool hinted = true;
    for (uint32_t b = 0; b < nblocks; b++) {
        if (blocks[b].n_rows && !blocks[b].data_bytes) hinted = false;
        hint_bytes += blocks[b].data_bytes;
        hint_rows += blocks[b].n_rows;
    }
    est_row = (double)seg->bitset_size + seg->capacity;
    for (uint32_t i = 0; i < seg->ncols; i++) est_row += seg->cols[i].dtype == MURR_UTF8 ? 20.0 : 0.0;
    if (hinted && hint_rows) est_row = (double)hint_bytes / (double)hint_rows;
    return MURR_OK;
}
}  // namespace

int murr_decode_enqueue_ix(murr_ctx_t* c, const murr_segment_t* seg, const uint32_t* proj,
                           uint32_t nproj, const murr_block_t* blocks, uint32_t nblocks,
                           const uint64_t* const* uidx, uint32_t stride, murr_array_t* outs) {
    murr_error_t* err = nullptr;
    std::vector<DecProj> dp;
    double est_row = 0;
    {
        const int pst = decode_prep(c, seg, proj, nproj, blocks, nblocks, uidx, stride, outs, dp, est_row);
        if (pst) return pst;
    }
    uint32_t nutf8 = 0;
    for (const DecProj& d : dp) nutf8 += d.is_utf8;
    // Per workgroup (NW waves: NW-1 consumers + 1 loader) a ring of S slots of
    // one fill each (F = 64 * KC * (NW-1) rows), P fills in flight:
    // (P-1) * E <= 63 (the loader's vmcnt field), S = P + 2, and the look-back
    // window (64 sub-tiles) must cover every sub-tile in flight:
    // (NW-1) * S < 64.  Take the first shape whose ring fits the LDS budget
    // with P >= 3 (else >= 2).
    double budget = 81920.0;  // bytes of LDS per workgroup (2 workgroups per CU)
    static const uint32_t shapes[][2] = {{8, 1}, {4, 2}, {8, 2}, {4, 4}, {4, 1}};
    uint32_t nw = 4, kc = 1, stage = 4096, depth = 2, slots = 4;
    auto plan = [&](uint32_t w, uint32_t k, uint32_t want_p, uint32_t* p_out, uint32_t* s_out, uint32_t* st_out) {
        const double f = 64.0 * k * (w - 1);
        uint32_t st = (uint32_t)round_up((uint64_t)(f * est_row * 1.25) + 64, 1024);
        st = std::min<uint32_t>(std::max<uint32_t>(st, 1024), 61440);
        const uint32_t ro = (uint32_t)round_up(8 * (uint64_t)(f + 1) + 16, 16);
        const uint32_t E = 1 + (ro + 1023) / 1024 + st / 1024;
        if (E > 63) return false;
        uint32_t p = std::min<uint32_t>(want_p, 1 + 63 / E);
        const uint32_t slot = 64 + ro + st + 32;
        for (; p >= 2; p--) {
            const uint32_t s = p + 2;
            if ((w - 1) * s >= 64) continue;
            const double lds = (double)s * slot + 2048.0 + 2048.0 * nutf8 + 16.0 * s * nutf8 + 4.0 * w * nproj;
            if (lds <= budget) { *p_out = p; *s_out = s; *st_out = st; return true; }
        }
        return false;
    };
    const uint32_t want_p = 8;
    bool found = false;
    for (uint32_t minp : {3u, 2u}) {
        for (const auto& sh : shapes) {
            uint32_t p, s, st;
            if (plan(sh[0], sh[1], want_p, &p, &s, &st) && p >= minp) {
                nw = sh[0]; kc = sh[1]; depth = p; slots = s; stage = st; found = true;
                break;
            }
        }
        if (found) break;
    }
    if (!found) {  // very wide rows: the smallest ring; fills past the stage go to HBM
        nw = 4; kc = 1; depth = 2; slots = 4; stage = 16384;
    }
    // Layout-specialised kernel (murr_jit.cpp), the default.  opts.kernel 2
    // selects the generic kernel; 1 makes a JIT failure an error; otherwise a
    // layout hiprtc cannot compile falls back to the generic kernel with one
    // message per process.
    c->stats.decodes++;
    {
        const int jmode = c->opts.kernel == 2 ? 0 : c->opts.kernel == 1 ? 1 : -1;
        uint64_t max_rows = 0;
        for (uint32_t b = 0; b < nblocks; b++) max_rows = std::max<uint64_t>(max_rows, blocks[b].n_rows);
        if (jmode != 0 && max_rows < 0x7FFFFFFFull) {
            std::string why;
            const JitLayout* jl = jit_layout(c->device, seg, &why, true);
            if (jl) {
                const int st = decode_enqueue_jit(c, seg, jl, proj, nproj, blocks, nblocks, outs, dp, est_row, false,
                                                  uidx, stride);
                jit_layout_unpin(jl);
                return st;
            }
            if (jmode == 1) {
                std::fprintf(stderr, "murr: JIT decode unavailable: %s\n", why.c_str());
                return MURR_E_INTERNAL;
            }
            static bool said = false;
            if (!said) {
                said = true;
                std::fprintf(stderr, "murr: JIT decode unavailable, using the generic kernel: %s\n", why.c_str());
            }
        }
    }
    const uint32_t rows = 64 * kc * (nw - 1);
    const uint64_t R = rows;
    std::vector<DecBlock> db(nblocks);
    uint64_t tiles = 0;
    uint32_t nonempty = 0;
    for (uint32_t b = 0; b < nblocks; b++) {
        db[b] = dec_block(blocks[b], tiles, nullptr);
        tiles += (blocks[b].n_rows + R - 1) / R;
        nonempty += blocks[b].n_rows != 0;
    }
    const bool verbose = c->opts.verbose != 0;
    std::vector<DecOut> dout((uint64_t)nblocks * nproj);
    for (uint64_t i = 0; i < dout.size(); i++)
        dout[i] = DecOut{(uint8_t*)outs[i].values, outs[i].validity, outs[i].offsets, outs[i].values_cap};

    const uint64_t nbp = (uint64_t)nblocks * nproj;
    const uint64_t z_err = 0, z_nulls = kErrBytes, z_lens = z_nulls + 8 * nbp, z_lb = z_lens + 8 * nbp;
    const uint64_t zbytes = round_up(z_lb + 8 * (uint64_t)nutf8 * tiles, 16);
    const uint64_t d_blocks = zbytes, d_proj = round_up(d_blocks + sizeof(DecBlock) * nblocks, 16);
    const uint64_t d_outs = round_up(d_proj + sizeof(DecProj) * nproj, 16);
    DecodeArgs a{};
    a.nproj = nproj;
    a.nutf8 = nutf8;
    a.stage = stage;
    decode_lds_plan(a, nw, kc, slots, depth);
    const uint32_t lds = a.lds_total;
    // Persistent grid: the occupancy answer (LDS-limited here), capped at 6 per CU.
    int bpc = std::max(1, std::min(decode_blocks_per_cu(nw, kc, lds), 6));
    uint64_t grid = std::min<uint64_t>(std::max<uint64_t>(tiles, 1), (uint64_t)c->cus * bpc);
    // Block-local mode when every workgroup gets whole blocks: no cross-tile
    // prefix protocol at all.  Otherwise tiles round-robin + window prefix.
    const bool local = nonempty >= grid;
    if (local) grid = std::max<uint64_t>(1, std::min<uint64_t>(grid, nonempty));
    const uint64_t d_end_desc = round_up(d_outs + sizeof(DecOut) * dout.size(), 16);
    const uint64_t dend = d_end_desc;
    int st = ensure_ws(c, dend, err);
    if (st) return st;
    // host scratch: [descriptors (dend - zbytes)] [readback z_lb bytes]
    // A small zeroed region travels with the descriptors in one H2D (one
    // stream op fewer per launch: it matters for small reads); a large one
    // (generic kernel, many tiles) is a device memset.
    const uint64_t hz = zbytes <= 65536 ? zbytes : 0;
    const uint64_t hdesc = d_end_desc - zbytes, rb = round_up(hz + dend - zbytes, 64);
    st = ensure_hs(c, rb + z_lb, err);
    if (st) return st;
    uint8_t* hd = c->hs + hz;
    if (hz) std::memset(c->hs, 0, hz);
    std::memcpy(hd + (d_blocks - zbytes), db.data(), sizeof(DecBlock) * nblocks);
    std::memcpy(hd + (d_proj - zbytes), dp.data(), sizeof(DecProj) * nproj);
    std::memcpy(hd + (d_outs - zbytes), dout.data(), sizeof(DecOut) * dout.size());

    if (!hz) HIPC(hipMemsetAsync(c->ws, 0, zbytes, c->stream));
    HIPC(upload_desc(c, c->ws + zbytes - hz, hz + hdesc));
    // Empty blocks: utf8 offsets = [0] (StringBuilder starts with offset 0).
    for (uint32_t b = 0; b < nblocks; b++)
        if (blocks[b].n_rows == 0)
            for (uint32_t p = 0; p < nproj; p++)
                if (dp[p].is_utf8 && outs[(uint64_t)b * nproj + p].offsets)
                    HIPC(hipMemsetAsync(outs[(uint64_t)b * nproj + p].offsets, 0, 4, c->stream));

    a.blocks = (const DecBlock*)(c->ws + d_blocks);
    a.proj = (const DecProj*)(c->ws + d_proj);
    a.outs = (const DecOut*)(c->ws + d_outs);
    a.lookback = (uint64_t*)(c->ws + z_lb);
    a.nulls = (unsigned long long*)(c->ws + z_nulls);
    a.lens = (unsigned long long*)(c->ws + z_lens);
    a.err = (unsigned long long*)(c->ws + z_err);
    a.total_tiles = tiles;
    a.nblocks = nblocks;
    a.bs = seg->bitset_size;
    a.local = local ? 1 : 0;
    for (uint32_t p = 0, u = 0; p < nproj; p++)
        if (dp[p].is_utf8 && u < 2) a.ufix[u++] = p;
    if (verbose)
        std::fprintf(stderr, "decode launch: grid %llu (%d/CU) tiles %llu shape %ux%u rows/tile %u stage %u slots %u depth %u lds %u local %d\n",
                     (unsigned long long)grid, bpc, (unsigned long long)tiles, nw, kc, rows, a.stage, slots, depth, lds, (int)local);
    if (kernel_events(c)) HIPC(hipEventRecord(c->k0, c->stream));
    if (tiles) {
        HIPC(launch_decode(a, nw, kc, (uint32_t)grid, c->stream));
        c->last_kernel = "decode_kernel";
    }
    c->stats.last_mode = 0;
    c->stats.last_grid = (uint32_t)grid;
    c->stats.last_shape_nw = nw;
    c->stats.last_shape_r = kc;
    if (kernel_events(c)) HIPC(hipEventRecord(c->k1, c->stream));
    c->timed = kernel_events(c);
    c->lk0 = c->lk1 = nullptr;
    HIPC(read_back(c, rb, z_lb));

    return pending_set(c, outs, blocks, nblocks, nproj, dp, rb);
}

uint64_t murr_utf8_index_len(const murr_segment_t* seg, uint64_t n_rows, uint32_t stride) {
    if (!valid_segment(seg) || !stride_ok(stride)) return 0;
    uint64_t nu = 0;
    for (uint32_t i = 0; i < seg->ncols; i++) nu += seg->cols[i].dtype == MURR_UTF8;
    return nu ? ((n_rows + stride - 1) / stride + 1) * nu : 0;
}

int murr_utf8_index(murr_ctx_t* c, const murr_segment_t* seg, const murr_block_t* block, uint32_t stride,
                    uint64_t* out) {
    return murr_utf8_index_update(c, seg, block, 0, stride, out);
}

int murr_utf8_index_update(murr_ctx_t* c, const murr_segment_t* seg, const murr_block_t* block, uint64_t from,
                           uint32_t stride, uint64_t* out) {
    murr_error_t* err = nullptr;
    if (!c || !valid_segment(seg) || !block || !stride_ok(stride) || c->pending || from > block->n_rows)
        return MURR_E_ARGUMENT;
    Utf8IndexArgs a{};
    for (uint32_t i = 0; i < seg->ncols; i++) {
        if (seg->cols[i].dtype != MURR_UTF8) continue;
        if (a.nu == kMaxUidxCols) return MURR_E_ARGUMENT;
        a.col[a.nu] = seg->cols[i].index;
        a.fo[a.nu] = seg->bitset_size + seg->cols[i].offset;
        a.nu++;
    }
    if (!a.nu) return MURR_OK;  // no utf8 column: nothing to index
    if (!out || (block->n_rows && (!block->data || (!block->row_off && !block->row_off32)))) return MURR_E_ARGUMENT;
    HIPC(hipSetDevice(c->device));
    const uint64_t nwin = utf8_index_windows(from, block->n_rows, stride);
    const int st = ensure_ws(c, 8 * std::max<uint64_t>(nwin, 1) * a.nu, err);
    if (st) return st;
    a.data = block->data;
    a.row_off = block->row_off;
    a.row_off32 = block->row_off32;
    a.out = out;
    a.part = (uint64_t*)c->ws;
    a.from = from;
    a.n = block->n_rows;
    a.stride = stride;
    a.bs = seg->bitset_size;
    HIPC(launch_utf8_index(a, c->stream));
    return MURR_OK;
}

int murr_utf8_row_lengths(murr_ctx_t* c, const murr_segment_t* seg, const murr_block_t* block, uint64_t from,
                          uint32_t* out) {
    murr_error_t* err = nullptr;
    if (!c || !valid_segment(seg) || !block || c->pending || from > block->n_rows) return MURR_E_ARGUMENT;
    Utf8IndexArgs a{};
    for (uint32_t i = 0; i < seg->ncols; i++) {
        if (seg->cols[i].dtype != MURR_UTF8) continue;
        if (a.nu == kMaxUidxCols) return MURR_E_ARGUMENT;
        a.col[a.nu] = seg->cols[i].index;
        a.fo[a.nu] = seg->bitset_size + seg->cols[i].offset;
        a.nu++;
    }
    if (!a.nu || from == block->n_rows) return MURR_OK;
    if (!out || !block->data || (!block->row_off && !block->row_off32)) return MURR_E_ARGUMENT;
    HIPC(hipSetDevice(c->device));
    a.data = block->data;
    a.row_off = block->row_off;
    a.row_off32 = block->row_off32;
    a.from = from;
    a.n = block->n_rows;
    a.bs = seg->bitset_size;
    HIPC(launch_utf8_row_lengths(a, out, c->stream));
    return MURR_OK;
}

}  // extern "C"
namespace {
int finish_counts(murr_ctx* c, const uint8_t* rb, murr_array_t* outs, uint32_t nblocks, uint32_t nproj,
                  const uint64_t* n_rows, const uint32_t* dtypes, murr_error_t* err);
int decode_collect(murr_ctx* c, murr_error_t* err);
}  // namespace
extern "C" {

int murr_decode_wait(murr_ctx_t* c, murr_error_t* err) {
    if (!c || !c->pending) return set_err(err, MURR_E_ARGUMENT);
    HIPC(hipStreamSynchronize(c->stream));
    return decode_collect(c, err);
}

namespace {
// A pending decode whose stream work (kernel and read-back) has finished:
// its counts and first error (murr_decode_wait after its synchronisation; the
// streaming host decode after the batch's event).
int decode_collect(murr_ctx* c, murr_error_t* err) {
    c->pending = false;
#ifdef MURR_TUNING
    if (c->opts.verbose && c->tl_off) print_timeline(c);
#endif
    const uint8_t* rb = c->hs + c->rb_off;
    unsigned long long word;
    std::memcpy(&word, rb, 8);
    uint32_t aborted = 0;
    std::memcpy(&aborted, rb + 8, 4);
    if (c->retry_local && aborted) {
        // a stream-mode wait timed out (the grid was not co-resident, e.g. a
        // shared GPU): the same decode in local mode, which never waits
        c->retry_local = false;
        c->stats.split_retries++;
        static bool said = false;
        if (!said) {
            said = true;
            std::fprintf(stderr, "murr: stream-mode decode timed out; re-running in local mode\n");
        }
        std::string why;
        const JitLayout* jl = jit_layout(c->device, &c->r_seg, &why, true);
        std::vector<DecProj> dp(c->r_proj.size());
        for (size_t p = 0; p < dp.size(); p++) {
            const murr_column_t& col = c->r_seg.cols[c->r_proj[p]];
            dp[p] = DecProj{col.dtype, col.index, col.offset, col.size, col.dtype == MURR_UTF8, 0};
        }
        const std::vector<uint32_t> proj = c->r_proj;
        const std::vector<murr_block_t> blocks = c->r_blocks;
        const int st = jl ? decode_enqueue_jit(c, &c->r_seg, jl, proj.data(), (uint32_t)proj.size(), blocks.data(),
                                               (uint32_t)blocks.size(), c->outs, dp, c->r_est, true)
                          : MURR_E_INTERNAL;
        jit_layout_unpin(jl);
        if (st) return set_err(err, st);
        return murr_decode_wait(c, err);
    }
    c->retry_local = false;
    return finish_counts(c, rb, c->outs, c->nblocks, c->nproj, c->n_rows.data(), c->dtypes.data(), err);
}
}  // namespace

namespace {
// The read-back counters of a finished decode -> the arrays' null counts and
// data lengths, and the first error.
int finish_counts(murr_ctx* c, const uint8_t* rb, murr_array_t* outs, uint32_t nblocks, uint32_t nproj,
                  const uint64_t* n_rows, const uint32_t* dtypes, murr_error_t* err) {
    unsigned long long word;
    std::memcpy(&word, rb, 8);
    const uint64_t nbp = (uint64_t)nblocks * nproj;
    const unsigned long long* nulls = (const unsigned long long*)(rb + kErrBytes);
    if (c->opts.verbose) {  // phase stamps of a stamped (MJ_STAMPS) tuning build
        const unsigned long long* stp = (const unsigned long long*)(rb + 16);
        if (stp[0] | stp[4]) {
            std::fprintf(stderr, "stamps (Gcycles, sum over waves; murr_jit_kernel.hip / murr_decode.hip Stamps):");
            for (uint32_t i = 0; i < kStampSlots; i++) std::fprintf(stderr, "%s %.3f", i == 4 ? " |" : "", stp[i] * 1e-9);
            std::fprintf(stderr, "\n");
        }
    }
    const unsigned long long* lens = nulls + nbp;
    for (uint32_t b = 0; b < nblocks; b++) {
        for (uint32_t p = 0; p < nproj; p++) {
            murr_array_t& o = outs[(uint64_t)b * nproj + p];
            const uint64_t n = n_rows[b];
            const uint32_t d = dtypes[p];
            o.null_count = nulls[(uint64_t)b * nproj + p];
            o.data_len = d == MURR_UTF8 ? lens[(uint64_t)b * nproj + p]
                         : d == MURR_BOOL ? (n + 7) / 8 : n * (uint64_t)dtype_size(d);
        }
    }
    if (err) std::memset(err, 0, sizeof *err);
    int st = unpack_err(word, err);
    if (st == MURR_E_CAPACITY && err) err->required = outs[(uint64_t)err->block * nproj + err->column].data_len;
    return st;
}
}  // namespace

// ---- prepared decode (murr_decode_plan) -----------------------------------------

struct murr_plan {
    murr_ctx* c = nullptr;
    std::vector<murr_column_t> cols;
    murr_segment_t seg{};
    std::vector<uint32_t> proj;
    std::vector<murr_block_t> blocks;
    std::vector<const uint64_t*> uidx;
    uint32_t stride = 0;
    murr_array_t* outs = nullptr;
    std::vector<DecProj> dp;
    std::vector<uint64_t> n_rows;
    std::vector<uint32_t> dtypes;
    double est_row = 0;
    const JitLayout* jl = nullptr;  // pinned while the plan lives
    uint32_t every = kTimeEvery;    // one run in `every` bracketed by timing events (0: none)
    bool replay = false;
    JitReplay r;
    bool sync_pending = false;  // (no replay) murr_decode_run_async ran the decode; wait returns its status
    int sync_status = 0;
    murr_error_t sync_err{};
};

extern "C" {

int murr_decode_plan(murr_ctx_t* c, const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj,
                     const murr_block_t* blocks, uint32_t nblocks, const uint64_t* const* uidx, uint32_t stride,
                     murr_array_t* outs, murr_plan_t** out) {
    if (!out) return MURR_E_ARGUMENT;
    *out = nullptr;
    std::vector<DecProj> dp;
    double est_row = 0;
    const int pst = decode_prep(c, seg, proj, nproj, blocks, nblocks, uidx, stride, outs, dp, est_row);
    if (pst) return pst;
    std::unique_ptr<murr_plan> P(new (std::nothrow) murr_plan());
    if (!P) return MURR_E_INTERNAL;
    P->c = c;
    P->cols.assign(seg->cols, seg->cols + seg->ncols);
    P->seg = *seg;
    P->seg.cols = P->cols.data();
    P->proj.assign(proj, proj + nproj);
    P->blocks.assign(blocks, blocks + nblocks);
    if (uidx) P->uidx.assign(uidx, uidx + nblocks);
    P->stride = stride;
    P->outs = outs;
    P->dp = dp;
    P->est_row = est_row;
    for (uint32_t b = 0; b < nblocks; b++) P->n_rows.push_back(blocks[b].n_rows);
    for (const DecProj& d : dp) P->dtypes.push_back(d.dtype);
    uint64_t max_rows = 0;
    for (uint32_t b = 0; b < nblocks; b++) max_rows = std::max<uint64_t>(max_rows, blocks[b].n_rows);
    if (c->opts.kernel != 2 && max_rows < 0x7FFFFFFFull && seg->ncols) {
        std::string why;
        P->jl = jit_layout(c->device, &P->seg, &why, true);
        if (P->jl) {
            const int st = decode_enqueue_jit(c, &P->seg, P->jl, P->proj.data(), nproj, P->blocks.data(), nblocks,
                                              outs, P->dp, est_row, false, uidx ? P->uidx.data() : nullptr, stride,
                                              &P->r);
            if (st) {
                P->r.release();
                jit_layout_unpin(P->jl);
                return st;
            }
            P->replay = true;
            if (hipEventCreate(&P->r.e0) != hipSuccess || hipEventCreate(&P->r.t1) != hipSuccess ||
                hipEventCreateWithFlags(&P->r.e1, hipEventDisableTiming) != hipSuccess) {
                P->r.release();
                jit_layout_unpin(P->jl);
                return MURR_E_HIP;
            }
        } else if (c->opts.kernel == 1) {
            return MURR_E_INTERNAL;
        }
    }
    *out = P.release();
    return MURR_OK;
}

int murr_decode_run_async(murr_plan_t* P) {
    if (!P) return MURR_E_ARGUMENT;
    murr_ctx* c = P->c;
    if (c->pending || P->r.inflight || P->sync_pending) return MURR_E_ARGUMENT;
    const uint32_t nblocks = (uint32_t)P->blocks.size(), nproj = (uint32_t)P->proj.size();
    if (!P->replay) {  // (generic kernel) the ordinary decode, done now; wait reports it
        P->sync_err = murr_error_t{};
        P->sync_status = murr_decode_blocks_ix(c, &P->seg, P->proj.data(), nproj, P->blocks.data(), nblocks,
                                               P->uidx.empty() ? nullptr : P->uidx.data(), P->stride, P->outs,
                                               &P->sync_err);
        P->sync_pending = true;
        return MURR_OK;
    }
    murr_error_t* err = nullptr;
    JitReplay& R = P->r;
    HIPC(hipSetDevice(c->device));
    c->stats.decodes++;
    // counter sets alternate: this run counts into `set`, which the previous
    // run zeroed (both were zeroed when the plan was made)
    const uint64_t run = R.runs++;
    const int set = (int)(run & 1);
    for (int32_t* o : R.empty_offsets) HIPC(hipMemsetAsync(o, 0, 4, c->stream));
    volatile uint64_t* done = (volatile uint64_t*)(R.hrb + R.z_lb);
    *done = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    uint64_t every = P->every;
#ifdef MURR_TUNING
    if (const char* e = std::getenv("MURR_TIME_EVERY")) every = std::max(1, std::atoi(e));  // A/B of the events' cost
#endif
    const bool timed = every && run % every == 0;
    if (timed) R.timed_runs++;
    if (timed) HIPC(hipEventRecord(R.e0, c->stream));
    for (const auto& ka : R.kargs[set])
        HIPC(jit_decode_launch(R.K, R.split, ka.data(), ka.size(), R.grid, R.lds, c->stream));
    R.end = timed ? R.t1 : R.e1;
    HIPC(hipEventRecord(R.end, c->stream));
    R.set = set;
    R.inflight = true;
    return MURR_OK;
}

}  // extern "C"

namespace {
int plan_wait(murr_plan_t* P, murr_error_t* err, bool end_sync);
}  // namespace

extern "C" {

int murr_decode_run_wait(murr_plan_t* P, murr_error_t* err) { return plan_wait(P, err, true); }

}  // extern "C"

namespace {
// end_sync: after the done flag, also wait for the kernel's end (its outputs
// visible beyond the context's stream); a prepared read whose outputs are
// consumed on that stream (its own D2H kernel, or the caller's work queued on
// it) skips it: 6 us of a 1000-key read (round 6)
int plan_wait(murr_plan_t* P, murr_error_t* err, bool end_sync) {
    if (!P) return set_err(err, MURR_E_ARGUMENT);
    murr_ctx* c = P->c;
    if (P->sync_pending) {
        P->sync_pending = false;
        if (err) *err = P->sync_err;
        return P->sync_status;
    }
    JitReplay& R = P->r;
    if (!R.inflight) return set_err(err, MURR_E_ARGUMENT);
    R.inflight = false;
    const int set = R.set;
    const uint32_t nblocks = (uint32_t)P->blocks.size(), nproj = (uint32_t)P->proj.size();
    HIPC(hipSetDevice(c->device));
    // The last workgroup's epilogue writes the counters here and sets `done`:
    // no read-back copy, no stream synchronisation.  Should the run end
    // without the flag (it cannot, short of a device fault), read the
    // counters back the ordinary way.
    volatile uint64_t* done = (volatile uint64_t*)(R.hrb + R.z_lb);
    bool flagged = false;
    if (!R.kargs[set].empty()) {
        for (uint64_t spin = 1;; spin++) {
            if (*done) { flagged = true; break; }
            if ((spin & 4095) == 0 && hipEventQuery(R.end) == hipSuccess) {
                flagged = *done != 0;
                break;
            }
            __builtin_ia32_pause();
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    // The flag says every workgroup has stored its outputs, but those stores
    // are ordered only within c->stream until the kernel ends (the epilogue's
    // atomics are relaxed): wait for the kernel's end, so the outputs are
    // visible to the host, other streams and peer GPUs when this returns.
    // The kernel is in its last workgroup's epilogue by now; a next run queued
    // behind it keeps the GPU busy meanwhile.
#ifdef MURR_TUNING
    static const bool nosync = std::getenv("MURR_PLAN_NOSYNC") != nullptr;  // A/B: the flag alone
    if (nosync) end_sync = false;
#endif
    if (flagged && end_sync) HIPC(hipEventSynchronize(R.end));
    if (!flagged) {
        if (!R.kargs[set].empty()) c->stats.readback_fallbacks++;
        HIPC(hipMemcpyAsync(R.hrb, set ? R.zb2 : R.dws, R.z_lb, hipMemcpyDeviceToHost, c->stream));
        HIPC(hipStreamSynchronize(c->stream));
    }
    if (R.timed_runs) {  // the plan's last timed run
        c->timed = true;
        c->lk0 = R.e0;
        c->lk1 = R.t1;
    }
    if (!R.kargs[0].empty()) c->last_kernel = "murr_jit_decode";
    c->stats.last_mode = R.mode;
    c->stats.last_grid = R.grid;
    c->stats.last_shape_nw = R.K.nw;
    c->stats.last_shape_r = R.K.r;
    uint32_t aborted = 0;
    std::memcpy(&aborted, R.hrb + 8, 4);
    if (R.split && R.emit && aborted) {
        // a split-mode look-back wait expired: the same decode in local mode
        c->stats.split_retries++;
        const int st = decode_enqueue_jit(c, &P->seg, P->jl, P->proj.data(), nproj, P->blocks.data(), nblocks,
                                          P->outs, P->dp, P->est_row, true);
        if (st) return set_err(err, st);
        return murr_decode_wait(c, err);
    }
    return finish_counts(c, R.hrb, P->outs, nblocks, nproj, P->n_rows.data(), P->dtypes.data(), err);
}
}  // namespace

extern "C" {

int murr_decode_run(murr_plan_t* P, murr_error_t* err) {
    const int st = murr_decode_run_async(P);
    if (st) return set_err(err, st);
    return murr_decode_run_wait(P, err);
}

int murr_plan_time_every(murr_plan_t* P, uint32_t every) {
    if (!P) return MURR_E_ARGUMENT;
    P->every = every;
    return MURR_OK;
}

void murr_plan_free(murr_plan_t* P) {
    if (!P) return;
    if (P->c) (void)hipSetDevice(P->c->device);
    if (P->r.dws) (void)hipStreamSynchronize(P->c->stream);
    if (P->c && P->r.e0 && P->c->lk0 == P->r.e0) {  // its events were the context's last timing
        P->c->lk0 = P->c->lk1 = nullptr;
        P->c->timed = false;
    }
    P->r.release();
    jit_layout_unpin(P->jl);
    delete P;
}

}  // extern "C"

int murr_decode_blocks(murr_ctx_t* c, const murr_segment_t* seg, const uint32_t* proj,
                       uint32_t nproj, const murr_block_t* blocks, uint32_t nblocks,
                       murr_array_t* outs, murr_error_t* err) {
    return murr_decode_blocks_ix(c, seg, proj, nproj, blocks, nblocks, nullptr, 0, outs, err);
}

int murr_decode_blocks_ix(murr_ctx_t* c, const murr_segment_t* seg, const uint32_t* proj,
                          uint32_t nproj, const murr_block_t* blocks, uint32_t nblocks,
                          const uint64_t* const* uidx, uint32_t stride, murr_array_t* outs, murr_error_t* err) {
    int st = murr_decode_enqueue_ix(c, seg, proj, nproj, blocks, nblocks, uidx, stride, outs);
    if (st) {
        if (err && st != MURR_E_HIP) set_err(err, st);
        else if (err && st == MURR_E_HIP) set_err(err, st, (int)hipGetLastError());
        return st;
    }
    return murr_decode_wait(c, err);
}

// ---- encode ------------------------------------------------------------------

uint64_t murr_encode_bound(const murr_segment_t* seg, uint64_t n, const uint64_t* utf8_bytes) {
    if (!seg) return 0;
    uint64_t b = n * ((uint64_t)seg->bitset_size + seg->capacity);
    for (uint32_t i = 0; i < seg->ncols; i++)
        if (seg->cols[i].dtype == MURR_UTF8) b += 4 * n + (utf8_bytes ? utf8_bytes[i] : 0);
    return b;
}

int murr_encode_batch(murr_ctx_t* c, const murr_segment_t* seg, const murr_col_in_t* cols,
                      uint64_t n, uint8_t* out_blob, uint64_t blob_cap, uint64_t* out_row_off,
                      uint64_t* blob_len, murr_error_t* err) {
    return murr_encode_batch_at(c, seg, cols, n, out_blob, blob_cap, out_row_off, 0, blob_len, err);
}

int murr_encode_batch_ix(murr_ctx_t* c, const murr_segment_t* seg, const murr_col_in_t* cols, uint64_t n,
                         uint8_t* out_blob, uint64_t blob_cap, uint64_t* out_row_off, uint32_t stride,
                         uint64_t* uidx, uint64_t* blob_len, murr_error_t* err) {
    if (!stride_ok(stride) || (murr_utf8_index_len(seg, n, stride) && !uidx)) return set_err(err, MURR_E_ARGUMENT);
    const int st = murr_encode_batch_at(c, seg, cols, n, out_blob, blob_cap, out_row_off, 0, blob_len, err);
    if (st) return st;
    const murr_block_t blk{out_blob, out_row_off, n, blob_len ? *blob_len : 0, nullptr};
    const int ist = murr_utf8_index_update(c, seg, &blk, 0, stride, uidx);
    if (ist) return set_err(err, ist);
    HIPC(hipStreamSynchronize(c->stream));
    return MURR_OK;
}

int murr_encode_batch_at(murr_ctx_t* c, const murr_segment_t* seg, const murr_col_in_t* cols,
                         uint64_t n, uint8_t* out_blob, uint64_t blob_cap, uint64_t* out_row_off,
                         uint64_t row_base, uint64_t* blob_len, murr_error_t* err) {
    if (!c || !valid_segment(seg) || (seg->ncols && !cols) || !out_row_off || c->pending)
        return set_err(err, MURR_E_ARGUMENT);
    if (n > 0xFFFFFFFFull * kTile) return set_err(err, MURR_E_ARGUMENT);
    HIPC(hipSetDevice(c->device));
    uint32_t nutf8 = 0;
    std::vector<EncCol> ec(seg->ncols);
    for (uint32_t i = 0; i < seg->ncols; i++) {
        const murr_column_t& col = seg->cols[i];
        if (n && (!cols[i].values || (col.dtype == MURR_UTF8 && !cols[i].offsets)))
            return set_err(err, MURR_E_ARGUMENT);
        ec[i] = EncCol{(const uint8_t*)cols[i].values, cols[i].validity, cols[i].offsets,
                       cols[i].offset, col.dtype, col.index, col.offset, col.size};
        nutf8 += col.dtype == MURR_UTF8;
    }
    const uint64_t fixed = (uint64_t)seg->bitset_size + seg->capacity;
    if (nutf8 == 0 && n * fixed > blob_cap) {
        set_err(err, MURR_E_CAPACITY);
        if (err) err->required = n * fixed;
        return MURR_E_CAPACITY;
    }
    if (n && !out_blob) return set_err(err, MURR_E_ARGUMENT);
    // Run-time specialised encode kernel unless the context asks for the
    // generic one (or it cannot be compiled: then the generic encode_kernel).
    const JitEncKernel* ek = nullptr;
    {
        const uint32_t ek_mode = c->opts.encode_kernel;
        if (ek_mode != 2 && seg->ncols) {
            std::string why;
            const uint32_t tile = jit_encode_tile(n, blob_cap);
            ek = jit_encode_kernel(c->device, seg->bitset_size, seg->capacity, ec.data(), seg->ncols,
                                   jit_encode_stage(n, blob_cap, tile), tile,
                                   jit_encode_sbw(n, blob_cap, seg->bitset_size + seg->capacity, nutf8_of(seg)), &why);
            if (!ek && (c->opts.verbose || ek_mode == 1))
                std::fprintf(stderr, "murr: JIT encode unavailable: %s\n", why.c_str());
            if (!ek && ek_mode == 1) return set_err(err, MURR_E_INTERNAL);
        }
    }
    const uint32_t tile = ek ? ek->tile : kTile;
    const uint64_t tiles = (n + tile - 1) / tile;
    // utf8 layouts: tile totals / starts, then the group sums (JIT scan)
    const uint64_t z_lb = 16,
                   zbytes = round_up(z_lb + 8 * (nutf8 ? tiles + 1 + (tiles + kEncScanPer - 1) / kEncScanPer : 0), 16);
    const uint64_t d_cols = zbytes, dend = round_up(d_cols + sizeof(EncCol) * ec.size(), 16);
    int st = ensure_ws(c, dend, err);
    if (st) return st;
    st = ensure_hs(c, round_up(dend - zbytes, 64) + 64, err);
    if (st) return st;
    std::memcpy(c->hs, ec.data(), sizeof(EncCol) * ec.size());
    const uint64_t rb = round_up(dend - zbytes, 64);
    HIPC(hipMemsetAsync(c->ws, 0, zbytes, c->stream));
    if (!ec.empty()) HIPC(hipMemcpyAsync(c->ws + d_cols, c->hs, sizeof(EncCol) * ec.size(),
                                         hipMemcpyHostToDevice, c->stream));
    if (n == 0) HIPC(hipMemcpyAsync(out_row_off, &row_base, 8, hipMemcpyHostToDevice, c->stream));
    EncodeArgs a{};
    a.row_base = row_base;
    a.cols = (const EncCol*)(c->ws + d_cols);
    a.out = out_blob;
    a.row_off = out_row_off;
    a.lookback = (uint64_t*)(c->ws + z_lb);
    a.err = (unsigned long long*)c->ws;
    a.n_rows = n;
    a.out_cap = blob_cap;
    a.total_tiles = tiles;
    a.ncols = seg->ncols;
    a.nutf8 = nutf8;
    a.bs = seg->bitset_size;
    a.cap = seg->capacity;
    // utf8 tile totals (murr_internal.h kEncSizes*): a utf8 column with a
    // validity buffer has them estimated first (exact when its null strings
    // are empty) and recounted by the sizes pass when the kernel finds one off
    bool inl = true;
    for (const EncCol& e : ec) inl = inl && (e.dtype != MURR_UTF8 || e.validity == nullptr);
    uint32_t sizes = inl ? kEncSizesInline : kEncSizesEstimate;
#ifdef MURR_TUNING
    if (std::getenv("MURR_ENC_EXACT")) sizes = inl ? kEncSizesInline : kEncSizesPass;  // A/B of the estimate
#endif
    HIPC(hipEventRecord(c->k0, c->stream));
    unsigned long long word = 0;
    uint64_t total = 0;
    for (;;) {
        if (tiles) {
            // persistent grid, co-resident (the utf8 window prefix waits on tiles t-G+1 .. t-1)
            const int per_cu = ek ? std::max(1, ek->bpc - 1) : c->enc_grid_per_cu;
            uint64_t grid = std::min<uint64_t>(tiles, (uint64_t)c->cus * per_cu);
            if (ek) {
                HIPC(jit_encode_launch(ek, a, (uint32_t)grid, c->stream, sizes));
                c->last_kernel = "murr_jit_encode";
            } else {
                HIPC(launch_encode(a, (uint32_t)grid, c->stream));
                c->last_kernel = "encode_kernel";
            }
        }
        HIPC(hipEventRecord(c->k1, c->stream));  // (after a recount: both runs)
        HIPC(hipMemcpyAsync(c->hs + rb, c->ws, 8, hipMemcpyDeviceToHost, c->stream));
        HIPC(hipMemcpyAsync(c->hs + rb + 8, out_row_off + n, 8, hipMemcpyDeviceToHost, c->stream));
        HIPC(hipStreamSynchronize(c->stream));
        std::memcpy(&word, c->hs + rb, 8);
        std::memcpy(&total, c->hs + rb + 8, 8);
        // an estimate off (or any error under estimates, which may be the
        // estimate's doing): recount exactly and encode again
        if (!(ek && nutf8 && sizes == kEncSizesEstimate && word)) break;
        c->stats.encode_recounts++;
        sizes = kEncSizesPass;
        HIPC(hipMemsetAsync(c->ws, 0, zbytes, c->stream));
    }
    c->timed = true;
    c->lk0 = c->lk1 = nullptr;
    total -= row_base;
    if (blob_len) *blob_len = total;
    if (err) std::memset(err, 0, sizeof *err);
    st = unpack_err(word, err);
    if (st == kEncStRecount) {  // an exact recount off: a bug, not the input's
        st = MURR_E_INTERNAL;
        if (err) err->status = st;
    }
    if (err) err->block = 0;
    if (st == MURR_E_CAPACITY && err) err->required = total;
    return st;
}

}  // extern "C"

// ---- host-memory path --------------------------------------------------------

// Decoded outputs of one block on their way to the host: one device region and
// one pinned region with the same layout (per column values, validity, utf8
// offsets; 64-B aligned parts), grown on demand and reused.
struct HostOut {
    uint8_t* dout = nullptr;
    uint64_t dout_cap = 0;
    uint8_t* hout = nullptr;
    uint64_t hout_cap = 0;
    std::vector<murr_array_t> arr;
    std::vector<uint64_t> off;  // per column: values, validity, offsets
};

struct murr_builder {
    murr_ctx* ctx = nullptr;
    std::vector<murr_column_t> cols;
    murr_segment_t seg{};
    std::vector<uint32_t> proj;
    // pinned staging of the blobs + row offsets (add_row appends here)
    uint8_t* hdata = nullptr;
    uint64_t hdata_len = 0, hdata_cap = 0;
    uint64_t* hoff = nullptr;
    uint64_t n = 0, hoff_cap = 0;
    uint64_t present = 0;
    // device buffers (grow-only)
    uint8_t* ddata = nullptr;
    uint64_t ddata_cap = 0;
    HostOut out;  // decoded outputs (device + pinned host)
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr, e3 = nullptr;
    double total_ms = 0;
    float h2d_ms = 0, k_ms = 0, d2h_ms = 0;
};

namespace {

// Context buffer pool: the smallest pooled buffer of the kind that holds
// `need` bytes, else a new allocation of at least `want`.
constexpr size_t kPoolMax = 32;
bool pool_take(murr_ctx* c, bool pinned, uint64_t need, uint64_t want, uint8_t** p, uint64_t* cap) {
    size_t best = c->pool.size();
    for (size_t i = 0; i < c->pool.size(); i++)
        if (c->pool[i].pinned == pinned && c->pool[i].cap >= need &&
            (best == c->pool.size() || c->pool[i].cap < c->pool[best].cap))
            best = i;
    if (best < c->pool.size()) {
        *p = c->pool[best].p;
        *cap = c->pool[best].cap;
        c->pool.erase(c->pool.begin() + best);
        return true;
    }
    *p = nullptr;
    if ((pinned ? hipHostMalloc(p, want, hipHostMallocDefault) : hipMalloc(p, want)) != hipSuccess) return false;
    *cap = want;
    return true;
}
void pool_give(murr_ctx* c, bool pinned, uint8_t* p, uint64_t cap) {
    if (!p) return;
    if (c && c->pool.size() < kPoolMax) {
        c->pool.push_back(murr_ctx::Buf{p, cap, pinned});
        return;
    }
    (void)(pinned ? hipHostFree(p) : hipFree(p));
}

bool grow_pinned(murr_ctx* c, uint8_t** p, uint64_t* cap, uint64_t need, uint64_t keep) {
    if (need <= *cap) return true;
    const uint64_t nc = std::max<uint64_t>(need, std::max<uint64_t>(*cap * 2, 1 << 16));
    uint8_t* q = nullptr;
    uint64_t qc = 0;
    if (!pool_take(c, true, need, nc, &q, &qc)) return false;
    if (*p) {
        if (keep) std::memcpy(q, *p, keep);
        pool_give(c, true, *p, *cap);
    }
    *p = q;
    *cap = qc;
    return true;
}

bool grow_dev(murr_ctx* c, uint8_t** p, uint64_t* cap, uint64_t need) {
    if (need <= *cap) return true;
    pool_give(c, false, *p, *cap);
    *p = nullptr;
    const uint64_t nc = round_up(std::max<uint64_t>(need, 1 << 16), 1 << 16);
    if (!pool_take(c, false, need, nc, p, cap)) { *cap = 0; return false; }
    return true;
}

// Decode one device block (enqueued behind whatever is on the stream) into
// o.dout and bring the projected arrays to o.hout; outs[p] point into o.hout.
// A small batch (the point-lookup case) copies its whole output region back
// in one D2H right behind the decode, with no round trip to learn the sizes;
// a large one waits for the sizes and copies exactly the bytes.  utf8_cap
// bounds the string bytes of any one utf8 column.  e2/e3 (optional) bracket
// the D2H.
int decode_to_host(murr_ctx* c, const murr_segment_t* seg, const uint32_t* proj, uint32_t np,
                   murr_block_t blk, uint64_t utf8_cap, HostOut& o, hipEvent_t e2, hipEvent_t e3,
                   murr_host_array_t* outs, murr_error_t* err) {
    const uint64_t n = blk.n_rows;
    const uint64_t bm = murr_bitmap_bytes(n);
    o.off.assign((size_t)np * 3, 0);
    uint64_t off = 0;
    for (uint32_t p = 0; p < np; p++) {
        const murr_column_t& col = seg->cols[proj[p]];
        uint64_t vb = col.dtype == MURR_UTF8 ? utf8_cap : col.dtype == MURR_BOOL ? bm : n * col.size;
        o.off[3 * p] = off;
        off = round_up(off + std::max<uint64_t>(vb, 8), 64);
        o.off[3 * p + 1] = off;
        off = round_up(off + std::max<uint64_t>(bm, 8), 64);
        o.off[3 * p + 2] = off;
        if (col.dtype == MURR_UTF8) off = round_up(off + (n + 1) * 4, 64);
    }
    const uint64_t total_out = std::max<uint64_t>(off, 64);
    if (!grow_dev(c, &o.dout, &o.dout_cap, total_out) || !grow_pinned(c, &o.hout, &o.hout_cap, total_out, 0))
        return set_err(err, MURR_E_HIP);
    o.arr.assign(np, murr_array_t{});
    for (uint32_t p = 0; p < np; p++) {
        murr_array_t& a = o.arr[p];
        a.values = o.dout + o.off[3 * p];
        a.validity = o.dout + o.off[3 * p + 1];
        a.offsets = seg->cols[proj[p]].dtype == MURR_UTF8 ? (int32_t*)(o.dout + o.off[3 * p + 2]) : nullptr;
        a.values_cap = utf8_cap;
    }
    constexpr uint64_t kOneCopy = 1 << 20;
    int st = murr_decode_enqueue(c, seg, proj, np, &blk, 1, o.arr.data());
    if (st) {
        if (err && st != MURR_E_HIP) set_err(err, st);
        else if (err) set_err(err, st, (int)hipGetLastError());
        return st;
    }
    if (total_out <= kOneCopy) {
        if (e2) HIPC(hipEventRecord(e2, c->stream));
        HIPC(hipMemcpyAsync(o.hout, o.dout, total_out, hipMemcpyDeviceToHost, c->stream));
        if (e3) HIPC(hipEventRecord(e3, c->stream));
        st = murr_decode_wait(c, err);
        if (st) return st;
    } else {
        st = murr_decode_wait(c, err);
        if (st) return st;
        if (e2) HIPC(hipEventRecord(e2, c->stream));
        for (uint32_t p = 0; p < np; p++) {
            const murr_array_t& a = o.arr[p];
            if (a.data_len)
                HIPC(hipMemcpyAsync(o.hout + o.off[3 * p], a.values, a.data_len, hipMemcpyDeviceToHost, c->stream));
            if (a.null_count)
                HIPC(hipMemcpyAsync(o.hout + o.off[3 * p + 1], a.validity, bm, hipMemcpyDeviceToHost, c->stream));
            if (a.offsets)
                HIPC(hipMemcpyAsync(o.hout + o.off[3 * p + 2], a.offsets, (n + 1) * 4, hipMemcpyDeviceToHost,
                                    c->stream));
        }
        if (e3) HIPC(hipEventRecord(e3, c->stream));
        HIPC(hipStreamSynchronize(c->stream));
    }
    for (uint32_t p = 0; p < np; p++) {
        const murr_array_t& a = o.arr[p];
        murr_host_array_t& h = outs[p];
        h.values = o.hout + o.off[3 * p];
        h.validity = a.null_count ? o.hout + o.off[3 * p + 1] : nullptr;
        h.offsets = a.offsets ? (const int32_t*)(o.hout + o.off[3 * p + 2]) : nullptr;
        h.length = n;
        h.null_count = a.null_count;
        h.values_len = a.data_len;
        h.dtype = seg->cols[proj[p]].dtype;
        h._pad = 0;
    }
    return MURR_OK;
}

bool push_off(murr_builder* b) {
    if (b->n + 2 > b->hoff_cap) {
        uint8_t* p = (uint8_t*)b->hoff;
        uint64_t capb = b->hoff_cap * 8;
        if (!grow_pinned(b->ctx, &p, &capb, (b->n + 2) * 8, (b->n + 1) * 8)) return false;
        b->hoff = (uint64_t*)p;
        b->hoff_cap = capb / 8;
    }
    b->hoff[++b->n] = b->hdata_len;
    return true;
}

}  // namespace

extern "C" {

int murr_builder_new(murr_ctx_t* c, const murr_segment_t* seg, const uint32_t* proj,
                     uint32_t nproj, uint64_t capacity, murr_builder_t** out) {
    if (!c || !out || !valid_segment(seg) || (nproj && !proj)) return MURR_E_ARGUMENT;
    for (uint32_t p = 0; p < nproj; p++)
        if (proj[p] >= seg->ncols) return MURR_E_BAD_COLUMN;
    murr_builder* b = new (std::nothrow) murr_builder();
    if (!b) return MURR_E_INTERNAL;
    b->ctx = c;
    b->cols.assign(seg->cols, seg->cols + seg->ncols);
    b->seg = *seg;
    b->seg.cols = b->cols.data();
    b->proj.assign(proj, proj + nproj);
    (void)hipSetDevice(c->device);
    uint64_t cap = std::max<uint64_t>(capacity, 16);
    uint64_t capb = 0;
    uint8_t* p = nullptr;
    if (!grow_pinned(c, &p, &capb, (cap + 2) * 8, 0)) { delete b; return MURR_E_HIP; }
    b->hoff = (uint64_t*)p;
    b->hoff_cap = capb / 8;
    b->hoff[0] = 0;
    if (!grow_pinned(c, &b->hdata, &b->hdata_cap, cap * ((uint64_t)seg->bitset_size + seg->capacity + 16), 0)) {
        murr_builder_free(b);
        return MURR_E_HIP;
    }
    for (hipEvent_t* e : {&b->e0, &b->e1, &b->e2, &b->e3}) {
        if (!c->event_pool.empty()) {
            *e = c->event_pool.back();
            c->event_pool.pop_back();
        } else {
            (void)hipEventCreate(e);
        }
    }
    *out = b;
    return MURR_OK;
}

// ReadBatchBuilder::add_row (read.rs:85-91): the row bytes are copied into the
// pinned staging block; decoding happens once per batch in build().
int murr_builder_add_row(murr_builder_t* b, const uint8_t* bytes, uint64_t len) {
    if (!b || (len && !bytes)) return MURR_E_ARGUMENT;
    if (len == 0) return MURR_E_MALFORMED_ROW;  // a present row is never empty (write.rs:21)
    if (!grow_pinned(b->ctx, &b->hdata, &b->hdata_cap, b->hdata_len + len, b->hdata_len)) return MURR_E_HIP;
    std::memcpy(b->hdata + b->hdata_len, bytes, len);
    b->hdata_len += len;
    b->present++;
    return push_off(b) ? MURR_OK : MURR_E_HIP;
}

// ReadBatchBuilder::add_empty (read.rs:93-98): a zero-length row.
int murr_builder_add_empty(murr_builder_t* b) {
    if (!b) return MURR_E_ARGUMENT;
    return push_off(b) ? MURR_OK : MURR_E_HIP;
}

int murr_builder_add_rows(murr_builder_t* b, const uint8_t* const* ptrs, const uint64_t* lens,
                          uint64_t n) {
    if (!b || (n && (!ptrs || !lens))) return MURR_E_ARGUMENT;
    for (uint64_t i = 0; i < n; i++) {
        int st = ptrs[i] ? murr_builder_add_row(b, ptrs[i], lens[i]) : murr_builder_add_empty(b);
        if (st) return st;
    }
    return MURR_OK;
}

// ReadBatchBuilder::build (read.rs:100-109): H2D, one decode launch, D2H.
int murr_builder_build(murr_builder_t* b, murr_host_array_t* outs, murr_error_t* err) {
    if (!b || (!b->proj.empty() && !outs)) return set_err(err, MURR_E_ARGUMENT);
    if (b->proj.empty()) return set_err(err, MURR_E_ARROW);
    auto t0 = std::chrono::steady_clock::now();
    murr_ctx* c = b->ctx;
    HIPC(hipSetDevice(c->device));
    const uint64_t n = b->n, np = b->proj.size();
    const uint64_t dbytes = round_up(b->hdata_len, 16) + 16;
    const uint64_t obytes = (n + 1) * 8;
    const uint64_t fixed = (uint64_t)b->seg.bitset_size + b->seg.capacity;
    const uint64_t utf8_cap = b->hdata_len > b->present * fixed ? b->hdata_len - b->present * fixed : 0;
    if (!grow_dev(c, &b->ddata, &b->ddata_cap, dbytes + obytes + 64)) return set_err(err, MURR_E_HIP);
    uint8_t* ddata = b->ddata;
    uint64_t* doff = (uint64_t*)(b->ddata + round_up(dbytes, 64));
    HIPC(hipEventRecord(b->e0, c->stream));
    if (b->hdata_len) HIPC(hipMemcpyAsync(ddata, b->hdata, b->hdata_len, hipMemcpyHostToDevice, c->stream));
    HIPC(hipMemcpyAsync(doff, b->hoff, obytes, hipMemcpyHostToDevice, c->stream));
    HIPC(hipEventRecord(b->e1, c->stream));
    murr_block_t blk{ddata, doff, n, b->hdata_len, nullptr};
    int st = decode_to_host(c, &b->seg, b->proj.data(), (uint32_t)np, blk, utf8_cap, b->out, b->e2, b->e3, outs, err);
    if (st) return st;
    (void)hipEventElapsedTime(&b->h2d_ms, b->e0, b->e1);
    murr_ctx_last_kernel_ms(c, &b->k_ms);
    (void)hipEventElapsedTime(&b->d2h_ms, b->e2, b->e3);
    b->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MURR_OK;
}

int murr_builder_last_timing(murr_builder_t* b, double* total_ms, float* h2d_ms, float* kernel_ms,
                             float* d2h_ms) {
    if (!b) return MURR_E_ARGUMENT;
    if (total_ms) *total_ms = b->total_ms;
    if (h2d_ms) *h2d_ms = b->h2d_ms;
    if (kernel_ms) *kernel_ms = b->k_ms;
    if (d2h_ms) *d2h_ms = b->d2h_ms;
    return MURR_OK;
}

void murr_builder_free(murr_builder_t* b) {
    if (!b) return;
    murr_ctx* c = b->ctx;
    if (c) (void)hipSetDevice(c->device);
    // buffers and events go back to the context's pool for the next builder
    pool_give(c, true, b->hdata, b->hdata_cap);
    pool_give(c, true, (uint8_t*)b->hoff, b->hoff_cap * 8);
    pool_give(c, true, b->out.hout, b->out.hout_cap);
    pool_give(c, false, b->ddata, b->ddata_cap);
    pool_give(c, false, b->out.dout, b->out.dout_cap);
    for (hipEvent_t e : {b->e0, b->e1, b->e2, b->e3}) {
        if (!e) continue;
        if (c) c->event_pool.push_back(e);
        else (void)hipEventDestroy(e);
    }
    delete b;
}

}  // extern "C"

// ---- streaming host decode (murr_hstream_*) ----------------------------------
// Batch reads back to back, host in, host out, `depth` batches in flight, each
// on its own slot: a context (stream, workspace), device input and output
// buffers, pinned output, all reused.  Batch i runs entirely on its slot's
// stream: the H2D of its blob and row offsets (copy engine from 1 MiB up,
// below that a copy kernel with the decode's descriptors), the decode, then
// one segment-copy kernel (murr_kernels.hip copy_segs_kernel) that writes its
// fixed-size arrays, exactly the decoded utf8 bytes (each column's length read
// from its final offset on the device) and the decode's counters into pinned
// host memory -- no host round trip between the decode and its D2H, and no
// cross-stream event.  next() waits on the batch's one event.  Measured
// against the alternatives on one box: copy engines both
// ways on two shared streams 10.4 GiB/s, kernel copies both ways 11.3, this
// split 12.4-12.9 (config B, pinned sources).  Tuning builds keep the others:
// MURR_HSTREAM_DMA=1, MURR_HSTREAM_H2D=kernel.

// Host copies of pageable batches into pinned staging, split over a few
// worker threads and the caller (one core copies ~2.6 MB -- a config B batch --
// in ~130 us, longer than the device needs for the batch).  Workers sleep
// between batches; a copy is cut into 256 KiB pieces taken off an atomic
// counter.
struct CopyPool {
    struct Piece {
        uint8_t* dst;
        const uint8_t* src;
        uint64_t n;
    };
    // One copy() call's pieces and counters.  Each call makes a new one and a
    // worker takes it under the lock, so a worker that wakes late for an
    // earlier call works on (and counts into) that call's job only, never on
    // a job the caller is building.
    struct Job {
        std::vector<Piece> pieces;
        std::atomic<size_t> next{0}, done{0};
    };
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv;
    std::shared_ptr<Job> cur;
    uint64_t gen = 0;
    bool stop = false;

    explicit CopyPool(unsigned n) {
        try {
            for (unsigned i = 0; i < n; i++) th.emplace_back([this] { work(); });
        } catch (...) {
            halt();  // (the threads already started end before the exception leaves)
            throw;
        }
    }
    ~CopyPool() { halt(); }
    void halt() {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th)
            if (t.joinable()) t.join();
    }
    static void drain(Job& j) {
        for (size_t i; (i = j.next.fetch_add(1)) < j.pieces.size(); j.done.fetch_add(1))
            std::memcpy(j.pieces[i].dst, j.pieces[i].src, j.pieces[i].n);
    }
    void work() {
        uint64_t seen = 0;
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> g(m);
                cv.wait(g, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
                j = cur;
            }
            if (j) drain(*j);
        }
    }
    // copy every (dst, src, n) of `parts`; returns when all bytes are copied
    void copy(const std::vector<Piece>& parts) {
        constexpr uint64_t kPiece = 256 << 10;
        auto j = std::make_shared<Job>();
        for (const Piece& p : parts)
            for (uint64_t o = 0; o < p.n; o += kPiece) j->pieces.push_back(Piece{p.dst + o, p.src + o, std::min(kPiece, p.n - o)});
        {
            std::lock_guard<std::mutex> g(m);
            cur = j;
            gen++;
        }
        cv.notify_all();
        drain(*j);
        while (j->done.load() < j->pieces.size()) std::this_thread::yield();
    }
};

struct HSlot {
    murr_ctx* c = nullptr;
    uint8_t* hin = nullptr;  // pinned staging: blobs | row offsets (unpinned sources)
    uint64_t hin_cap = 0;
    uint8_t* din = nullptr;  // device input: blobs | row offsets
    uint64_t din_cap = 0;
    HostOut out;
    uint64_t n = 0, h2d_bytes = 0, d2h_bytes = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;  // H2D start / end (H2D stream)
    hipEvent_t ed = nullptr;                // decode done (slot stream)
    hipEvent_t e2 = nullptr, e3 = nullptr;  // fixed-size D2H start / end (D2H stream)
    hipEvent_t e4 = nullptr, e5 = nullptr;  // utf8 bytes D2H start / end (D2H stream)
    int submit_status = MURR_OK;  // an enqueue that failed: next() reports it
    murr_error_t submit_err{};
    bool timed = false;           // this batch's copies are bracketed by timing events
    bool drained = false;         // decode waited for, counters read, D2H queued (or its error kept)
    uint64_t ub = 0;              // utf8 bytes of its D2H
};

struct murr_hstream {
    murr_ctx* owner = nullptr;
    std::vector<murr_column_t> cols;
    murr_segment_t seg{};
    std::vector<uint32_t> proj;
    std::vector<HSlot> slots;
    hipStream_t s_h2d = nullptr, s_d2h = nullptr;
    bool fused = true;            // D2H (and H2D unless `h2d_engine`) by segment-copy kernels on the slot streams
    bool h2d_engine = true;       // (fused) H2D of batches >= kEngineMinBytes by copy-engine copies on the slot stream
    std::unique_ptr<CopyPool> pool;  // pageable batches' staging copies (created on the first large one)
    bool pool_failed = false;        // (no threads: single-threaded copies)
    uint64_t head = 0, tail = 0;  // batches submitted / returned
    murr_hstream_stats_t stats{};
#ifdef MURR_TUNING
    // submit phases (MURR_HSTREAM_PHASES=1, printed at free), ms summed over
    // batches: 0 progress, 1 source / staging, 2 H2D enqueue, 3 output layout,
    // 4 decode enqueue (descriptors, launch, copy kernels), 5 event record
    double ph[6] = {0, 0, 0, 0, 0, 0};
#endif
};

namespace {
#ifdef MURR_TUNING
struct PhaseClock {  // (batches past the first 16 only: first-use allocations and the compile excluded)
    double* ph;
    bool on;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(int k) {
        const auto now = std::chrono::steady_clock::now();
        if (on) ph[k] += std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
    }
};
#define HS_LAP(k) pc.lap(k)
#else
#define HS_LAP(k) ((void)0)
#endif
}  // namespace

namespace {

constexpr uint64_t kEngineMinBytes = 1ull << 20;
constexpr uint64_t kPoolMinBytes = 1ull << 20;  // pageable batches from here are staged by the copy pool
constexpr unsigned kPoolThreads = 3;             // workers (the caller copies too)

// The device address of pinned host bytes (hipHostMalloc / hipHostRegister),
// or null when `p` is not pinned memory the device can read.
const uint8_t* pinned_dev_view(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return a.type == hipMemoryTypeHost && a.devicePointer ? (const uint8_t*)a.devicePointer : nullptr;
}

// Enqueue batch `s` (everything after the staging copy is asynchronous).  The
// output region is laid out as decode_to_host's, its utf8 parts bounded by the
// blob bytes.
int hstream_enqueue(murr_hstream* h, HSlot& s, const uint8_t* data, const void* row_off, uint32_t w, uint64_t n,
                    bool pinned, murr_error_t* err) {
    murr_ctx* c = s.c;
    // The context's fused-transfer state is set for one decode enqueue only:
    // clear it on every way out, so a failed batch leaves nothing behind for
    // the next one on this slot (a stale `xin` would copy old sources).
    struct XferReset {
        murr_ctx* c;
        ~XferReset() {
            c->xfer = false;
            c->xin.clear();
            c->xout.clear();
        }
    } xreset{c};
#ifdef MURR_TUNING
    PhaseClock pc{h->ph, h->head >= 16};
#endif
    HIPC(hipSetDevice(c->device));
    // row offsets: u64, or u32 (murr_hstream_submit32: half the index bytes over PCIe)
    auto off_at = [&](uint64_t i) -> uint64_t {
        return w == 4 ? ((const uint32_t*)row_off)[i] : ((const uint64_t*)row_off)[i];
    };
    const uint64_t b0 = n ? off_at(0) : 0, b1 = n ? off_at(n) : 0;
    if (b1 < b0) return set_err(err, MURR_E_ARGUMENT);
    const uint64_t bytes = b1 - b0, head = b0 & 15;
    const uint64_t dbytes = round_up(head + bytes + 16, 64), obytes = (n + 1) * w;
    if (!grow_dev(c, &s.din, &s.din_cap, dbytes + obytes)) return set_err(err, MURR_E_HIP);
    const uint8_t* src_data = data + (b0 - head);
    const uint8_t* src_off = (const uint8_t*)row_off;
    // H2D: the copy engine for large batches; below ~1 MiB its fixed cost per
    // copy (~10 us, two copies) dominates, and the copy kernel takes the bytes
    // (config C's 1000-key reads: 2.8 -> 3.6 GiB/s)
    const bool engine = h->fused && h->h2d_engine && head + bytes + obytes >= kEngineMinBytes;
    if (pinned && h->fused && !engine) {
        // the copy kernel reads the caller's pinned bytes at their device addresses
        const uint8_t* dd = pinned_dev_view(src_data);
        const uint8_t* doo = pinned_dev_view(row_off);
        if (dd && doo) {
            src_data = dd;
            src_off = doo;
        } else {
            pinned = false;  // (not pinned after all: staged like pageable bytes)
        }
    }
    if (!pinned) {
        // one host copy into the slot's pinned staging (the caller may reuse
        // its buffers as soon as submit returns)
        if (!grow_pinned(c, &s.hin, &s.hin_cap, dbytes + obytes, 0)) return set_err(err, MURR_E_HIP);
        if (head + bytes + obytes >= kPoolMinBytes && !h->pool && !h->pool_failed) {
            try {
                h->pool.reset(new CopyPool(kPoolThreads));
            } catch (...) {
                h->pool_failed = true;
            }
        }
        if (h->pool && head + bytes + obytes >= kPoolMinBytes) {
            h->pool->copy({CopyPool::Piece{s.hin, src_data, head + bytes},
                           CopyPool::Piece{s.hin + dbytes, (const uint8_t*)row_off, obytes}});
        } else {
            if (head + bytes) std::memcpy(s.hin, src_data, head + bytes);
            std::memcpy(s.hin + dbytes, row_off, obytes);
        }
        src_data = s.hin;
        src_off = s.hin + dbytes;
    }
    uint8_t* doff = s.din + dbytes;
    HS_LAP(1);
    s.timed = (h->head & 7) == 0;  // every eighth batch carries timing events
    if (engine) {
        // input copies by the copy engine, on the slot stream ahead of the decode
        if (s.timed) HIPC(hipEventRecord(s.e0, c->stream));
        if (head + bytes) HIPC(hipMemcpyAsync(s.din, src_data, head + bytes, hipMemcpyHostToDevice, c->stream));
        HIPC(hipMemcpyAsync(doff, src_off, obytes, hipMemcpyHostToDevice, c->stream));
        if (s.timed) HIPC(hipEventRecord(s.e1, c->stream));
    } else if (h->fused) {
        // input copies: with the decode's descriptors, in one kernel (murr_decode_enqueue)
        c->xin.assign({CopySeg{src_data, s.din, head + bytes, nullptr}, CopySeg{src_off, doff, obytes, nullptr}});
    } else {
        if (s.timed) HIPC(hipEventRecord(s.e0, h->s_h2d));
        if (head + bytes) HIPC(hipMemcpyAsync(s.din, src_data, head + bytes, hipMemcpyHostToDevice, h->s_h2d));
        HIPC(hipMemcpyAsync(doff, src_off, obytes, hipMemcpyHostToDevice, h->s_h2d));
        HIPC(hipEventRecord(s.e1, h->s_h2d));
        HIPC(hipStreamWaitEvent(c->stream, s.e1, 0));
    }
    s.h2d_bytes = head + bytes + obytes;
    HS_LAP(2);
    // row i of the block is data[row_off[i]..]: the block's data pointer sits
    // row_off[0] & ~15 bytes before the staged bytes (16-B aligned)
    murr_block_t blk{s.din - (b0 - head), w == 8 ? (const uint64_t*)doff : nullptr, n, b1,
                     w == 4 ? (const uint32_t*)doff : nullptr};
    const uint64_t utf8_cap = std::max<uint64_t>(bytes, 8);  // any one utf8 column's string bytes
    const uint32_t np = (uint32_t)h->proj.size();
    const uint64_t bm = murr_bitmap_bytes(n);
    HostOut& o = s.out;
    // layout: every fixed-size part first (one D2H right behind the decode),
    // then the utf8 values (exact bytes, copied in next())
    o.off.assign((size_t)np * 3, 0);
    uint64_t off = 0;
    for (uint32_t p = 0; p < np; p++) {
        const murr_column_t& col = h->seg.cols[h->proj[p]];
        if (col.dtype != MURR_UTF8) {
            o.off[3 * p] = off;
            off = round_up(off + std::max<uint64_t>(col.dtype == MURR_BOOL ? bm : n * col.size, 8), 64);
        }
        o.off[3 * p + 1] = off;
        off = round_up(off + std::max<uint64_t>(bm, 8), 64);
        if (col.dtype == MURR_UTF8) {
            o.off[3 * p + 2] = off;
            off = round_up(off + (n + 1) * 4, 64);
        }
    }
    const uint64_t fixed_out = std::max<uint64_t>(off, 64);
    for (uint32_t p = 0; p < np; p++)
        if (h->seg.cols[h->proj[p]].dtype == MURR_UTF8) {
            o.off[3 * p] = off;
            off = round_up(off + utf8_cap, 64);
        }
    const uint64_t total_out = std::max<uint64_t>(off, 64);
    if (!grow_dev(c, &o.dout, &o.dout_cap, total_out) || !grow_pinned(c, &o.hout, &o.hout_cap, total_out, 0))
        return set_err(err, MURR_E_HIP);
    o.arr.assign(np, murr_array_t{});
    for (uint32_t p = 0; p < np; p++) {
        murr_array_t& a = o.arr[p];
        a.values = o.dout + o.off[3 * p];
        a.validity = o.dout + o.off[3 * p + 1];
        a.offsets = h->seg.cols[h->proj[p]].dtype == MURR_UTF8 ? (int32_t*)(o.dout + o.off[3 * p + 2]) : nullptr;
        a.values_cap = utf8_cap;
    }
    if (h->fused) {
        // output copies: the fixed-size parts, then each utf8 column's bytes
        // up to its final offset (exactly the decoded bytes), with the
        // decode's counters, in one kernel behind the decode
        c->xout.assign({CopySeg{o.dout, o.hout, fixed_out, nullptr}});
        for (uint32_t p = 0; p < np; p++)
            if (o.arr[p].offsets)
                c->xout.push_back(CopySeg{o.dout + o.off[3 * p], o.hout + o.off[3 * p], utf8_cap, o.arr[p].offsets + n});
        c->xfer = true;
        c->xtimed = s.timed;
        c->xe[0] = engine ? s.e4 : s.e0;  // (engine H2D: e0/e1 bracket the copies above)
        c->xe[1] = engine ? s.e5 : s.e1;
        c->xe[2] = s.e2;
        c->xe[3] = s.e3;
    }
    HS_LAP(3);
    const int st = murr_decode_enqueue(c, &h->seg, h->proj.data(), np, &blk, 1, o.arr.data());
    if (st) return set_err(err, st, st == MURR_E_HIP ? (int)hipGetLastError() : 0);
    HS_LAP(4);
    HIPC(hipEventRecord(s.ed, c->stream));  // the decode and its counters' read-back are done
    HS_LAP(5);
    s.d2h_bytes = fixed_out;  // (the fixed-size part, queued with the utf8 bytes once the counters are in)
    s.n = n;
    s.drained = false;
    return MURR_OK;
}

// Batch s's decode is done: read its counters (null counts, utf8 bytes,
// errors) and queue its D2H on the D2H stream -- the fixed-size arrays in one
// copy, then exactly the decoded utf8 bytes -- closed by event e3.  An error
// is kept for next() (the slot then has nothing to copy).
void hstream_drain(murr_hstream* h, HSlot& s) {
    if (s.drained) return;
    s.drained = true;
    if (s.submit_status) return;
    murr_error_t e{};
    const uint64_t retries = s.c->stats.split_retries;
    const int st = decode_collect(s.c, &e);  // (its event `ed` has completed)
    if (st) {
        s.submit_status = st;
        s.submit_err = e;
        return;
    }
    const HostOut& o = s.out;
    bool ok = true;
    if (h->fused) {
        // its copies ran behind the decode; a decode re-run (split mode timed
        // out, murr_decode_wait) came after them: copy again
        s.ub = 0;
        for (uint32_t p = 0; p < h->proj.size(); p++)
            if (o.arr[p].offsets) s.ub += o.arr[p].data_len;
        if (s.c->stats.split_retries != retries) {
            ok = hipMemcpy(o.hout, o.dout, s.d2h_bytes, hipMemcpyDeviceToHost) == hipSuccess;
            for (uint32_t p = 0; ok && p < h->proj.size(); p++)
                if (o.arr[p].offsets && o.arr[p].data_len)
                    ok = hipMemcpy(o.hout + o.off[3 * p], o.arr[p].values, o.arr[p].data_len, hipMemcpyDeviceToHost) == hipSuccess;
        }
        if (!ok) {
            s.submit_status = MURR_E_HIP;
            s.submit_err = murr_error_t{};
            s.submit_err.status = MURR_E_HIP;
            s.submit_err.hip_error = (int)hipGetLastError();
        }
        return;
    }
    if (s.timed) ok = ok && hipEventRecord(s.e2, h->s_d2h) == hipSuccess;
    ok = ok && hipMemcpyAsync(o.hout, o.dout, s.d2h_bytes, hipMemcpyDeviceToHost, h->s_d2h) == hipSuccess;
    s.ub = 0;
    for (uint32_t p = 0; ok && p < h->proj.size(); p++) {
        const murr_array_t& a = o.arr[p];
        if (a.offsets && a.data_len) {
            ok = hipMemcpyAsync(o.hout + o.off[3 * p], a.values, a.data_len, hipMemcpyDeviceToHost, h->s_d2h) == hipSuccess;
            s.ub += a.data_len;
        }
    }
    ok = ok && hipEventRecord(s.e3, h->s_d2h) == hipSuccess;
    if (!ok) {
        s.submit_status = MURR_E_HIP;
        s.submit_err = murr_error_t{};
        s.submit_err.status = MURR_E_HIP;
        s.submit_err.hip_error = (int)hipGetLastError();
    }
}

// Queue the D2H of every batch, oldest first, whose decode has finished (no
// wait): next() then finds its copy under way or done.
void hstream_progress(murr_hstream* h) {
    if (h->fused) return;  // (nothing to queue: the copies follow the decode on its stream)
    for (uint64_t j = h->tail; j < h->head; j++) {
        HSlot& s = h->slots[j % h->slots.size()];
        if (s.drained) continue;
        if (!s.submit_status) {
            (void)hipSetDevice(s.c->device);
            if (hipEventQuery(s.ed) != hipSuccess) break;  // (in order: a later batch waits for this one)
        }
        hstream_drain(h, s);
    }
}

}  // namespace

extern "C" {

int murr_hstream_new(murr_ctx_t* c, const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj,
                     uint32_t depth, murr_hstream_t** out) {
    if (!c || !out || !valid_segment(seg) || (nproj && !proj) || depth < 2 || depth > 8) return MURR_E_ARGUMENT;
    *out = nullptr;
    if (nproj == 0) return MURR_E_ARROW;  // RecordBatch::try_new, read.rs:106-108
    if (nproj > kMaxProj) return MURR_E_ARGUMENT;
    for (uint32_t p = 0; p < nproj; p++)
        if (proj[p] >= seg->ncols) return MURR_E_BAD_COLUMN;
    murr_hstream* h = new (std::nothrow) murr_hstream();
    if (!h) return MURR_E_INTERNAL;
    h->owner = c;
    h->cols.assign(seg->cols, seg->cols + seg->ncols);
    h->seg = *seg;
    h->seg.cols = h->cols.data();
    h->proj.assign(proj, proj + nproj);
    h->slots.resize(depth);
#ifdef MURR_TUNING
    if (std::getenv("MURR_HSTREAM_DMA")) h->fused = false;  // A/B: DMA-engine copies
    if (const char* e = std::getenv("MURR_HSTREAM_H2D")) h->h2d_engine = std::string(e) != "kernel";
#endif
    int st = hipSetDevice(c->device) == hipSuccess ? MURR_OK : MURR_E_HIP;
    if (!st && (hipStreamCreateWithFlags(&h->s_h2d, hipStreamNonBlocking) != hipSuccess ||
                hipStreamCreateWithFlags(&h->s_d2h, hipStreamNonBlocking) != hipSuccess))
        st = MURR_E_HIP;
    for (HSlot& s : h->slots) {
        if (!st) st = murr_ctx_create(c->device, &s.c);
        if (!st) st = murr_ctx_set_opts(s.c, &c->opts);
        for (hipEvent_t* e : {&s.e0, &s.e1, &s.e2, &s.e3, &s.e4, &s.e5})
            if (!st && hipEventCreate(e) != hipSuccess) st = MURR_E_HIP;
        if (!st && hipEventCreateWithFlags(&s.ed, hipEventDisableTiming) != hipSuccess) st = MURR_E_HIP;
    }
    if (st) {
        murr_hstream_free(h);
        return st;
    }
    *out = h;
    return MURR_OK;
}

namespace {
int hstream_submit(murr_hstream_t* h, const uint8_t* data, const void* row_off, uint32_t w, uint64_t n_rows,
                   uint32_t flags, murr_error_t* err) {
    if (!h || !row_off || (n_rows && !data) || h->head - h->tail >= h->slots.size())
        return set_err(err, MURR_E_ARGUMENT);
    const auto t0 = std::chrono::steady_clock::now();
    struct Clock {  // host time of this call, however it returns
        murr_hstream* h;
        std::chrono::steady_clock::time_point t0;
        ~Clock() { h->stats.host_submit_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
    } clock{h, t0};
#ifdef MURR_TUNING
    PhaseClock pc{h->ph, h->head >= 16};
#endif
    hstream_progress(h);  // D2H of the batches whose decode finished, queued early
    HS_LAP(0);
    HSlot& s = h->slots[h->head % h->slots.size()];
    s.submit_err = murr_error_t{};
    s.submit_status = hstream_enqueue(h, s, data, row_off, w, n_rows, (flags & MURR_HSTREAM_PINNED) != 0, &s.submit_err);
    if (s.submit_status && s.c->pending) {  // (an enqueue failure after the launch: drain it)
        murr_error_t e2{};
        (void)murr_decode_wait(s.c, &e2);
    }
    h->head++;
    return MURR_OK;
}
}  // namespace

int murr_hstream_submit(murr_hstream_t* h, const uint8_t* data, const uint64_t* row_off, uint64_t n_rows,
                        uint32_t flags, murr_error_t* err) {
    return hstream_submit(h, data, row_off, 8, n_rows, flags, err);
}

int murr_hstream_submit32(murr_hstream_t* h, const uint8_t* data, const uint32_t* row_off, uint64_t n_rows,
                          uint32_t flags, murr_error_t* err) {
    return hstream_submit(h, data, row_off, 4, n_rows, flags, err);
}

int murr_hstream_next(murr_hstream_t* h, murr_host_array_t* outs, murr_error_t* err) {
    if (!h || !outs || h->tail == h->head) return set_err(err, MURR_E_ARGUMENT);
    struct Clock {
        murr_hstream* h;
        std::chrono::steady_clock::time_point t0;
        ~Clock() { h->stats.host_next_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
    } clock{h, std::chrono::steady_clock::now()};
    HSlot& s = h->slots[h->tail % h->slots.size()];
    if (!s.drained && !s.submit_status) {  // its decode (fused: and its copies) still running: wait
        HIPC(hipSetDevice(s.c->device));
        const auto w0 = std::chrono::steady_clock::now();
        const hipError_t we = hipEventSynchronize(s.ed);
        h->stats.host_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        HIPC(we);
    }
    hstream_drain(h, s);
    h->tail++;
    hstream_progress(h);  // and the next ones' D2H behind it, if their decodes are done
    if (s.submit_status) {
        if (err) *err = s.submit_err;
        return s.submit_status;
    }
    murr_ctx* c = s.c;
    HIPC(hipSetDevice(c->device));
    if (!h->fused) {  // its D2H landed (fused: with the decode's event)
        const auto w0 = std::chrono::steady_clock::now();
        const hipError_t we = hipEventSynchronize(s.e3);
        h->stats.host_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        HIPC(we);
    }
    const HostOut& o = s.out;
    const uint64_t ub = s.ub;
    if (s.timed) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, s.e0, s.e1) == hipSuccess) h->stats.h2d_ms += ms;
        if (murr_ctx_last_kernel_ms(c, &ms) == MURR_OK) h->stats.kernel_ms += ms;
        if (hipEventElapsedTime(&ms, s.e2, s.e3) == hipSuccess) h->stats.d2h_ms += ms;
        h->stats.timed_batches++;
    }
    h->stats.h2d_bytes += s.h2d_bytes;
    h->stats.d2h_bytes += s.d2h_bytes + ub;
    h->stats.batches++;
    for (uint32_t p = 0; p < h->proj.size(); p++) {
        const murr_array_t& a = o.arr[p];
        murr_host_array_t& ha = outs[p];
        ha.values = o.hout + o.off[3 * p];
        ha.validity = a.null_count ? o.hout + o.off[3 * p + 1] : nullptr;
        ha.offsets = a.offsets ? (const int32_t*)(o.hout + o.off[3 * p + 2]) : nullptr;
        ha.length = s.n;
        ha.null_count = a.null_count;
        ha.values_len = a.data_len;
        ha.dtype = h->seg.cols[h->proj[p]].dtype;
        ha._pad = 0;
    }
    return MURR_OK;
}

int murr_hstream_stats(murr_hstream_t* h, murr_hstream_stats_t* out) {
    if (!h || !out) return MURR_E_ARGUMENT;
    *out = h->stats;
    return MURR_OK;
}

void murr_hstream_free(murr_hstream_t* h) {
    if (!h) return;
#ifdef MURR_TUNING
    if (std::getenv("MURR_HSTREAM_PHASES") && h->head > 16)
        std::fprintf(stderr,
                     "hstream submit phases (us per batch over %llu): progress %.2f  source %.2f  h2d %.2f  layout %.2f  "
                     "decode_enqueue %.2f  event %.2f\n",
                     (unsigned long long)h->head - 16, h->ph[0] * 1e3 / (h->head - 16), h->ph[1] * 1e3 / (h->head - 16),
                     h->ph[2] * 1e3 / (h->head - 16), h->ph[3] * 1e3 / (h->head - 16), h->ph[4] * 1e3 / (h->head - 16),
                     h->ph[5] * 1e3 / (h->head - 16));
#endif
    if (h->owner) (void)hipSetDevice(h->owner->device);
    if (h->s_h2d) (void)hipStreamSynchronize(h->s_h2d);
    if (h->s_d2h) (void)hipStreamSynchronize(h->s_d2h);
    for (HSlot& s : h->slots) {
        if (!s.c) continue;
        (void)hipSetDevice(s.c->device);
        if (s.c->pending) {
            murr_error_t e{};
            (void)murr_decode_wait(s.c, &e);
        }
        (void)hipStreamSynchronize(s.c->stream);
        pool_give(s.c, true, s.hin, s.hin_cap);
        pool_give(s.c, false, s.din, s.din_cap);
        pool_give(s.c, true, s.out.hout, s.out.hout_cap);
        pool_give(s.c, false, s.out.dout, s.out.dout_cap);
        for (hipEvent_t e : {s.e0, s.e1, s.ed, s.e2, s.e3, s.e4, s.e5})
            if (e) (void)hipEventDestroy(e);
        murr_ctx_destroy(s.c);  // (frees the pooled buffers too)
    }
    if (h->s_d2h) (void)hipStreamSynchronize(h->s_d2h);
    if (h->s_h2d) (void)hipStreamDestroy(h->s_h2d);
    if (h->s_d2h) (void)hipStreamDestroy(h->s_d2h);
    delete h;
}

}  // extern "C"

// ---- resident read, host keys in, host arrays out ---------------------------

// Reads whose worst case (keys x longest row) passes this size the gather
// exactly (two phases); resident.py's TWO_PHASE_BYTES is the same bound.
constexpr uint64_t kTwoPhaseBytes = 64ull << 20;

struct murr_reader {
    murr_ctx* ctx = nullptr;
    std::vector<murr_column_t> cols;
    murr_segment_t seg{};
    uint8_t* hkeys = nullptr;   // pinned: rebased key offsets, then the key bytes
    uint64_t hkeys_cap = 0;
    uint8_t* dwork = nullptr;   // device: keys, gather offsets, rows, needed, gathered rows
    uint64_t dwork_cap = 0;
    HostOut out;
};

extern "C" {

int murr_reader_new(murr_ctx_t* c, const murr_segment_t* seg, murr_reader_t** out) {
    if (!c || !out || !valid_segment(seg)) return MURR_E_ARGUMENT;
    murr_reader* r = new (std::nothrow) murr_reader();
    if (!r) return MURR_E_INTERNAL;
    r->ctx = c;
    r->cols.assign(seg->cols, seg->cols + seg->ncols);
    r->seg = *seg;
    r->seg.cols = r->cols.data();
    *out = r;
    return MURR_OK;
}

// Table::read (src/io/table/mod.rs:114-129) over a device-resident table in
// one call: the keys go up in one H2D, lookup + gather + decode run on the
// stream, the arrays come back in one D2H (small reads) -- the per-key
// MultiGet + ReadBatchBuilder of RocksDBStore::read (rocksdb/mod.rs:241-267)
// with no host work per key.
int murr_reader_read(murr_reader_t* r, const murr_index_t* x, const uint8_t* blob, const uint64_t* row_off,
                     uint64_t blob_bytes, uint64_t max_row, const uint8_t* key_data, const int32_t* key_offsets,
                     uint64_t key_offset, uint64_t nq, const uint32_t* proj, uint32_t nproj,
                     murr_host_array_t* outs, murr_error_t* err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!r || !x || (nproj && (!proj || !outs)) || (nq && (!key_offsets || !key_data)))
        return set_err(err, MURR_E_ARGUMENT);
    if (!nproj) return set_err(err, MURR_E_ARROW);  // no columns and no row count (table/mod.rs:124)
    for (uint32_t p = 0; p < nproj; p++)
        if (proj[p] >= r->seg.ncols) return set_err(err, MURR_E_BAD_COLUMN);
    murr_ctx* c = r->ctx;
    if (x->device != c->device || c->pending) return set_err(err, MURR_E_ARGUMENT);
    if (nq >= kMissing) return set_err(err, MURR_E_ARGUMENT);
    HIPC(hipSetDevice(c->device));
    // 1. keys: rebased offsets + bytes in pinned staging, one H2D
    const int32_t k0 = nq ? key_offsets[key_offset] : 0;
    const uint64_t kbytes = nq ? (uint64_t)(key_offsets[key_offset + nq] - k0) : 0;
    const uint64_t offb = round_up((nq + 1) * 4, 64);
    const uint64_t hk = offb + round_up(kbytes, 16) + 16;
    if (!grow_pinned(c, &r->hkeys, &r->hkeys_cap, hk, 0)) return set_err(err, MURR_E_HIP);
    int32_t* ho = (int32_t*)r->hkeys;
    ho[0] = 0;
    for (uint64_t i = 1; i <= nq; i++) ho[i] = key_offsets[key_offset + i] - k0;
    if (kbytes) std::memcpy(r->hkeys + offb, key_data + k0, kbytes);
    // 2. device work: keys | out_row_off | rows | needed | gathered rows
    const uint64_t fixed = (uint64_t)r->seg.bitset_size + r->seg.capacity;
    const uint64_t bound = std::max<uint64_t>(nq * max_row, 16);
    const bool two_phase = bound > kTwoPhaseBytes;
    const uint64_t o_off = round_up(hk, 256), o_rows = round_up(o_off + (nq + 1) * 8, 256),
                   o_need = round_up(o_rows + (nq + 1) * 4, 256), o_data = o_need + 256;
    uint64_t data_cap = two_phase ? 0 : bound;
    if (!grow_dev(c, &r->dwork, &r->dwork_cap, o_data + data_cap + 16)) return set_err(err, MURR_E_HIP);
    uint8_t* w = r->dwork;
    HIPC(hipMemcpyAsync(w, r->hkeys, hk, hipMemcpyHostToDevice, c->stream));
    const int32_t* dq_off = (const int32_t*)w;
    const uint8_t* dq_data = w + offb;
    uint64_t* doff = (uint64_t*)(w + o_off);
    uint32_t* drows = (uint32_t*)(w + o_rows);
    uint64_t* dneed = (uint64_t*)(w + o_need);
    uint64_t gathered = bound;
    int st;
    if (!two_phase) {
        st = murr_index_gather(c, x, dq_data, dq_off, nq, blob, row_off, w + o_data, data_cap, doff, nullptr, dneed);
        if (st) return set_err(err, st);
    } else {
        // exact sizing: lookup + offsets, one 8-byte read-back, then the copy
        st = murr_index_gather(c, x, dq_data, dq_off, nq, blob, row_off, nullptr, 0, doff, drows, dneed);
        if (st) return set_err(err, st);
        HIPC(hipMemcpyAsync(&gathered, dneed, 8, hipMemcpyDeviceToHost, c->stream));
        HIPC(hipStreamSynchronize(c->stream));
        if (!grow_dev(c, &r->dwork, &r->dwork_cap, o_data + gathered + 16)) {
            // grow_dev does not keep contents: redo the first phase on the new buffer
            return set_err(err, MURR_E_HIP);
        }
        if (r->dwork != w) {
            w = r->dwork;
            HIPC(hipMemcpyAsync(w, r->hkeys, hk, hipMemcpyHostToDevice, c->stream));
            dq_off = (const int32_t*)w;
            dq_data = w + offb;
            doff = (uint64_t*)(w + o_off);
            drows = (uint32_t*)(w + o_rows);
            dneed = (uint64_t*)(w + o_need);
            st = murr_index_gather(c, x, dq_data, dq_off, nq, blob, row_off, nullptr, 0, doff, drows, dneed);
            if (st) return set_err(err, st);
        }
        st = murr_index_gather_copy(c, drows, nq, blob, row_off, doff, w + o_data);
        if (st) return set_err(err, st);
    }
    // 3. decode + D2H.  The tile-sizing hint is the table's mean row x keys
    // (never read past: rows end at doff[nq]).
    const uint64_t mean = x->n ? blob_bytes / x->n : fixed;
    const uint64_t hint = std::min<uint64_t>(gathered, std::max<uint64_t>(16, mean * nq));
    murr_block_t blk{w + o_data, doff, nq, two_phase ? std::max<uint64_t>(gathered, 16) : hint, nullptr};
    const uint64_t utf8_cap = two_phase ? gathered : (max_row > fixed ? nq * (max_row - fixed) : 0);
    return decode_to_host(c, &r->seg, proj, nproj, blk, utf8_cap, r->out, nullptr, nullptr, outs, err);
}

void murr_reader_free(murr_reader_t* r) {
    if (!r) return;
    murr_ctx* c = r->ctx;
    if (c) (void)hipSetDevice(c->device);
    pool_give(c, true, r->hkeys, r->hkeys_cap);
    pool_give(c, false, r->dwork, r->dwork_cap);
    pool_give(c, true, r->out.hout, r->out.hout_cap);
    pool_give(c, false, r->out.dout, r->out.dout_cap);
    delete r;
}

}  // extern "C"

// ---- prepared resident read (murr_read_plan_*) ------------------------------
// Table::read repeated with one projection and key-count class over a
// resident table (src/io/table/mod.rs:114-129 over src/io/store/memory.rs:
// 28-45, the shape benches/read_block.rs / read_plain.rs loop).  Made once:
// the gather's device work area, the decode's output buffers and its prepared
// launch (murr_decode_plan: descriptors and kernel arguments resident, the
// counters handed to pinned host memory by the kernel's last workgroup),
// pinned key staging and pinned arrays.  A run enqueues on the context's
// stream: lookup + gather (the probe reads host keys straight from pinned
// memory: no key copy), the decode, and (host variant) one segment-copy kernel
// of the arrays into pinned memory; then waits once.  No descriptor upload, no
// counter read-back copy, no copy engine.  A run of nq <= cap keys decodes cap
// rows: queries [nq, cap) are misses without a lookup (empty rows), and the
// arrays are reported at nq rows.

struct murr_read_plan {
    murr_ctx* ctx = nullptr;
    std::vector<murr_column_t> cols;
    murr_segment_t seg{};
    std::vector<uint32_t> proj;
    std::vector<uint32_t> dtypes;
    const murr_index_t* x = nullptr;
    const uint8_t* blob = nullptr;
    const uint64_t* row_off = nullptr;
    const uint32_t* row_ulen = nullptr;  // the table's per-row utf8 string bytes (null: none)
    uint32_t nu = 0;                     // utf8 columns the gather indexes (0: split-mode decode)
    uint64_t cap = 0, data_cap = 0, utf8_cap = 0;
    uint8_t* dwork = nullptr;  // device: gather offsets (cap+1) | rows (cap) | needed | utf8 index | gathered rows
    uint64_t dwork_cap = 0;
    uint64_t* doff = nullptr;
    uint32_t* drows = nullptr;
    uint64_t* dneed = nullptr;
    uint64_t* duidx = nullptr;  // the gathered block's utf8 index, stride 64 (written by the gather)
    uint8_t* ddata = nullptr;
    uint8_t* hkeys = nullptr;  // pinned: rebased key offsets (cap + 1), then the key bytes
    uint64_t hkeys_cap = 0;
    HostOut out;
    std::vector<CopySeg> d2h;  // the arrays into pinned memory (host runs)
    murr_plan* dplan = nullptr;
    hipEvent_t ev = nullptr;
#ifdef MURR_TUNING
    // run phases (MURR_READ_PHASES=1, printed at free), ms summed over runs:
    // 0 keys staged, 1 gather (+ index) launches, 2 decode launch, 3 D2H
    // launch, 4 decode wait, 5 D2H wait
    double ph[6] = {0, 0, 0, 0, 0, 0};
    uint64_t runs = 0;
    // gather_fused's phase clocks (MURR_GATHER_STAMPS=1), us summed over runs:
    // 0 dispatch skew, 1 probe, 2 look-back, 3 publish, 4 copy (means over
    // groups), 5 span, 6 the slowest group's look-back; [0] device runs, [1]
    // host runs (keys read over PCIe)
    uint64_t* dstamps = nullptr;
    double gs[2][7] = {};
    uint64_t gruns[2] = {0, 0};
#endif
};

namespace {
#ifdef MURR_TUNING
struct RunClock {
    double* ph;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(int k) {
        const auto now = std::chrono::steady_clock::now();
        ph[k] += std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
    }
};
#define RP_CLOCK RunClock rc{r->ph}; r->runs++
#define RP_LAP(k) rc.lap(k)
#else
#define RP_CLOCK ((void)0)
#define RP_LAP(k) ((void)0)
#endif

int read_plan_gather(murr_read_plan* r, const uint8_t* q_data, const int32_t* q_off, uint64_t nq) {
    murr_ctx* c = r->ctx;
    murr_error_t* err = nullptr;
    if (const int st = ensure_aux(c, gather_scratch_words(r->cap), err)) return st;
    IndexArgs a = index_args(r->x, q_data, q_off, r->cap);
    a.nq_live = nq;  // (>= 1: a run of no keys launches nothing)
    a.rows = r->drows;
    a.blob = r->blob;
    a.row_off = r->row_off;
    a.sizes = r->doff;
    a.out = r->ddata;
    a.out_cap = r->data_cap;
    a.needed = r->dneed;
    a.scratch = c->aux;
    if (const int st = small_gather_words(c, &a, err)) return st;
    if (r->nu) {  // (set only when the fused gather runs: cap <= 1024)
        if (!a.lb) return MURR_E_INTERNAL;
        a.ulen = r->row_ulen;
        a.uidx = r->duidx;
        a.nu = r->nu;
    }
    const murr_index* x = r->x;
    bool use_rc = x->rc && x->cached == x->n && (!r->nu || x->rc_nu == r->nu);  // the slot cache holds every row
#ifdef MURR_TUNING
    if (std::getenv("MURR_INDEX_NOCACHE")) use_rc = false;  // (A/B)
#endif
    if (use_rc) {
        a.kp = x->kp;
        a.rc = x->rc;
        a.ru = x->ru;
        a.nu_rc = x->rc_nu;
    }
#ifdef MURR_TUNING
    if (a.lb && std::getenv("MURR_GATHER_STAMPS")) {
        if (!r->dstamps) HIPC(hipMalloc(&r->dstamps, 8 * kGatherGroups * kGatherStamps));
        a.stamps = r->dstamps;
    }
#endif
    HIPC(launch_gather(a, c->stream));
    return MURR_OK;
}

#ifdef MURR_TUNING
// One run's gather phase clocks (after its wait), into r->gs.
void read_plan_stamps(murr_read_plan* r, int host) {
    if (!r->dstamps) return;
    const uint32_t G = (uint32_t)((r->cap + 63) / 64);
    uint64_t t[kGatherGroups * kGatherStamps];
    if (hipMemcpy(t, r->dstamps, 8 * G * kGatherStamps, hipMemcpyDeviceToHost) != hipSuccess) return;
    uint64_t b = ~0ull, e = 0, s0 = 0, lbmax = 0;
    double ph[4] = {0, 0, 0, 0};
    for (uint32_t g = 0; g < G; g++) {
        const uint64_t* x = t + g * kGatherStamps;
        b = std::min(b, x[0]);
        s0 = std::max(s0, x[0]);
        e = std::max(e, x[4]);
        lbmax = std::max(lbmax, x[2] - x[1]);
        for (uint32_t k = 0; k < 4; k++) ph[k] += (double)(x[k + 1] - x[k]);
    }
    double* gs = r->gs[host];
    gs[0] += (s0 - b) * 0.01;  // (100 MHz ticks -> us)
    for (uint32_t k = 0; k < 4; k++) gs[1 + k] += ph[k] / G * 0.01;
    gs[5] += (e - b) * 0.01;
    gs[6] += lbmax * 0.01;
    r->gruns[host]++;
}
#define RP_STAMPS(host) read_plan_stamps(r, host)
#else
#define RP_STAMPS(host) ((void)0)
#endif

// The plan's arrays at nq rows (padding rows are misses: null in every column).
void read_plan_report(const murr_read_plan* r, uint64_t nq, murr_array_t* dev, murr_host_array_t* host) {
    const uint64_t pad = r->cap - nq;
    for (size_t p = 0; p < r->proj.size(); p++) {
        const murr_array_t& a = r->out.arr[p];
        const uint32_t d = r->dtypes[p];
        const uint64_t nulls = a.null_count >= pad ? a.null_count - pad : 0;
        const uint64_t vlen = d == MURR_UTF8 ? a.data_len : d == MURR_BOOL ? (nq + 7) / 8 : nq * (uint64_t)dtype_size(d);
        if (dev) {
            dev[p] = a;
            dev[p].null_count = nulls;
            dev[p].data_len = vlen;
        }
        if (host) {
            murr_host_array_t& h = host[p];
            h.values = r->out.hout + r->out.off[3 * p];
            h.validity = nulls ? r->out.hout + r->out.off[3 * p + 1] : nullptr;
            h.offsets = a.offsets ? (const int32_t*)(r->out.hout + r->out.off[3 * p + 2]) : nullptr;
            h.length = nq;
            h.null_count = nulls;
            h.values_len = vlen;
            h.dtype = d;
            h._pad = 0;
        }
    }
}
}  // namespace

extern "C" {

int murr_read_plan_new(murr_ctx_t* c, const murr_segment_t* seg, const murr_index_t* x, const uint8_t* arena,
                       const uint64_t* row_off, const uint32_t* row_ulen, uint64_t arena_bytes, uint64_t max_row,
                       const uint32_t* proj, uint32_t nproj, uint64_t cap, murr_read_plan_t** out) {
    murr_error_t* err = nullptr;
    if (!out) return MURR_E_ARGUMENT;
    *out = nullptr;
    if (!c || !x || !valid_segment(seg) || !row_off || !proj || !nproj || !cap || cap >= kMissing ||
        x->device != c->device || c->pending || (x->n && !arena))
        return MURR_E_ARGUMENT;
    for (uint32_t p = 0; p < nproj; p++)
        if (proj[p] >= seg->ncols) return MURR_E_BAD_COLUMN;
    const uint64_t fixed = (uint64_t)seg->bitset_size + seg->capacity;
    const uint64_t data_cap = std::max<uint64_t>(cap * max_row, 16);
    if (data_cap > kTwoPhaseBytes) return MURR_E_ARGUMENT;  // (such reads size their gather exactly: murr_reader_read)
    HIPC(hipSetDevice(c->device));
    std::unique_ptr<murr_read_plan, void (*)(murr_read_plan*)> r(new (std::nothrow) murr_read_plan(),
                                                                 [](murr_read_plan* q) { murr_read_plan_free(q); });
    if (!r) return MURR_E_INTERNAL;
    r->ctx = c;
    r->cols.assign(seg->cols, seg->cols + seg->ncols);
    r->seg = *seg;
    r->seg.cols = r->cols.data();
    r->proj.assign(proj, proj + nproj);
    for (uint32_t p = 0; p < nproj; p++) r->dtypes.push_back(seg->cols[proj[p]].dtype);
    r->x = x;
    r->blob = arena;
    r->row_off = row_off;
    r->cap = cap;
    r->data_cap = data_cap;
    r->utf8_cap = max_row > fixed ? cap * (max_row - fixed) : 0;
    // the gathered block's utf8 index, built by the fused gather from the
    // table's per-row string bytes (§3.4): layouts of 1 .. kGatherMaxU utf8
    // columns and up to 1024 keys; otherwise the decode takes the block in
    // split mode
    uint32_t nu = 0;
    for (uint32_t i = 0; i < seg->ncols; i++) nu += seg->cols[i].dtype == MURR_UTF8;
    r->row_ulen = row_ulen;
    r->nu = row_ulen && nu >= 1 && nu <= kGatherMaxU && cap <= 64 * kGatherGroups ? nu : 0u;
#ifdef MURR_TUNING
    if (std::getenv("MURR_READ_NOIDX")) r->nu = 0;
#endif
    // device work: offsets | rows | needed | utf8 index | gathered rows (16-B aligned)
    const uint64_t o_rows = round_up((cap + 1) * 8, 256), o_need = round_up(o_rows + cap * 4, 256),
                   o_uidx = o_need + 256, o_data = round_up(o_uidx + 8 * ((cap + 63) / 64 + 1) * std::max(nu, 1u), 256);
    if (!grow_dev(c, &r->dwork, &r->dwork_cap, o_data + data_cap + 16)) return MURR_E_HIP;
    r->doff = (uint64_t*)r->dwork;
    r->drows = (uint32_t*)(r->dwork + o_rows);
    r->dneed = (uint64_t*)(r->dwork + o_need);
    r->duidx = (uint64_t*)(r->dwork + o_uidx);
    r->ddata = r->dwork + o_data;
    // arrays: the fixed-size parts first (values, validity, utf8 offsets), then
    // the utf8 bytes, so the D2H is one segment plus one per utf8 column
    HostOut& o = r->out;
    const uint64_t bm = murr_bitmap_bytes(cap);
    o.off.assign((size_t)nproj * 3, 0);
    uint64_t off = 0;
    for (uint32_t p = 0; p < nproj; p++) {
        const murr_column_t& col = seg->cols[proj[p]];
        if (col.dtype != MURR_UTF8) {
            o.off[3 * p] = off;
            off = round_up(off + std::max<uint64_t>(col.dtype == MURR_BOOL ? bm : cap * col.size, 8), 64);
        }
        o.off[3 * p + 1] = off;
        off = round_up(off + std::max<uint64_t>(bm, 8), 64);
        if (col.dtype == MURR_UTF8) {
            o.off[3 * p + 2] = off;
            off = round_up(off + (cap + 1) * 4, 64);
        }
    }
    const uint64_t fixed_out = std::max<uint64_t>(off, 64);
    for (uint32_t p = 0; p < nproj; p++)
        if (seg->cols[proj[p]].dtype == MURR_UTF8) {
            o.off[3 * p] = off;
            off = round_up(off + std::max<uint64_t>(r->utf8_cap, 8), 64);
        }
    const uint64_t total_out = std::max<uint64_t>(off, 64);
    if (!grow_dev(c, &o.dout, &o.dout_cap, total_out) || !grow_pinned(c, &o.hout, &o.hout_cap, total_out, 0))
        return MURR_E_HIP;
    o.arr.assign(nproj, murr_array_t{});
    r->d2h.assign({CopySeg{o.dout, o.hout, fixed_out, nullptr}});
    for (uint32_t p = 0; p < nproj; p++) {
        murr_array_t& a = o.arr[p];
        a.values = o.dout + o.off[3 * p];
        a.validity = o.dout + o.off[3 * p + 1];
        a.offsets = seg->cols[proj[p]].dtype == MURR_UTF8 ? (int32_t*)(o.dout + o.off[3 * p + 2]) : nullptr;
        a.values_cap = r->utf8_cap;
        if (a.offsets)  // exactly the decoded bytes: the length is the final offset, read on the device
            r->d2h.push_back(CopySeg{o.dout + o.off[3 * p], o.hout + o.off[3 * p], r->utf8_cap, a.offsets + cap});
    }
    // the decode, prepared over the gather's block (its tile-sizing hint: the
    // table's mean row x cap; rows end at doff[cap], never read past)
    const uint64_t mean = x->n ? arena_bytes / x->n : fixed;
    murr_block_t blk{r->ddata, r->doff, cap, std::min<uint64_t>(data_cap, std::max<uint64_t>(16, mean * cap)), nullptr};
    // With the gather's utf8 index the decode cuts the block into one-pass
    // virtual blocks; without one it takes the block in split mode (two
    // passes and a look-back).  Indexing the gathered block in kernels of its
    // own -- murr_utf8_index's two, or a one-workgroup gather that also
    // indexed -- cost more than the single pass saved.
    const uint64_t* ux[1] = {r->duidx};
    int st = murr_decode_plan(c, &r->seg, r->proj.data(), nproj, &blk, 1, r->nu ? ux : nullptr, r->nu ? 64u : 0u,
                              o.arr.data(), &r->dplan);
    if (st) return st;
    (void)murr_plan_time_every(r->dplan, 0);  // (no timing events between the run's kernels)
    HIPC(hipEventCreateWithFlags(&r->ev, hipEventDisableTiming));
    *out = r.release();
    return MURR_OK;
}

int murr_read_plan_run_device(murr_read_plan_t* r, const uint8_t* q_data, const int32_t* q_offsets, uint64_t nq,
                              murr_array_t* outs, murr_error_t* err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!r || !outs || nq > r->cap || (nq && (!q_data || !q_offsets))) return set_err(err, MURR_E_ARGUMENT);
    murr_ctx* c = r->ctx;
    if (c->pending) return set_err(err, MURR_E_ARGUMENT);
    if (!nq) {  // no keys: empty arrays, nothing launched
        for (size_t p = 0; p < r->proj.size(); p++) {
            outs[p] = r->out.arr[p];
            outs[p].null_count = outs[p].data_len = 0;
        }
        return MURR_OK;
    }
    HIPC(hipSetDevice(c->device));
    RP_CLOCK;
    int st = read_plan_gather(r, q_data, q_offsets, nq);
    if (st) return set_err(err, st);
    RP_LAP(1);
    st = murr_decode_run_async(r->dplan);
    if (st) return set_err(err, st);
    RP_LAP(2);
    st = plan_wait(r->dplan, err, false);  // (its outputs are consumed on c->stream)
    if (st) return st;
    RP_LAP(4);
    RP_STAMPS(0);
    read_plan_report(r, nq, outs, nullptr);
    return MURR_OK;
}

int murr_read_plan_run(murr_read_plan_t* r, const uint8_t* key_data, const int32_t* key_offsets, uint64_t key_offset,
                       uint64_t nq, murr_host_array_t* outs, murr_error_t* err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!r || !outs || nq > r->cap || (nq && (!key_data || !key_offsets))) return set_err(err, MURR_E_ARGUMENT);
    murr_ctx* c = r->ctx;
    if (c->pending) return set_err(err, MURR_E_ARGUMENT);
    if (!nq) {  // no keys: empty arrays, nothing launched
        for (size_t p = 0; p < r->proj.size(); p++)
            outs[p] = murr_host_array_t{r->out.hout, nullptr, r->out.arr[p].offsets ? (const int32_t*)r->out.hout : nullptr,
                                        0, 0, 0, r->dtypes[p], 0};
        std::memset(r->out.hout, 0, 8);  // (the one offset of an empty utf8 array: 0)
        return MURR_OK;
    }
    HIPC(hipSetDevice(c->device));
    RP_CLOCK;
    // keys: rebased offsets + bytes in pinned staging, read by the probe in place
    const int32_t k0 = nq ? key_offsets[key_offset] : 0;
    const uint64_t kbytes = nq ? (uint64_t)(key_offsets[key_offset + nq] - k0) : 0;
    const uint64_t offb = round_up((nq + 1) * 4, 64);
    if (!grow_pinned(c, &r->hkeys, &r->hkeys_cap, offb + round_up(kbytes, 16) + 16, 0)) return set_err(err, MURR_E_HIP);
    int32_t* ho = (int32_t*)r->hkeys;
    ho[0] = 0;
    for (uint64_t i = 1; i <= nq; i++) ho[i] = key_offsets[key_offset + i] - k0;
    if (kbytes) std::memcpy(r->hkeys + offb, key_data + k0, kbytes);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    RP_LAP(0);
    int st = read_plan_gather(r, r->hkeys + offb, ho, nq);
    if (st) return set_err(err, st);
    RP_LAP(1);
    st = murr_decode_run_async(r->dplan);
    if (st) return set_err(err, st);
    RP_LAP(2);
    // the arrays into pinned memory, queued behind the decode on the same stream
    HIPC(launch_copy_segs(r->d2h.data(), (uint32_t)r->d2h.size(), kCopyGridOut, c->stream));
    HIPC(hipEventRecord(r->ev, c->stream));
    RP_LAP(3);
    st = plan_wait(r->dplan, err, false);  // (its outputs are consumed on c->stream)
    if (st) {
        (void)hipEventSynchronize(r->ev);
        return st;
    }
    RP_LAP(4);
    HIPC(hipEventSynchronize(r->ev));
    RP_LAP(5);
    RP_STAMPS(1);
    read_plan_report(r, nq, nullptr, outs);
    return MURR_OK;
}

uint64_t murr_read_plan_capacity(const murr_read_plan_t* r) { return r ? r->cap : 0; }

void murr_read_plan_free(murr_read_plan_t* r) {
    if (!r) return;
#ifdef MURR_TUNING
    if (std::getenv("MURR_READ_PHASES") && r->runs)
        std::fprintf(stderr,
                     "read plan phases (us per run over %llu, cap %llu): keys %.2f  gather %.2f  decode launch %.2f  "
                     "d2h launch %.2f  decode wait %.2f  d2h wait %.2f\n",
                     (unsigned long long)r->runs, (unsigned long long)r->cap, r->ph[0] * 1e3 / r->runs,
                     r->ph[1] * 1e3 / r->runs, r->ph[2] * 1e3 / r->runs, r->ph[3] * 1e3 / r->runs,
                     r->ph[4] * 1e3 / r->runs, r->ph[5] * 1e3 / r->runs);
    for (int h = 0; h < 2; h++)
        if (r->gruns[h]) {
            const double* gs = r->gs[h];
            const double n = (double)r->gruns[h];
            std::fprintf(stderr,
                         "gather stamps, %s runs (us per run over %llu, %llu groups; means over groups): dispatch skew "
                         "%.2f  probe %.2f  look-back %.2f (slowest %.2f)  publish %.2f  copy %.2f  span %.2f\n",
                         h ? "host" : "device", (unsigned long long)r->gruns[h],
                         (unsigned long long)((r->cap + 63) / 64), gs[0] / n, gs[1] / n, gs[2] / n, gs[6] / n,
                         gs[3] / n, gs[4] / n, gs[5] / n);
        }
    if (r->dstamps) (void)hipFree(r->dstamps);
#endif
    murr_ctx* c = r->ctx;
    if (c) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    if (r->dplan) murr_plan_free(r->dplan);
    if (r->ev) (void)hipEventDestroy(r->ev);
    pool_give(c, true, r->hkeys, r->hkeys_cap);
    pool_give(c, false, r->dwork, r->dwork_cap);
    pool_give(c, true, r->out.hout, r->out.hout_cap);
    pool_give(c, false, r->out.dout, r->out.dout_cap);
    delete r;
}

}  // extern "C"

extern "C" {

// ---- RocksDB data blocks (murr_sst.hip) --------------

void murr_sst_result_free(murr_ctx_t* c, murr_sst_result_t* r) {
    if (!r) return;
    if (c) (void)hipSetDevice(c->device);
    for (void* p : {(void*)r->keys, (void*)r->key_offsets, (void*)r->values, (void*)r->value_offsets,
                    (void*)r->seqs, (void*)r->types})
        if (p && !(c && dev_free_cached(c, p))) {
            dev_forget(p);  // (no context: a recorded output is released, and its record with it)
            (void)hipFree(p);
        }
    std::memset(r, 0, sizeof *r);
}

// Decode data blocks into entries: sst_count (a thread per block inflates a
// tier-0 block into its HBM slot and counts its entries; larger blocks are
// flagged tier 1 or 2), the scans placing every
// block's entries, one 40-byte read-back that sizes the outputs, sst_decode.
// Tier-2 blocks add a raw buffer, sst_big_count and a second read-back.
// Scratch comes from the context pool.  Synchronous.
int murr_sst_decode(murr_ctx_t* c, const murr_sst_block_t* blocks, uint32_t nblocks, murr_sst_result_t* out,
                    murr_error_t* err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!c || !out || (nblocks && !blocks) || c->pending) return set_err(err, MURR_E_ARGUMENT);
    std::memset(out, 0, sizeof *out);
    HIPC(hipSetDevice(c->device));
    bool dev_table = false;  // the descriptors in device memory (used in place)
    if (nblocks) {
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, blocks) == hipSuccess) dev_table = at.type == hipMemoryTypeDevice;
        else (void)hipGetLastError();
    }
    if (!dev_table)
        for (uint32_t b = 0; b < nblocks; b++)
            if (blocks[b].size && !blocks[b].data) return set_err(err, MURR_E_ARGUMENT);
    const uint64_t nb = nblocks, nparts = (nb + 1023) / 1024;
    // scratch: err | totals[5] | nlist | descriptors | tier rlen list | ulen uoff ne kb vb eoff koff voff | parts
    const uint64_t o_tot = 8, o_nlist = 56, o_desc = 64, o_tier = round_up(o_desc + sizeof(SstBlock) * nb, 16);
    const uint64_t o_arr = round_up(o_tier + 3 * 4 * nb, 16), o_part = o_arr + 8 * 8 * nb;
    const uint64_t scratch_bytes = o_part + 8 * 4 * std::max<uint64_t>(nparts, 1) + 64;
    const uint64_t slot_bytes = kSstSlot * nb + 64;  // tier-0 blocks between sst_count and sst_decode
    uint8_t *w = nullptr, *raw = nullptr, *slots = nullptr;
    uint64_t w_cap = 0, raw_cap = 0, slots_cap = 0;
    if (!pool_take(c, false, scratch_bytes, round_up(scratch_bytes, 1 << 20), &w, &w_cap))
        return set_err(err, MURR_E_HIP, (int)hipErrorOutOfMemory);
    if (!pool_take(c, false, slot_bytes, round_up(slot_bytes, 1 << 20), &slots, &slots_cap)) {
        pool_give(c, false, w, w_cap);
        return set_err(err, MURR_E_HIP, (int)hipErrorOutOfMemory);
    }
    auto fail = [&](int st) {
        (void)hipStreamSynchronize(c->stream);
        pool_give(c, false, w, w_cap);
        pool_give(c, false, slots, slots_cap);
        pool_give(c, false, raw, raw_cap);
        murr_sst_result_free(c, out);
        return st;
    };
#define SSTC(expr)                                                           \
    do {                                                                     \
        hipError_t _e = (expr);                                              \
        if (_e != hipSuccess) return fail(set_err(err, MURR_E_HIP, (int)_e)); \
    } while (0)
    static_assert(sizeof(SstBlock) == sizeof(murr_sst_block_t), "murr_sst_block_t is the device descriptor");
    SSTC(hipMemsetAsync(w, 0, 64, c->stream));
    if (nb && !dev_table)
        SSTC(hipMemcpyAsync(w + o_desc, blocks, sizeof(SstBlock) * nb, hipMemcpyHostToDevice, c->stream));
    SstArgs a{};
    a.blocks = dev_table ? (const SstBlock*)blocks : (const SstBlock*)(w + o_desc);
    a.nblocks = nb;
    a.tier = (uint32_t*)(w + o_tier);
    a.rlen = a.tier + nb;
    a.list = a.tier + 2 * nb;
    a.nlist = (uint32_t*)(w + o_nlist);
    a.slots = slots;
    uint64_t* arr = (uint64_t*)(w + o_arr);
    a.ulen = arr;
    a.uoff = arr + nb;
    a.ne = arr + 2 * nb;
    a.kb = arr + 3 * nb;
    a.vb = arr + 4 * nb;
    a.eoff = arr + 5 * nb;
    a.koff = arr + 6 * nb;
    a.voff = arr + 7 * nb;
    a.err = (unsigned long long*)w;
    uint64_t* tot = (uint64_t*)(w + o_tot);  // [0] entries [1] key bytes [2] value bytes [3] big bytes
    uint64_t* part = (uint64_t*)(w + o_part);
    uint64_t host[5] = {0, 0, 0, 0, 0};  // err, totals
    // entries, key bytes, value bytes (and after the count pass tier-2 raw bytes)
    auto scans = [&](bool with_raw) -> hipError_t {
        hipError_t e;
        ScanSet S{{a.ne, a.kb, a.vb, a.ulen}, {a.eoff, a.koff, a.voff, a.uoff}, {tot, tot + 1, tot + 2, tot + 3},
                  part, with_raw ? 4u : 3u, 0u};
        if ((e = launch_scan_u64_n(S, nb, c->stream)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(host, w, 40, hipMemcpyDeviceToHost, c->stream)) != hipSuccess) return e;
        return hipStreamSynchronize(c->stream);
    };
    if (nb) {
        SSTC(launch_sst_count(a, c->stream));
        SSTC(scans(true));
        if (host[4]) {  // big blocks: inflated to raw by one thread each, counted, placed again
            if (!pool_take(c, false, host[4] + 16, round_up(host[4] + 16, 1 << 20), &raw, &raw_cap))
                return fail(set_err(err, MURR_E_HIP, (int)hipErrorOutOfMemory));
            a.raw = raw;
            SSTC(launch_sst_big_count(a, c->stream));
            SSTC(scans(false));
        }
        if (host[0]) return fail(unpack_err(host[0], err));
    }
    const uint64_t n = host[1], kbytes = host[2], vbytes = host[3];
    if (kbytes > 0x7FFFFFFFull) return fail(set_err(err, MURR_E_OFFSET_OVERFLOW));
    // outputs (the caller's), then the entries
    // (through the context's reuse cache: murr_sst_result_free / murr_dev_free give them back)
    SSTC(dev_alloc_cached(c, kbytes + 16, (void**)&out->keys));
    SSTC(dev_alloc_cached(c, 4 * (n + 1), (void**)&out->key_offsets));
    SSTC(dev_alloc_cached(c, vbytes + 16, (void**)&out->values));
    SSTC(dev_alloc_cached(c, 8 * (n + 1), (void**)&out->value_offsets));
    SSTC(dev_alloc_cached(c, 8 * std::max<uint64_t>(n, 1), (void**)&out->seqs));
    SSTC(dev_alloc_cached(c, std::max<uint64_t>(n, 1), (void**)&out->types));
    SSTC(hipMemsetAsync(out->key_offsets, 0, 4, c->stream));
    SSTC(hipMemsetAsync(out->value_offsets, 0, 8, c->stream));
    out->n = n;
    out->key_bytes = kbytes;
    out->value_bytes = vbytes;
    if (n) {
        a.keys = out->keys;
        a.key_off = out->key_offsets;
        a.vals = out->values;
        a.val_off = out->value_offsets;
        a.seqs = out->seqs;
        a.types = out->types;
        SSTC(hipEventRecord(c->k0, c->stream));
        SSTC(launch_sst_decode(a, c->stream));
        if (raw) SSTC(launch_sst_big_decode(a, c->stream));
        SSTC(hipEventRecord(c->k1, c->stream));
        c->timed = true;
    c->lk0 = c->lk1 = nullptr;
        c->last_kernel = "sst_decode";
    }
    SSTC(hipStreamSynchronize(c->stream));
#undef SSTC
    pool_give(c, false, w, w_cap);
    pool_give(c, false, slots, slots_cap);
    pool_give(c, false, raw, raw_cap);
    return MURR_OK;
}

// Host-memory encode: H2D Arrow buffers, murr_encode_batch, D2H blobs + offsets.
int murr_encode_host(murr_ctx_t* c, const murr_segment_t* seg, const murr_host_col_in_t* cols,
                     uint64_t n, uint8_t** out_blob, uint64_t* blob_len, uint64_t** out_row_off,
                     murr_error_t* err) {
    if (!c || !valid_segment(seg) || (seg->ncols && !cols) || !out_blob || !blob_len || !out_row_off)
        return set_err(err, MURR_E_ARGUMENT);
    HIPC(hipSetDevice(c->device));
    std::vector<void*> dbufs;
    auto cleanup = [&]() { for (void* p : dbufs) (void)hipFree(p); };
    std::vector<murr_col_in_t> din(seg->ncols);
    std::vector<uint64_t> utf8_bytes(seg->ncols, 0);
    auto up = [&](const void* h, uint64_t bytes, const void** d) -> int {
        *d = nullptr;
        if (!h) return MURR_OK;
        void* p = nullptr;
        if (hipMalloc(&p, round_up(bytes ? bytes : 1, 16) + 16) != hipSuccess) return MURR_E_HIP;
        dbufs.push_back(p);
        if (bytes && hipMemcpyAsync(p, h, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess)
            return MURR_E_HIP;
        *d = p;
        return MURR_OK;
    };
    for (uint32_t i = 0; i < seg->ncols; i++) {
        const murr_host_col_in_t& hc = cols[i];
        const uint32_t dt = seg->cols[i].dtype;
        const uint64_t e = hc.col.offset + n;
        int st = up(hc.col.values, hc.values_bytes, &din[i].values);
        if (!st) st = up(hc.col.validity, (e + 7) / 8, (const void**)&din[i].validity);
        if (!st && dt == MURR_UTF8) st = up(hc.col.offsets, (e + 1) * 4, (const void**)&din[i].offsets);
        din[i].offset = hc.col.offset;
        if (st) { cleanup(); return set_err(err, st); }
        if (dt == MURR_UTF8 && hc.col.offsets && n)
            utf8_bytes[i] = (uint64_t)(hc.col.offsets[e] - hc.col.offsets[hc.col.offset]);
    }
    const uint64_t cap = murr_encode_bound(seg, n, utf8_bytes.data());
    uint8_t* dblob = nullptr;
    uint64_t* doff = nullptr;
    if (hipMalloc(&dblob, round_up(cap + 16, 16)) != hipSuccess ||
        hipMalloc(&doff, (n + 1) * 8) != hipSuccess) {
        if (dblob) (void)hipFree(dblob);
        cleanup();
        return set_err(err, MURR_E_HIP);
    }
    dbufs.push_back(dblob);
    dbufs.push_back(doff);
    uint64_t len = 0;
    int st = murr_encode_batch(c, seg, din.data(), n, dblob, cap, doff, &len, err);
    if (st) { cleanup(); return st; }
    uint8_t* hb = nullptr;
    uint64_t* ho = nullptr;
    if (hipHostMalloc(&hb, round_up(len + 16, 16), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&ho, (n + 1) * 8, hipHostMallocDefault) != hipSuccess) {
        if (hb) (void)hipHostFree(hb);
        cleanup();
        return set_err(err, MURR_E_HIP);
    }
    hipError_t e1 = len ? hipMemcpyAsync(hb, dblob, len, hipMemcpyDeviceToHost, c->stream) : hipSuccess;
    hipError_t e2 = hipMemcpyAsync(ho, doff, (n + 1) * 8, hipMemcpyDeviceToHost, c->stream);
    hipError_t e3 = hipStreamSynchronize(c->stream);
    cleanup();
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess) {
        (void)hipHostFree(hb);
        (void)hipHostFree(ho);
        return set_err(err, MURR_E_HIP, (int)(e1 ? e1 : e2 ? e2 : e3));
    }
    *out_blob = hb;
    *blob_len = len;
    *out_row_off = ho;
    return MURR_OK;
}

}  // extern "C"

// ---- Arrow IPC framing on the device (murr_ipc.cpp plans, murr_ipc.hip packs) ----
extern "C" {

int murr_ipc_batch_device(murr_ctx_t* c, const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj,
                          const murr_array_t* arrays, uint64_t n_rows, uint32_t alignment, uint8_t* dev_out,
                          uint64_t cap, uint64_t* out_len, murr_error_t* err) {
    set_err(err, MURR_OK);
    if (!c || !out_len || !valid_segment(seg) || (nproj && (!proj || !arrays)) || !ipc_align_ok(alignment))
        return set_err(err, MURR_E_ARGUMENT);
    if (!nproj) return set_err(err, MURR_E_ARROW);  // RecordBatch without columns (read.rs:106-108)
    std::vector<uint64_t> nulls(nproj), lens(nproj);
    for (uint32_t p = 0; p < nproj; p++) {
        if (proj[p] >= seg->ncols) return set_err(err, MURR_E_BAD_COLUMN);
        nulls[p] = arrays[p].null_count;
        lens[p] = arrays[p].data_len;
    }
    IpcPlan plan;
    ipc_batch_plan(seg, proj, nproj, n_rows, nulls.data(), lens.data(), alignment, &plan);
    const uint64_t meta = plan.meta.size(), total = meta + plan.body_len;
    *out_len = total;
    if (!dev_out) return MURR_OK;
    if (cap < total) {
        set_err(err, MURR_E_CAPACITY);
        if (err) err->required = total;
        return MURR_E_CAPACITY;
    }
    // Job table + metadata bytes, staged through pinned memory in one H2D.
    std::vector<IpcJob> jobs;
    jobs.reserve(plan.buf_off.size() + 1);
    jobs.push_back(IpcJob{nullptr, dev_out, meta, meta});  // src patched below
    uint64_t max_padded = meta;
    for (size_t i = 0; i < plan.buf_off.size(); i++) {
        const uint64_t len = plan.buf_len[i];
        const uint64_t padded = round_up(len, alignment);
        if (!padded) continue;
        const murr_array_t& a = arrays[plan.buf_field[i]];
        const void* src = plan.buf_kind[i] == kIpcValidity  ? (const void*)a.validity
                          : plan.buf_kind[i] == kIpcOffsets ? (const void*)a.offsets
                                                            : a.values;
        if (!src) return set_err(err, MURR_E_ARGUMENT);
        jobs.push_back(IpcJob{(const uint8_t*)src, dev_out + meta + plan.buf_off[i], len, padded});
        max_padded = std::max(max_padded, padded);
    }
    const uint64_t jb = round_up(jobs.size() * sizeof(IpcJob), 16), stage = jb + meta;
    uint8_t *hp = nullptr, *dp = nullptr;
    uint64_t hcap = 0, dcap = 0;
    if (!pool_take(c, true, stage, std::max<uint64_t>(stage, 1 << 16), &hp, &hcap)) return set_err(err, MURR_E_HIP);
    if (!pool_take(c, false, stage, std::max<uint64_t>(stage, 1 << 16), &dp, &dcap)) {
        pool_give(c, true, hp, hcap);
        return set_err(err, MURR_E_HIP);
    }
    jobs[0].src = dp + jb;
    std::memcpy(hp, jobs.data(), jobs.size() * sizeof(IpcJob));
    std::memcpy(hp + jb, plan.meta.data(), meta);
    hipError_t e = hipMemcpyAsync(dp, hp, stage, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_ipc_pack((const IpcJob*)dp, (uint32_t)jobs.size(), max_padded, c->stream);
    hipError_t e2 = hipStreamSynchronize(c->stream);
    pool_give(c, true, hp, hcap);
    pool_give(c, false, dp, dcap);
    if (e != hipSuccess || e2 != hipSuccess) return hip_fail(err, e != hipSuccess ? e : e2);
    c->last_kernel = "ipc_pack";
    return MURR_OK;
}

}  // extern "C"
