// murr_jit.cpp — run-time specialisation of the decode kernel.
//
// A table's segment layout (SegmentSchema, src/io/schema.rs:8-54) and a read's
// projection (Table::read, src/io/table/mod.rs:114-129) are fixed for the life
// of many batch reads, so the decode kernel is compiled for them: the host
// writes a prelude of #defines (bitset size, per projected column: kind, field
// offset, null bit; tile shape) in front of murr_jit_kernel.hip (embedded in
// this library) and compiles it with hiprtc for gfx950.  Code objects are
// cached per (device, prelude) for the life of the process.  A layout that
// cannot be compiled falls back to the generic kernel (murr_decode.hip).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/murr_codec.h"
#include "murr_internal.h"

namespace murr {

namespace {

const char* const kJitSrc =
#include "murr_jit_src.inc"
    ;
const char* const kJitEncSrc =
#include "murr_jit_encode_src.inc"
    ;

// ---- code-object cache ----------------------------------------------------------
//
// Compiled layouts are kept per (device, prelude) in memory (bounded, least
// recently used evicted) and on disk, so a process that opens a table whose
// layout an earlier process compiled loads the code object instead of running
// hiprtc.  Disk directory: $MURR_JIT_CACHE, else $HOME/.cache/murr ("0" or an
// unwritable directory disables it).

uint64_t fnv64(const std::string& s, uint64_t h = 0xcbf29ce484222325ull) {
    for (unsigned char ch : s) h = (h ^ ch) * 0x100000001b3ull;
    return h;
}

std::string cache_dir() {
    const char* e = std::getenv("MURR_JIT_CACHE");
    if (e) return std::string(e) == "0" ? std::string() : std::string(e);
    const char* home = std::getenv("HOME");
    if (!home || !*home) return std::string();
    return std::string(home) + "/.cache/murr";
}

bool read_file(const std::string& path, std::vector<char>* out) {
    FILE* fp = std::fopen(path.c_str(), "rb");
    if (!fp) return false;
    char buf[65536];
    size_t n;
    out->clear();
    while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) out->insert(out->end(), buf, buf + n);
    std::fclose(fp);
    return !out->empty();
}

void write_file_atomic(const std::string& dir, const std::string& name, const std::vector<char>& data) {
    if (dir.empty()) return;
    ::mkdir((dir.substr(0, dir.rfind('/'))).c_str(), 0755);
    ::mkdir(dir.c_str(), 0755);
    const std::string tmp = dir + "/." + name + "." + std::to_string((long)::getpid());
    FILE* fp = std::fopen(tmp.c_str(), "wb");
    if (!fp) return;
    const bool ok = std::fwrite(data.data(), 1, data.size(), fp) == data.size();
    std::fclose(fp);
    if (!ok || std::rename(tmp.c_str(), (dir + "/" + name).c_str()) != 0) std::remove(tmp.c_str());
}

// hiprtc compile of `src` for gfx950 (or the disk cache's copy of it).
bool compile_code(const std::string& src, const char* name, std::vector<char>* code, std::string* why) {
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    const std::string dir = cache_dir();
    std::string file;
    if (!dir.empty()) {
        // key: the source, the options and the compiler (hiprtc's version: a
        // code object from another ROCm release is never reused)
        int vmaj = 0, vmin = 0;
        if (hiprtcVersion(&vmaj, &vmin) != HIPRTC_SUCCESS) vmaj = vmin = -1;
        const std::string salt = std::string(opts[0]) + opts[1] + opts[2] + " hiprtc " + std::to_string(vmaj) + "." +
                                 std::to_string(vmin) + " " + std::to_string(HIP_VERSION);
        char hex[32];
        std::snprintf(hex, sizeof hex, "%016llx", (unsigned long long)fnv64(src, fnv64(salt)));
        file = std::string(name) + "-" + hex + ".co";
        if (read_file(dir + "/" + file, code)) return true;
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), name, 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        *why = "hiprtcCreateProgram failed";
        return false;
    }
    const hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
    if (r != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n + 1, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        *why = std::string("hiprtc: ") + hiprtcGetErrorString(r) + "\n" + log;
        hiprtcDestroyProgram(&prog);
        return false;
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    code->assign(n, 0);
    hiprtcGetCode(prog, code->data());
    hiprtcDestroyProgram(&prog);
    if (!file.empty()) write_file_atomic(dir, file, *code);
    return true;
}

// ---- decode: one module per segment layout ------------------------------------------

struct Entry {
    hipModule_t mod = nullptr;
    JitLayout k;
    bool ok = false;
    std::string why;
    uint64_t used = 0;
    int device = 0;
};

std::mutex g_mu;
std::map<std::string, std::unique_ptr<Entry>> g_cache;
uint64_t g_clock = 0;
size_t kMaxLayouts = 64;  // murr_jit_cache_limit (tests) may lower it

// Evict the least recently used layouts beyond kMaxLayouts, never `keep`
// (the entry being returned; caller holds g_mu).  A JitLayout pointer handed
// out earlier may still be in use: a launch enqueued on some stream, or a
// caller between jit_layout() and its launch.  So an evicted entry's module is
// not unloaded here: the entry moves to a retired list, and retired modules
// are unloaded only once the list passes kMaxLayouts, after a device-wide
// synchronise (every enqueued launch has finished by then) and only for
// entries not pinned (jit_layout(..., pin = true) until jit_layout_unpin).
std::vector<std::unique_ptr<Entry>> g_retired;
std::map<const JitLayout*, int> g_pins;

void evict(const Entry* keep) {
    while (g_cache.size() > kMaxLayouts) {
        auto victim = g_cache.end();
        for (auto it = g_cache.begin(); it != g_cache.end(); ++it)
            if (it->second.get() != keep && (victim == g_cache.end() || it->second->used < victim->second->used))
                victim = it;
        if (victim == g_cache.end()) return;
        g_retired.push_back(std::move(victim->second));
        g_cache.erase(victim);
    }
    if (g_retired.size() <= kMaxLayouts) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    std::vector<std::unique_ptr<Entry>> still;
    for (auto& e : g_retired) {
        if (g_pins.count(&e->k)) {
            still.push_back(std::move(e));
            continue;
        }
        if (e->mod) {
            (void)hipSetDevice(e->device);
            (void)hipDeviceSynchronize();
            (void)hipModuleUnload(e->mod);
        }
    }
    (void)hipSetDevice(cur);
    g_retired.swap(still);
}

// tuning builds (make tuning) only: MURR_JIT_DEFS="NAME=VALUE,..." extra
// #defines (ablation variants of the decode and encode kernels)
void tuning_defs(std::ostringstream& o) {
#ifndef MURR_TUNING
    (void)o;
#else
    if (const char* e = std::getenv("MURR_JIT_DEFS")) {
        std::string d(e);
        size_t pos = 0;
        while (pos < d.size()) {
            size_t end = d.find(',', pos);
            if (end == std::string::npos) end = d.size();
            std::string kv = d.substr(pos, end - pos);
            const size_t eq = kv.find('=');
            if (!kv.empty()) o << "#define " << (eq == std::string::npos ? kv : kv.substr(0, eq) + " " + kv.substr(eq + 1)) << "\n";
            pos = end + 1;
        }
    }
#endif
}

// Prelude: the segment layout (src/io/schema.rs:23-54), nothing of the
// projection.  MJ_COLS(X) lists every column as X(index, width, row offset of
// its field, utf8 ordinal); width 0 = utf8 slot, 9 = bool byte.
std::string prelude(const murr_segment_t* seg) {
    std::ostringstream o;
    uint32_t nu = 0;
    for (uint32_t c = 0; c < seg->ncols; c++) nu += seg->cols[c].dtype == MURR_UTF8;
    o << "#define MJ_BS " << seg->bitset_size << "\n#define MJ_FIX " << seg->bitset_size + seg->capacity
      << "\n#define MJ_NCOLS " << seg->ncols << "\n#define MJ_NUTF8 " << nu << "\n#define MJ_COLS(X)";
    for (uint32_t c = 0, u = 0; c < seg->ncols; c++) {
        const murr_column_t& col = seg->cols[c];
        const uint32_t w = col.dtype == MURR_UTF8 ? 0u : col.dtype == MURR_BOOL ? 9u : col.size;
        o << " X(" << col.index << ", " << w << ", " << seg->bitset_size + col.offset << ", "
          << (w == 0 ? u++ : 0u) << ")";
    }
    o << "\n";
    // non-temporal value and offset stores for layouts with 1- or 2-byte
    // columns (a wave's store of such a column is a partial line): C 0.475 ->
    // 0.465 ms, D shard 0.082 -> 0.074, D at 10 M rows 0.497 -> 0.482; B
    // (f32 + utf8, whole lines) 0.753 -> 0.772, so plain there
    // (profiles/r04/probes/ab26.txt)
    bool narrow = false;
    for (uint32_t c = 0; c < seg->ncols; c++)
        narrow |= seg->cols[c].dtype != MURR_UTF8 && seg->cols[c].dtype != MURR_BOOL && seg->cols[c].size <= 2;
    o << "#define MJ_OUT_NT_LAYOUT " << (narrow ? 1 : 0) << "\n";
    tuning_defs(o);
    return o.str();
}

// The kernel source: embedded, or (tuning) the file MURR_JIT_SRC names.
std::string kernel_source() {
#ifdef MURR_TUNING
    if (const char* f = std::getenv("MURR_JIT_SRC")) {
        std::vector<char> t;
        if (read_file(f, &t)) return std::string(t.begin(), t.end());
    }
#endif
    return kJitSrc;
}

bool compile(Entry& e, const std::string& pre, int device) {
    std::vector<char> code;
    if (!compile_code(pre + kernel_source(), "murr_jit_decode", &code, &e.why)) return false;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    hipError_t he = hipModuleLoadData(&e.mod, code.data());
    for (uint32_t s = 0; s < kJitShapes && he == hipSuccess; s++) {
        JitShapeK& k = e.k.shapes[s];
        k.nw = kJitShapeTab[s][0];
        k.r = kJitShapeTab[s][1];
        k.nslot = kJitShapeTab[s][2];
        k.tr = 64 * (k.nw - 1) * k.r;
        static std::atomic<uint64_t> g_uid{0};
        k.uid = ++g_uid;
        const std::string sh = std::to_string(k.nw) + "x" + std::to_string(k.r) + (k.nslot == 2 ? "" : "s3");
        he = hipModuleGetFunction(&k.fn, e.mod, ("murr_jit_decode_" + sh).c_str());
        if (he == hipSuccess) he = hipModuleGetFunction(&k.fn_split, e.mod, ("murr_jit_decode_split_" + sh).c_str());
    }
    (void)hipSetDevice(cur);
    if (he != hipSuccess) {
        e.why = std::string("module load: ") + hipGetErrorString(he);
        return false;
    }
    return true;
}

}  // namespace

// LDS bytes of a shape (murr_jit_kernel.hip Shape): nslot ring slots [row
// offsets | stage], the span and tile rings, counters, tile prefixes, the
// decode waves' utf8 totals and the loader's 1 KiB prefetch scratch.
uint32_t jit_lds_bytes(uint32_t nw, uint32_t r, uint32_t nslot, uint32_t stage, uint32_t nutf8) {
    const uint32_t tr = 64 * (nw - 1) * r;
    const uint32_t ro = ((tr + 1) * 4 + 16 + 15) & ~15u;  // = Shape::RO_BYTES
    const uint32_t nu = std::max<uint32_t>(nutf8, 1);
    return nslot * (ro + stage + 64) + 128 + 256 + 32 + 8 * nu + ((8 * nu * (nw - 1) + 15) & ~15u) + 1024;
}

const JitLayout* jit_layout(int device, const murr_segment_t* seg, std::string* why, bool pin) {
    const std::string pre = prelude(seg);
#ifdef MURR_TUNING
    const char* srcf = std::getenv("MURR_JIT_SRC");
#else
    const char* srcf = nullptr;
#endif
    const std::string key = std::to_string(device) + "\n" + (srcf ? srcf : "") + "\n" + pre;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(key);
    if (it == g_cache.end()) {
        auto e = std::make_unique<Entry>();
        e->ok = compile(*e, pre, device);
        e->k.ncols = seg->ncols;
        e->device = device;
        it = g_cache.emplace(key, std::move(e)).first;
    }
    Entry* e = it->second.get();
    e->used = ++g_clock;  // before evict: the new entry is the most recent
    evict(e);
    if (!e->ok) {
        if (why) *why = e->why;
        return nullptr;
    }
    if (pin) g_pins[&e->k]++;  // under the lock: no eviction can unload it before the caller launches
    return &e->k;
}

void jit_layout_unpin(const JitLayout* k) {
    if (!k) return;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_pins.find(k);
    if (it != g_pins.end() && --it->second <= 0) g_pins.erase(it);
}

size_t jit_layout_cached() {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_cache.size();
}

size_t jit_layout_limit(size_t n) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (n) kMaxLayouts = n;
    return kMaxLayouts;
}

hipError_t jit_decode_launch(const JitShapeK& k, bool split, const void* args, size_t bytes, uint32_t grid,
                             uint32_t lds, hipStream_t s) {
    size_t sz = bytes;
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, const_cast<void*>(args), HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    return hipModuleLaunchKernel(split ? k.fn_split : k.fn, grid, 1, 1, 64 * k.nw, 1, 1, lds, s, nullptr, cfg);
}

// ---- encode ------------------------------------------------------------------

namespace {

struct EncEntry {
    hipModule_t mod = nullptr;
    JitEncKernel k{};
    bool ok = false;
    std::string why;
};
std::map<std::string, std::unique_ptr<EncEntry>> g_enc;

std::string enc_prelude(uint32_t bs, uint32_t cap, const EncCol* cols, uint32_t ncols, uint32_t stage,
                        uint32_t tile, uint32_t sbw) {
    std::ostringstream o;
    uint32_t nutf8 = 0;
    bool uval = false;  // a utf8 column with a validity buffer: estimated tile sizes, checked
    for (uint32_t c = 0; c < ncols; c++) {
        nutf8 += cols[c].dtype == MURR_UTF8;
        uval = uval || (cols[c].dtype == MURR_UTF8 && cols[c].validity);
    }
    o << "#define MJE_CHECK " << (uval ? 1 : 0) << "\n";
    o << "#define MJE_BS " << bs << "\n#define MJE_CAP " << cap << "\n#define MJE_NCOLS " << ncols
      << "\n#define MJE_NUTF8 " << nutf8 << "\n#define MJE_STAGE " << stage << "\n#define MJE_TILE " << tile
      << "\n#define MJE_SCAN_PER " << kEncScanPer << "\n#define MJE_SBW " << sbw
      << "\n#define MJE_COLS(X)";
    for (uint32_t c = 0, u = 0; c < ncols; c++) {
        const uint32_t kind = cols[c].dtype == MURR_UTF8 ? 0u : cols[c].dtype == MURR_BOOL ? 9u : cols[c].width;
        o << " X(" << c << ", " << kind << ", " << cols[c].soff << ", " << (kind == 0 ? u++ : 0u) << ")";
    }
    o << "\n";
    tuning_defs(o);
    return o.str();
}

}  // namespace

// LDS stage of one 256-row tile: 8, 16 or 32 KiB, the smallest that holds
// the mean blob (blob_cap / n_rows, the bound the caller sized) with a quarter
// of headroom.  Small stages let eight workgroups share a CU; a tile over its
// stage is written straight to HBM (correct, slower).  Three variants per
// layout at most (each one compile, cached).
uint32_t jit_encode_stage(uint64_t n_rows, uint64_t blob_cap, uint32_t tile) {
    const uint64_t mean = n_rows ? (blob_cap + n_rows - 1) / n_rows : 128;
    const uint64_t want = tile * mean * 5 / 4 + 64;
    return want <= 8192 ? 8192u : want <= 16384 ? 16384u : 32768u;
}

// Rows per encode tile (= threads per workgroup): 256 for every layout.
// Measured (profiles/r03/probes/enc_tile_ab.txt): 128-row tiles for wide rows
// (twice the workgroups per CU, half the rows between barriers) took config
// C from 1.07 to 1.59 ms; 512 rows 3.7 ms; B and E within 3 % at 128 / 512.
uint32_t jit_encode_tile(uint64_t n_rows, uint64_t blob_cap) {
    (void)n_rows;
    (void)blob_cap;
#ifdef MURR_TUNING
    if (const char* e = std::getenv("MURR_ENC_TILE")) {  // A/B
        const int t = std::atoi(e);
        if (t == 64 || t == 128 || t == 256 || t == 512) return (uint32_t)t;
    }
#endif
    return 256u;
}

// Off in release builds: staging the strings measured slower than the
// per-lane prefetch (config C columns 1.24 vs 1.04 ms, B 0.248 vs 0.231 ms;
// profiles/r04/probes): the LDS round trips at emit time cost more than the
// scattered loads they replace.  Tuning builds: MURR_ENC_SBW=auto|bytes.
uint32_t jit_encode_sbw(uint64_t n_rows, uint64_t blob_cap, uint32_t fixed, uint32_t nutf8) {
    if (!nutf8) return 0;
#ifdef MURR_TUNING
    const char* e = std::getenv("MURR_ENC_SBW");
    if (!e) return 0;
    if (std::strcmp(e, "auto")) return (uint32_t)std::atoi(e);
#else
    return 0;
#endif
    const double per_row = n_rows ? std::max(0.0, (double)blob_cap / (double)n_rows - fixed - 4.0 * nutf8) : 16.0;
    const double want = 1.25 * 64.0 * per_row + 16.0 * (nutf8 + 1);
    uint32_t b = 512;
    while (b < 4096 && b < want) b *= 2;
    return b;
}

const JitEncKernel* jit_encode_kernel(int device, uint32_t bs, uint32_t cap, const EncCol* cols, uint32_t ncols,
                                      uint32_t stage, uint32_t tile, uint32_t sbw, std::string* why) {
    const std::string pre = enc_prelude(bs, cap, cols, ncols, stage, tile, sbw);
    const std::string key = std::to_string(device) + "\n" + pre;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_enc.find(key);
    if (it == g_enc.end()) {
        auto e = std::make_unique<EncEntry>();
        std::vector<char> code;
        if (compile_code(pre + kJitEncSrc, "murr_jit_encode", &code, &e->why)) {
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(device);
            hipError_t he = hipModuleLoadData(&e->mod, code.data());
            if (he == hipSuccess) he = hipModuleGetFunction(&e->k.fn, e->mod, "murr_jit_encode");
            if (he == hipSuccess) he = hipModuleGetFunction(&e->k.fn_sizes, e->mod, "murr_jit_encode_sizes");
            if (he == hipSuccess) he = hipModuleGetFunction(&e->k.fn_scan, e->mod, "murr_jit_encode_scan");
            int bpc = 0;
            if (he == hipSuccess &&
                (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, e->k.fn, tile, 0) != hipSuccess || bpc < 1))
                bpc = 1;
            e->k.bpc = bpc;
            e->k.tile = tile;
            if (he != hipSuccess) e->why = std::string("module load: ") + hipGetErrorString(he);
            e->ok = he == hipSuccess;
            (void)hipSetDevice(cur);
        }
        it = g_enc.emplace(key, std::move(e)).first;
    }
    if (!it->second->ok) {
        if (why) *why = it->second->why;
        return nullptr;
    }
    return &it->second->k;
}

hipError_t jit_encode_launch(const JitEncKernel* k, const EncodeArgs& a, uint32_t grid, hipStream_t s,
                             uint32_t sizes) {
    EncodeArgs args = a;
    size_t sz = sizeof(args);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    if (a.nutf8) {
        // tile starts: tile sums (a workgroup per tile), then their exclusive
        // scan over kEncScanPer-tile groups (group sums, then prefixes: each group adds up the sums before it)
        const uint32_t tiles = (uint32_t)std::min<uint64_t>(a.total_tiles, 0x7FFFFFFFull);
        const uint32_t groups = (uint32_t)((a.total_tiles + kEncScanPer - 1) / kEncScanPer);
        // (no utf8 column with a validity buffer: the scan derives the tile
        // totals from the offsets itself, murr_jit_encode.hip sizes_inline)
        hipError_t e = sizes != kEncSizesPass
                           ? hipSuccess
                           : hipModuleLaunchKernel(k->fn_sizes, tiles, 1, 1, k->tile, 1, 1, 0, s, nullptr, cfg);
        struct {
            EncodeArgs a;
            uint32_t pass;
        } sa{a, sizes == kEncSizesEstimate ? 3u : 0u};
        size_t ssz = sizeof(sa);
        void* scfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &sa, HIP_LAUNCH_PARAM_BUFFER_SIZE, &ssz, HIP_LAUNCH_PARAM_END};
        if (e == hipSuccess) e = hipModuleLaunchKernel(k->fn_scan, groups, 1, 1, 1024, 1, 1, 0, s, nullptr, scfg);
        bool scan3 = false;  // the group sums scanned by a launch of their own (A/B)
#ifdef MURR_TUNING
        scan3 = std::getenv("MURR_ENC_SCAN3") != nullptr;
#endif
        if (scan3) {
            sa.pass = 2;
            if (e == hipSuccess) e = hipModuleLaunchKernel(k->fn_scan, 1, 1, 1, 1024, 1, 1, 0, s, nullptr, scfg);
        }
        sa.pass = scan3 ? 1u : 4u;
        if (e == hipSuccess) e = hipModuleLaunchKernel(k->fn_scan, groups, 1, 1, 1024, 1, 1, 0, s, nullptr, scfg);
        if (e != hipSuccess) return e;
    }
    // A workgroup per tile (no workgroup waits on another): the hardware
    // refills a CU's slots as tiles finish.  Also for fixed-width layouts,
    // where it beat a persistent grid walking tiles (config E 0.319 vs
    // 0.363 ms, 0.70 vs 0.62 of HBM peak); a persistent grid that prefetches
    // the next tile's loads behind the current stores was slower on B and C.
    grid = (uint32_t)std::min<uint64_t>(a.total_tiles, 0x7FFFFFFFull);
#ifdef MURR_TUNING
    if (const char* g = std::getenv("MURR_ENC_GRID"))  // workgroups per CU of a persistent grid (A/B)
        if (std::atoi(g)) grid = (uint32_t)std::min<uint64_t>(a.total_tiles, (uint64_t)std::atoi(g) * 256);
#endif
    return hipModuleLaunchKernel(k->fn, grid, 1, 1, k->tile, 1, 1, 0, s, nullptr, cfg);
}

}  // namespace murr
