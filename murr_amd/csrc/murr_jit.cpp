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

#include <cstdio>
#include <cstdlib>
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

struct Entry {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    JitKernel k;
    bool ok = false;
    std::string why;
};

std::mutex g_mu;
std::map<std::string, std::unique_ptr<Entry>> g_cache;

std::string prelude(uint32_t bs, const DecProj* dp, uint32_t nproj, uint32_t nutf8, const JitShape& s) {
    std::ostringstream o;
    o << "#define MJ_NW " << s.nw << "\n#define MJ_R " << s.r << "\n#define MJ_SLOTS " << s.slots << "\n#define MJ_STAGE " << s.stage
      << (std::getenv("MURR_JIT_STAMPS") ? "\n#define MJ_STAMPS 1" : "")
      << (std::getenv("MURR_JIT_RO8") ? "\n#define MJ_RO8 1" : "") << "\n#define MJ_BS " << bs << "\n#define MJ_NPROJ " << nproj << "\n#define MJ_NUTF8 " << nutf8
      << "\n#define MJ_FIXED_GROUPS";
    // fixed columns in groups of `group` (loads of a group precede its stores)
    uint32_t group = 4;
    if (const char* e = std::getenv("MURR_JIT_GROUP")) group = std::max(1, std::atoi(e));  // tuning
    for (uint32_t p = 0, inq = 0, ng = 0; p < nproj; p++) {
        if (dp[p].is_utf8) continue;
        if (inq == 0) o << (ng++ ? ">, G<" : " G<");
        else o << ", ";
        o << "FC<" << p << ", " << (dp[p].dtype == MURR_BOOL ? 0u : dp[p].width) << ", " << bs + dp[p].offset << ", "
          << dp[p].bit << ">";
        if (++inq == group) inq = 0;
    }
    {
        bool any = false;
        for (uint32_t p = 0; p < nproj; p++) any |= !dp[p].is_utf8;
        if (any) o << ">";
    }
    o << "\n#define MJ_UTF8_COLS";
    for (uint32_t p = 0, u = 0; p < nproj; p++)
        if (dp[p].is_utf8) o << (u ? ", " : " ") << "UC<" << p << ", " << u++ << ", " << bs + dp[p].offset << ", " << dp[p].bit << ">";
    o << "\n#define MJ_FIXED(X)";
    for (uint32_t p = 0; p < nproj; p++)
        if (!dp[p].is_utf8)
            o << " X(" << p << ", " << (dp[p].dtype == MURR_BOOL ? 0u : dp[p].width) << ", " << bs + dp[p].offset
              << ", " << dp[p].bit << ")";
    o << "\n#define MJ_UTF8(X)";
    for (uint32_t p = 0, u = 0; p < nproj; p++)
        if (dp[p].is_utf8) o << " X(" << p << ", " << u++ << ", " << bs + dp[p].offset << ", " << dp[p].bit << ")";
    o << "\n#define MJ_COL_FO";
    for (uint32_t p = 0; p < nproj; p++) o << (p ? ", " : " ") << bs + dp[p].offset;
    o << "\n#define MJ_COL_BIT";
    for (uint32_t p = 0; p < nproj; p++) o << (p ? ", " : " ") << dp[p].bit;
    o << "\n#define MJ_COL_WID";
    for (uint32_t p = 0; p < nproj; p++) o << (p ? ", " : " ") << (dp[p].is_utf8 ? 0u : dp[p].width);
    o << "\n";
    // tuning: MURR_JIT_DEFS="NAME=VALUE,..." extra #defines (ablation builds)
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
    return o.str();
}

// The kernel source: embedded, or (tuning) the file MURR_JIT_SRC names.
std::string kernel_source() {
    if (const char* f = std::getenv("MURR_JIT_SRC")) {
        if (FILE* fp = std::fopen(f, "rb")) {
            std::string t;
            char buf[65536];
            size_t n;
            while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) t.append(buf, n);
            std::fclose(fp);
            return t;
        }
    }
    return kJitSrc;
}

bool compile(Entry& e, const std::string& pre, int device, const JitShape& s) {
    const std::string src = pre + kernel_source();
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "murr_jit_decode.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        e.why = "hiprtcCreateProgram failed";
        return false;
    }
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    const hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
    if (r != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n + 1, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        e.why = std::string("hiprtc: ") + hiprtcGetErrorString(r) + "\n" + log;
        hiprtcDestroyProgram(&prog);
        return false;
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    std::vector<char> code(n);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    int cur = 0;
    hipGetDevice(&cur);
    hipSetDevice(device);
    hipError_t he = hipModuleLoadData(&e.mod, code.data());
    if (he == hipSuccess) he = hipModuleGetFunction(&e.fn, e.mod, "murr_jit_decode");
    if (he == hipSuccess) he = hipModuleGetFunction(&e.k.fn_len, e.mod, "murr_jit_lengths");
    if (he != hipSuccess) {
        e.why = std::string("module load: ") + hipGetErrorString(he);
        hipSetDevice(cur);
        return false;
    }
    const uint32_t tr = jit_tile_rows(s);
    e.k.lds = jit_lds_bytes(s);
    e.k.tr = tr;
    e.k.threads = 64 * s.nw;
    int bpc = 0;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, e.fn, e.k.threads, e.k.lds) != hipSuccess || bpc < 1)
        bpc = 1;
    e.k.bpc = bpc;
    e.k.fn = e.fn;
    hipSetDevice(cur);
    return true;
}

}  // namespace

// Rows per tile and LDS bytes of a shape (murr_jit_kernel.hip TR, LDS_TOTAL):
// NW-1 consumer waves x R chunks of 64 rows; two slots [row offsets | stage],
// the span ring and the consumers' utf8 wave totals.
uint32_t jit_tile_rows(const JitShape& s) { return 64 * (s.nw - 1) * s.r; }
uint32_t jit_lds_bytes(const JitShape& s) {
    const uint32_t ro8 = std::getenv("MURR_JIT_RO8") ? 2 : 1;  // tuning: unpacked row offsets
    const uint32_t ro = ((jit_tile_rows(s) + 1) * 4 * ro8 + 16 + 15) & ~15u;
    const uint32_t wt = (4 * std::max<uint32_t>(s.nutf8, 1) * (s.nw - 1) + 15) & ~15u;
    return s.slots * (ro + s.stage + 64) + 128 + 16 + wt;
}

const JitKernel* jit_decode_kernel(int device, uint32_t bs, const DecProj* dp, uint32_t nproj, uint32_t nutf8,
                                   const JitShape& shape, std::string* why) {
    const std::string pre = prelude(bs, dp, nproj, nutf8, shape);
    const char* srcf = std::getenv("MURR_JIT_SRC");
    const std::string key = std::to_string(device) + "\n" + (srcf ? srcf : "") + "\n" + pre;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(key);
    if (it == g_cache.end()) {
        auto e = std::make_unique<Entry>();
        e->ok = compile(*e, pre, device, shape);
        it = g_cache.emplace(key, std::move(e)).first;
    }
    if (!it->second->ok) {
        if (why) *why = it->second->why;
        return nullptr;
    }
    return &it->second->k;
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

std::string enc_prelude(uint32_t bs, uint32_t cap, const EncCol* cols, uint32_t ncols, uint32_t stage) {
    std::ostringstream o;
    uint32_t nutf8 = 0;
    for (uint32_t c = 0; c < ncols; c++) nutf8 += cols[c].dtype == MURR_UTF8;
    o << "#define MJE_BS " << bs << "\n#define MJE_CAP " << cap << "\n#define MJE_NCOLS " << ncols
      << "\n#define MJE_NUTF8 " << nutf8 << "\n#define MJE_STAGE " << stage << "\n#define MJE_COLS(X)";
    for (uint32_t c = 0, u = 0; c < ncols; c++) {
        const uint32_t kind = cols[c].dtype == MURR_UTF8 ? 0u : cols[c].dtype == MURR_BOOL ? 9u : cols[c].width;
        o << " X(" << c << ", " << kind << ", " << cols[c].soff << ", " << (kind == 0 ? u++ : 0u) << ")";
    }
    o << "\n";
    return o.str();
}

}  // namespace

const JitEncKernel* jit_encode_kernel(int device, uint32_t bs, uint32_t cap, const EncCol* cols, uint32_t ncols,
                                      std::string* why) {
    const uint32_t stage = 32768;
    const std::string pre = enc_prelude(bs, cap, cols, ncols, stage);
    const std::string key = std::to_string(device) + "\n" + pre;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_enc.find(key);
    if (it == g_enc.end()) {
        auto e = std::make_unique<EncEntry>();
        const std::string src = pre + kJitEncSrc;
        hiprtcProgram prog;
        const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
        if (hiprtcCreateProgram(&prog, src.c_str(), "murr_jit_encode.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
            e->why = "hiprtcCreateProgram failed";
        } else {
            const hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
            if (r != HIPRTC_SUCCESS) {
                size_t n = 0;
                hiprtcGetProgramLogSize(prog, &n);
                std::string log(n + 1, '\0');
                if (n) hiprtcGetProgramLog(prog, &log[0]);
                e->why = std::string("hiprtc: ") + hiprtcGetErrorString(r) + "\n" + log;
            } else {
                size_t n = 0;
                hiprtcGetCodeSize(prog, &n);
                std::vector<char> code(n);
                hiprtcGetCode(prog, code.data());
                int cur = 0;
                (void)hipGetDevice(&cur);
                (void)hipSetDevice(device);
                hipError_t he = hipModuleLoadData(&e->mod, code.data());
                if (he == hipSuccess) he = hipModuleGetFunction(&e->k.fn, e->mod, "murr_jit_encode");
                if (he == hipSuccess) he = hipModuleGetFunction(&e->k.fn_sizes, e->mod, "murr_jit_encode_sizes");
                if (he == hipSuccess) he = hipModuleGetFunction(&e->k.fn_scan, e->mod, "murr_jit_encode_scan");
                int bpc = 0;
                if (he == hipSuccess &&
                    (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, e->k.fn, 256, 0) != hipSuccess || bpc < 1))
                    bpc = 1;
                e->k.bpc = bpc;
                if (he != hipSuccess) e->why = std::string("module load: ") + hipGetErrorString(he);
                e->ok = he == hipSuccess;
                (void)hipSetDevice(cur);
            }
            hiprtcDestroyProgram(&prog);
        }
        it = g_enc.emplace(key, std::move(e)).first;
    }
    if (!it->second->ok) {
        if (why) *why = it->second->why;
        return nullptr;
    }
    return &it->second->k;
}

hipError_t jit_encode_launch(const JitEncKernel* k, const EncodeArgs& a, uint32_t grid, hipStream_t s) {
    EncodeArgs args = a;
    size_t sz = sizeof(args);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    if (a.nutf8) {
        // tile starts: tile sums (a workgroup per tile), then their exclusive
        // scan over 4096-tile groups (sums, one-workgroup scan of the sums, prefixes)
        const uint32_t tiles = (uint32_t)std::min<uint64_t>(a.total_tiles, 0x7FFFFFFFull);
        const uint32_t groups = (uint32_t)((a.total_tiles + 4095) / 4096);
        hipError_t e = hipModuleLaunchKernel(k->fn_sizes, tiles, 1, 1, 256, 1, 1, 0, s, nullptr, cfg);
        struct {
            EncodeArgs a;
            uint32_t pass;
        } sa{a, 0};
        size_t ssz = sizeof(sa);
        void* scfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &sa, HIP_LAUNCH_PARAM_BUFFER_SIZE, &ssz, HIP_LAUNCH_PARAM_END};
        if (e == hipSuccess) e = hipModuleLaunchKernel(k->fn_scan, groups, 1, 1, 1024, 1, 1, 0, s, nullptr, scfg);
        sa.pass = 2;
        if (e == hipSuccess) e = hipModuleLaunchKernel(k->fn_scan, 1, 1, 1, 1024, 1, 1, 0, s, nullptr, scfg);
        sa.pass = 1;
        if (e == hipSuccess) e = hipModuleLaunchKernel(k->fn_scan, groups, 1, 1, 1024, 1, 1, 0, s, nullptr, scfg);
        if (e != hipSuccess) return e;
        grid = tiles;  // no co-resident grid needed: a workgroup per tile
    }
    return hipModuleLaunchKernel(k->fn, grid, 1, 1, 256, 1, 1, 0, s, nullptr, cfg);
}

hipError_t jit_decode_launch(const JitKernel* k, const JitArgs& a, uint32_t grid, hipStream_t s, bool lengths) {
    JitArgs args = a;
    size_t sz = sizeof(args);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    return hipModuleLaunchKernel(lengths ? k->fn_len : k->fn, grid, 1, 1, k->threads, 1, 1, k->lds, s, nullptr, cfg);
}

}  // namespace murr
