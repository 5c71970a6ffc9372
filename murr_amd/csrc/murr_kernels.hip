// murr_kernels.hip — gfx950 kernels for murr's row-blob codec.
//
// decode: row blobs -> Arrow buffers (replaces ReadBatchBuilder::add_row /
//         add_empty / build and the per-dtype ColumnEncoders:
//         src/io/row/read.rs:62-110, src/io/codec/primitive.rs:38-61,
//         bool_.rs:85-104, utf8.rs:85-105)
// encode: Arrow buffers -> row blobs (replaces Table::write's row loop with
//         WriteRow + ColumnDecoders: src/io/table/mod.rs:97-109,
//         src/io/row/write.rs:19-52, primitive.rs:85-95, bool_.rs:111-117,
//         utf8.rs:113-119)
//
// Both are byte movement: HBM-bound, no MFMA.  One workgroup = 4 waves = one
// 256-row tile, thread-per-row.  A tile's blob bytes are contiguous in HBM, so
// they are staged into LDS with 16-B coalesced loads (decode) or assembled in
// LDS and written out with 16-B coalesced stores (encode); each lane then
// extracts its row's fields from LDS with aligned dword reads + v_alignbyte.
// Validity and bool bitmaps come straight out of __ballot: one 64-bit word per
// wave.  UTF-8 offsets (decode) and row offsets (encode) need a prefix sum
// across tiles: a wave-level shuffle scan, an LDS combine across the 4 waves,
// and a one-hop window sum across tiles (see window_prefix).  Tiles are
// assigned round-robin to a persistent grid that fits on the chip at once, so
// every tile a prefix waits on is resident or finished.
#include "murr_internal.h"

namespace murr {

namespace {

#define GAS __attribute__((address_space(1)))
#define LAS __attribute__((address_space(3)))
#define CAS __attribute__((address_space(4)))
// Global-address-space views of generic pointers: global_* instead of flat_*
// instructions (flat ones also tie up lgkmcnt and cost issue slots).
template <class T> __device__ __forceinline__ GAS T* gp(T* p) { return (GAS T*)p; }
template <class T> __device__ __forceinline__ const GAS T* gp(const T* p) { return (const GAS T*)p; }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kUtf8 = 0, kBool = 1;
constexpr uint32_t kSpinLimit = 1u << 22;
// Ablation switches and phase stamps (MURR_DEBUG_DECODE) exist only in a
// `make DEBUG=1` build; the production kernel carries none of their branches.
#ifndef MURR_DECODE_DEBUG
#define MURR_DECODE_DEBUG 0
#endif
constexpr bool kDbg = MURR_DECODE_DEBUG != 0;
enum : uint32_t { kStUtf8 = 1, kStOverflow = 4, kStMalformed = 5, kStCapacity = 6, kStInternal = 10 };

__device__ __forceinline__ void report(unsigned long long* err, uint64_t key) {
    __hip_atomic_fetch_max(gp(err), (unsigned long long)~key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- wave / block scan helpers (wave64) --------------------------------------
__device__ __forceinline__ uint64_t shfl_up64(uint64_t x, int d) {
    uint32_t lo = __shfl_up((uint32_t)x, d, 64), hi = __shfl_up((uint32_t)(x >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int m) {
    uint32_t lo = __shfl_xor((uint32_t)x, m, 64), hi = __shfl_xor((uint32_t)(x >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = shfl_up64(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) x += shfl_xor64(x, m);
    return x;
}

// Wave64 inclusive scan of u32 on DPP (VALU only; __shfl_* lowers to
// ds_bpermute, an LDS round trip per step): Hillis-Steele within each 16-lane
// row (row_shr 1/2/4/8), then row_bcast:15 into rows 1 and 3 and row_bcast:31
// into rows 2 and 3 (GFX9 DPP controls, kept on gfx950).
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}
__device__ __forceinline__ uint32_t wave_total_u32(uint32_t v) {
    return __builtin_amdgcn_readlane(wave_scan_u32(v), 63);
}

// Block-wide (256 threads) inclusive scan; returns inclusive value, sets *agg.
__device__ __forceinline__ uint64_t block_incl_scan(uint64_t x, uint64_t* s_w, uint64_t* agg) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = wave_incl_scan(x, lane);
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) {
        uint64_t v = s_w[w];
        pre += (w < wave) ? v : 0;
        tot += v;
    }
    __syncthreads();  // s_w reusable afterwards
    *agg = tot;
    return pre + inc;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops,
// not for its vector-memory ops, so LDS-DMA in flight survives it
// (__syncthreads() emits s_waitcnt vmcnt(0) and would drain it).
// threadIdx.x made opaque at each use: stops the compiler from hoisting the
// many lane masks derived from it out of the tile loop into SGPR pairs, which
// overflowed the SGPR file and spilled (recomputing a mask is one VALU op).
__device__ __forceinline__ uint32_t tidx() {
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Cross-tile prefix by a one-hop window sum.  Tiles are dealt round-robin to
// a persistent grid of G workgroups, so tile t's workgroup processed tile t-G
// itself and kept its inclusive prefix (`base`).  What lies between is the
// aggregate of tiles (t-G, t): each tile publishes its aggregate (+1, so 0 =
// not yet) in one 8-byte agent-scope store right after its length scan, and
// the whole workgroup sums the <= G-1 granules in parallel (agent-scope relaxed
// loads = sc1: bypass this CU's L1; MI355X_MICROARCH.md R2 hand-off form).
// Only tiles that are resident or done are ever waited on; spins are bounded.
template <int NW>  // waves in the workgroup
__device__ __forceinline__ uint64_t window_prefix(const uint64_t* st, uint64_t lo, uint64_t t, uint64_t base,
                                  LAS uint64_t* s_w, unsigned long long* err, uint64_t ekey) {
    constexpr int K = 4;  // granules per thread per pass
    constexpr uint32_t NT = 64 * NW;
    const uint32_t tid = tidx(), lane = tid & 63, wave = tid >> 6;
    uint64_t sum = 0;
    for (uint64_t j0 = lo; j0 < t; j0 += NT * K) {
        uint64_t v[K];
#pragma unroll
        for (int i = 0; i < K; i++) {  // every load in flight before the first check
            const uint64_t j = j0 + i * NT + tid;
            v[i] = j < t ? __hip_atomic_load(gp(st) + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1;
        }
#pragma unroll
        for (int i = 0; i < K; i++) {
            const uint64_t j = j0 + i * NT + tid;
            uint32_t spins = 0;
            while (v[i] == 0) {
                __builtin_amdgcn_s_sleep(2);
                v[i] = __hip_atomic_load(gp(st) + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (++spins > kSpinLimit) {
                    report(err, ekey | kStInternal);
                    v[i] = 1;
                    break;
                }
            }
            sum += v[i] - 1;
        }
    }
    sum = wave_sum(sum);
    if (lane == 0) s_w[wave] = sum;
    lds_barrier();
    uint64_t tot = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) tot += s_w[w];
    lds_barrier();
    return base + tot;
}

__device__ __forceinline__ void publish(uint64_t* p, uint64_t v) {
    __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// UTF-8 well-formedness (Unicode Table 3-7 = Rust core::str::from_utf8).
struct Utf8Dfa {
    uint32_t need = 0, lo = 0x80, hi = 0xBF;
    bool bad = false;
    __device__ __forceinline__ void step(uint32_t c) {
        if (need == 0) {
            if (c < 0x80) return;
            if (c >= 0xC2 && c <= 0xDF) { need = 1; lo = 0x80; hi = 0xBF; }
            else if (c == 0xE0) { need = 2; lo = 0xA0; hi = 0xBF; }
            else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) { need = 2; lo = 0x80; hi = 0xBF; }
            else if (c == 0xED) { need = 2; lo = 0x80; hi = 0x9F; }
            else if (c == 0xF0) { need = 3; lo = 0x90; hi = 0xBF; }
            else if (c >= 0xF1 && c <= 0xF3) { need = 3; lo = 0x80; hi = 0xBF; }
            else if (c == 0xF4) { need = 3; lo = 0x80; hi = 0x8F; }
            else bad = true;
        } else {
            if (c < lo || c > hi) bad = true;
            lo = 0x80; hi = 0xBF; need--;
        }
    }
    __device__ __forceinline__ bool ok() const { return !bad && need == 0; }
};

// Copy buf[0..span) (LDS) to out[g0..g0+span) with aligned 16-B stores; the
// unaligned head and tail bytes with byte stores.  `tid` / `nt`: the calling
// lanes (a wave or the workgroup).
__device__ __forceinline__ void write_out(const LAS uint8_t* buf, GAS uint8_t* out, uint64_t g0,
                                          uint64_t span, uint32_t tid, uint32_t nt) {
    const uint64_t g1 = g0 + span;
    const uint64_t a0 = (g0 + 15) & ~15ull, a1 = g1 & ~15ull;
    if (a0 >= a1) {
        for (uint64_t k = tid; k < span; k += nt) out[g0 + k] = buf[k];
        return;
    }
    if (tid < a0 - g0) out[g0 + tid] = buf[tid];
    if (tid < g1 - a1) out[a1 + tid] = buf[a1 - g0 + tid];
    const uint32_t lb0 = (uint32_t)(a0 - g0);
    const uint32_t sh = lb0 & 3u;
    const LAS uint32_t* w = (const LAS uint32_t*)buf;
    const uint64_t nch = (a1 - a0) >> 4;
    GAS u32x4* o = reinterpret_cast<GAS u32x4*>(out + a0);
    for (uint64_t c = tid; c < nch; c += nt) {
        const uint32_t q = (lb0 >> 2) + 4 * (uint32_t)c;
        const uint32_t d0 = w[q], d1 = w[q + 1], d2 = w[q + 2], d3 = w[q + 3], d4 = w[q + 4];
        u32x4 v;
        v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
        v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
        v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
        v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
        o[c] = v;
    }
}

// ---- decode -------------------------------------------------------------------
// Persistent workgroups of 4 waves walk their tiles (t, t+G, t+2G, ...) with a
// two-deep LDS pipeline: right after the barrier that makes tile i resident,
// every wave issues its share of tile i+1's LDS-DMA (row-offset slice + blob
// bytes, global_load_lds_dwordx4, 1 KiB per wave-instruction), so HBM stays
// busy while tile i is decoded from LDS:
//   A: utf8 cells parsed (cached in LDS), 64-row chunk totals -> chunk
//      prefixes, tile aggregate published for the cross-tile prefix
//   F: validity of every column (__ballot words), fixed-width and bool values
//   B: per utf8 column: cross-tile prefix (window_prefix), i32 offsets, string
//      bytes assembled per wave in LDS and stored 16 B wide, UTF-8 checked.
// Everything wave-uniform (descriptors, chunk prefixes, output bases) lives in
// SGPRs: descriptor tables are read through the constant address space
// (s_load, lgkmcnt: no vmcnt wait that would drain the LDS-DMA in flight), and
// per-row arithmetic is 32-bit, relative to the tile.
__device__ __forceinline__ DecBlock ldblk(const DecodeArgs& A, uint64_t i) {
    const CAS DecBlock* p = (const CAS DecBlock*)A.blocks + i;
    DecBlock r;
    r.data = p->data; r.row_off = p->row_off; r.n_rows = p->n_rows; r.tile_base = p->tile_base;
    return r;
}
__device__ __forceinline__ DecProj ldproj(const DecodeArgs& A, uint64_t i) {
    const CAS DecProj* p = (const CAS DecProj*)A.proj + i;
    DecProj r;
    r.dtype = p->dtype; r.bit = p->bit; r.offset = p->offset; r.width = p->width;
    r.is_utf8 = p->is_utf8; r.uslot = p->uslot;
    return r;
}
__device__ __forceinline__ DecOut ldout(const DecodeArgs& A, uint64_t i) {
    const CAS DecOut* p = (const CAS DecOut*)A.outs + i;
    DecOut r;
    r.values = p->values; r.validity = p->validity; r.offsets = p->offsets; r.values_cap = p->values_cap;
    return r;
}
__device__ __forceinline__ uint32_t sgpr(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t sgpr64(uint64_t v) {
    return ((uint64_t)sgpr((uint32_t)(v >> 32)) << 32) | sgpr((uint32_t)v);
}

struct DecTile {
    uint64_t t, tfirst, r0;
    uint64_t base, end, abase;  // blob span of the tile, 16-B aligned start
    uint32_t b, nr, last, ok;
};

struct DecLayout {     // byte offsets inside one LDS tile buffer
    uint32_t pre, rowoff, stage, bytes;
};

__host__ __device__ inline DecLayout dec_layout(uint32_t R, uint32_t nutf8, uint32_t stage) {
    DecLayout L;
    L.pre = 0;  // [nutf8][R/64 + 1] u32 chunk prefixes (+ tile aggregate)
    L.rowoff = ((4 * nutf8 * (R / 64 + 1) + 15) & ~15u);
    L.stage = L.rowoff + ((8 * (R + 1) + 16 + 15) & ~15u);
    L.bytes = L.stage + stage + 32;
    return L;
}

// What the pipeline carries per tile (few SGPRs): the tile, its block and its
// blob span.  Everything else is re-derived from the block descriptor.
struct TileRef {
    uint64_t t, base, end;
    uint32_t b, ok;
};

__device__ __forceinline__ TileRef make_ref(const DecodeArgs& A, uint64_t t, uint32_t b) {
    const DecBlock blk = ldblk(A, b);
    const uint64_t r0 = (t - blk.tile_base) * A.rows_per_tile;
    const uint64_t nr = min((uint64_t)A.rows_per_tile, blk.n_rows - r0);
    // Vector loads (HBM latency): a tile's span is fetched one pipeline step
    // before its DMA is issued, and the loop-top vmcnt(0) that waits for the
    // DMA covers them, so they never stall.  (As scalar loads they shared
    // lgkmcnt with LDS traffic, and the first LDS wait exposed their latency.)
    const GAS uint64_t* ro = gp(blk.row_off) + r0;
    TileRef r;
    r.t = t;
    r.b = b;
    r.base = __builtin_nontemporal_load(ro);
    r.end = __builtin_nontemporal_load(ro + nr);
    r.ok = 1;
    return r;
}

__device__ __forceinline__ uint64_t tiles_end(const DecodeArgs& A, uint32_t b) {
    return b + 1 < A.nblocks ? ldblk(A, b + 1).tile_base : A.total_tiles;
}

// First tile of this workgroup.  Block-local mode: workgroup w owns blocks
// w, w+G, ... whole, in tile order.  Window mode: tiles w, w+G, w+2G, ...
__device__ __forceinline__ TileRef first_ref(const DecodeArgs& A) {
    TileRef r;
    r.ok = 0;
    r.t = r.base = r.end = 0;
    r.b = 0;
    const uint32_t w = blockIdx.x, G = gridDim.x;
    if (A.local) {
        for (uint32_t b = w; b < A.nblocks; b += G)
            if (tiles_end(A, b) > ldblk(A, b).tile_base) return make_ref(A, ldblk(A, b).tile_base, b);
        return r;
    }
    if (w >= A.total_tiles) return r;
    uint32_t b = 0;
    while (b + 1 < A.nblocks && ldblk(A, b + 1).tile_base <= w) b++;
    return make_ref(A, w, b);
}

__device__ __forceinline__ TileRef next_ref(const DecodeArgs& A, const TileRef& c) {
    TileRef r;
    r.ok = 0;
    r.t = r.base = r.end = 0;
    r.b = 0;
    if (!c.ok) return r;
    const uint32_t G = gridDim.x;
    if (A.local) {
        if (c.t + 1 < tiles_end(A, c.b)) return make_ref(A, c.t + 1, c.b);
        for (uint32_t b = c.b + G; b < A.nblocks; b += G)
            if (tiles_end(A, b) > ldblk(A, b).tile_base) return make_ref(A, ldblk(A, b).tile_base, b);
        return r;
    }
    const uint64_t t = c.t + G;
    if (t >= A.total_tiles) return r;
    uint32_t b = c.b;
    while (b + 1 < A.nblocks && ldblk(A, b + 1).tile_base <= t) b++;
    return make_ref(A, t, b);
}

__device__ __forceinline__ DecTile tile_of(const DecodeArgs& A, const TileRef& r) {
    const DecBlock blk = ldblk(A, r.b);
    DecTile T;
    T.t = r.t;
    T.b = r.b;
    T.tfirst = blk.tile_base;
    T.r0 = (r.t - blk.tile_base) * A.rows_per_tile;
    T.nr = (uint32_t)min((uint64_t)A.rows_per_tile, blk.n_rows - T.r0);
    T.last = T.r0 + T.nr == blk.n_rows;
    T.base = sgpr64(r.base);  // loaded by every lane (vector load), uniform
    T.end = sgpr64(r.end);
    T.abase = T.base & ~15ull;
    T.ok = r.ok;
    return T;
}

// Issue tile T's LDS-DMA: row-offset slice [r0, r0+nr] and, when it fits the
// stage, the blob span rounded out to 16-B granules (never past the granule
// holding the last byte, so never past the allocation).  No waits here.
__device__ __forceinline__ void issue_stage(const DecodeArgs& A, const DecTile& T, LAS uint8_t* buf,
                                            const DecLayout& L) {
    const uint32_t lane = tidx() & 63, wave = tidx() >> 6;
    const GAS uint64_t* ro = gp(ldblk(A, T.b).row_off) + T.r0;
    const uintptr_t s0 = (uintptr_t)ro & ~(uintptr_t)15;
    const uint32_t nb_off = (uint32_t)((((uintptr_t)ro - s0) + (uint64_t)(T.nr + 1) * 8 + 15) & ~15ull);
    const GAS uint8_t* go = (const GAS uint8_t*)s0;
    for (uint32_t c = wave; c * 1024 < nb_off; c += kDW) {
        const uint32_t off = c * 1024 + lane * 16;
        if (off < nb_off)
            __builtin_amdgcn_global_load_lds((const GAS void*)(go + off), (LAS void*)(buf + L.rowoff + c * 1024),
                                             16, 0, 0);
    }
    const uint64_t span = ((T.end + 15) & ~15ull) - T.abase;
    if (span <= A.stage) {
        const GAS uint8_t* g = gp(ldblk(A, T.b).data) + T.abase;
        const uint32_t nb = (uint32_t)span;
        for (uint32_t c = wave; c * 1024 < nb; c += kDW) {
            const uint32_t off = c * 1024 + lane * 16;
            if (off < nb)
                __builtin_amdgcn_global_load_lds((const GAS void*)(g + off), (LAS void*)(buf + L.stage + c * 1024),
                                                 16, 0, 0);
        }
    }
}

// Tile bytes: staged in LDS (the hot path) or, for the rare tile whose rows
// outgrew the stage, read from HBM by an out-of-line copy of the decoder.
struct StageSrc {
    static constexpr bool kHbm = false;
    const LAS uint8_t* s;  // 16-B aligned, >= 16 B of padding past the data
    __device__ __forceinline__ uint32_t u32(uint32_t a) const {
        const LAS uint32_t* w = (const LAS uint32_t*)(s + (a & ~3u));
        return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
    }
    __device__ __forceinline__ uint64_t u64(uint32_t a) const {
        const LAS uint32_t* w = (const LAS uint32_t*)(s + (a & ~3u));
        const uint32_t sh = a & 3u, w0 = w[0], w1 = w[1], w2 = w[2];
        return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) |
               ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    }
    __device__ __forceinline__ uint32_t u8(uint32_t a) const { return s[a]; }
    // first n <= 4 bytes at a (padding makes the over-read safe)
    __device__ __forceinline__ uint32_t head(uint32_t a, uint32_t n) const {
        const uint32_t v = u32(a);
        return n >= 4 ? v : v & ((1u << (8 * n)) - 1);
    }
};
struct HbmSrc {
    static constexpr bool kHbm = true;
    const GAS uint8_t* g;  // 16-B aligned; never reads a dword holding no requested byte
    __device__ __forceinline__ uint32_t u32(uint32_t a) const {
        const GAS uint32_t* w = (const GAS uint32_t*)(g + (a & ~3u));
        const uint32_t sh = a & 3u;
        return sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
    }
    __device__ __forceinline__ uint64_t u64(uint32_t a) const {
        return (uint64_t)u32(a) | ((uint64_t)u32(a + 4) << 32);
    }
    __device__ __forceinline__ uint32_t u8(uint32_t a) const { return g[a]; }
    __device__ __forceinline__ uint32_t head(uint32_t a, uint32_t n) const {
        uint32_t v = 0;
        for (uint32_t q = 0; q < n && q < 4; q++) v |= (uint32_t)g[a + q] << (8 * q);
        return v;
    }
};

template <class Src>
__device__ __forceinline__ bool utf8_valid_slow(Src src, uint32_t at, uint32_t n) {
    Utf8Dfa dfa;
    for (uint32_t q = 0; q < n; q++) dfa.step(src.u8(at + q));
    return dfa.ok();
}

// read_dynamic (read.rs:45-55) for one non-null cell: string length and
// payload address; *bad = a slice the reference would panic on.
template <class Src>
__device__ __forceinline__ uint32_t utf8_cell(const Src& src, uint32_t ra, uint32_t rl, uint32_t bs,
                                              uint32_t fo, bool want, uint32_t* pay, bool* bad) {
    *pay = 0;
    *bad = false;
    if (!want) return 0;
    if (fo + 4 > rl) { *bad = true; return 0; }
    const uint32_t vlen = rl - bs;
    const uint32_t prel = src.u32(ra + fo);
    if ((uint64_t)prel + 4 > vlen) { *bad = true; return 0; }
    const uint32_t l = src.u32(ra + bs + prel);
    if ((uint64_t)prel + 4 + l > vlen) { *bad = true; return 0; }
    *pay = ra + bs + prel + 4;
    return l;
}


struct DecLds {  // this workgroup's LDS regions besides the tile buffers
    LAS uint32_t* nulls;  // [4][nproj] per-wave null counts of the current tile
    LAS uint64_t* w;      // [4] scratch for window_prefix
    LAS uint64_t* mine;   // [4][nutf8] per wave: the last inclusive prefix
    LAS uint64_t* st;     // [8] diagnostic stamps
    LAS uint64_t* cell;   // [cell_cols][R] (slen << 32 | payload address)
};

__device__ __forceinline__ void dstamp(const DecodeArgs& A, const DecLds& S, int j) {
    if (kDbg && (A.debug & 8) && tidx() == 0) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        S.st[j] += t - S.st[7];
        S.st[7] = t;
    }
}

// One projected column of one tile, rows dealt as in the tile comment: this
// wave's 64-row chunks k*4 + wave.  KIND: 0 utf8, 1 bool, 3 one-byte values,
// else the value width in bytes.  Straight-line per row: row offsets from the staged slice,
// null bit, value (or utf8 slot + length), ballot -> validity word.  Reads for
// the LDS stage are unguarded (stale or out-of-range LDS reads are harmless
// and masked); HBM reads are clamped to the tile start when not wanted.
// Returns this wave's null count; sets bits k of *badk for malformed rows.
template <int KIND, int KMAX, class Src>
__device__ __forceinline__ uint32_t dec_column(const DecodeArgs& A, const Src& src, const DecTile& T,
                                               const LAS uint32_t* ro, uint32_t nk, const DecProj& pc,
                                               const DecOut& o, LAS uint64_t* cell, LAS uint32_t* pre_u,
                                               uint32_t* badk) {
    const uint32_t tid = tidx(), lane = tid & 63, wave = tid >> 6;
    const uint32_t bs = A.bs, abase = (uint32_t)T.abase;
    const uint32_t fo = bs + pc.offset, nbyte = pc.bit >> 3, nbit = pc.bit & 7;
    GAS uint64_t* vwords = gp((uint64_t*)o.validity) + (T.r0 >> 6) + wave;
    // The KMAX chunks advance level by level (row offsets -> null byte and
    // value / slot -> string length), so each level's LDS reads are all in
    // flight before the first wait: KMAX independent chains, not one long one.
    // Every read is unconditional and its use a select (a read inside a branch
    // costs an exec-mask save/restore and a wait of its own; stage reads at
    // stale or out-of-range LDS addresses are harmless; HBM reads are pointed
    // at the tile start when not wanted).  Chunks past the tile have no
    // active lane.
    uint32_t ra[KMAX], rl[KMAX];
    bool act[KMAX], present[KMAX];
#pragma unroll
    for (uint32_t k = 0; k < KMAX; k++) {
        const uint32_t i = k * kDT + tid;
        act[k] = i < T.nr;
        const uint32_t a0 = ro[2 * i], a1 = ro[2 * i + 2];
        ra[k] = a0 - abase;
        rl[k] = act[k] ? a1 - a0 : 0;
        present[k] = rl[k] >= bs && rl[k] != 0;
    }
    uint32_t nb[KMAX], v0[KMAX];
    uint64_t v8[KMAX];
#pragma unroll
    for (uint32_t k = 0; k < KMAX; k++) {
        nb[k] = src.u8(Src::kHbm && !present[k] ? 0 : ra[k] + nbyte);
        constexpr uint32_t W = KIND == 0 ? 4 : KIND == 1 || KIND == 3 ? 1 : KIND;
        const uint32_t a = Src::kHbm && !(present[k] && fo + W <= rl[k]) ? 0 : ra[k] + fo;
        if constexpr (KIND == 8) v8[k] = src.u64(a);
        else if constexpr (KIND == 4 || KIND == 0) v0[k] = src.u32(a);  // utf8: the slot
        else if constexpr (KIND == 2) v0[k] = src.head(a, 2);
        else v0[k] = src.u8(a);
    }
    uint32_t len[KMAX];
    if constexpr (KIND == 0) {
#pragma unroll
        for (uint32_t k = 0; k < KMAX; k++) {
            // read_dynamic (read.rs:45-55): slot -> payload offset p (relative to
            // the static region), u32 length at p, bytes at p + 4
            const bool p_ok = present[k] && fo + 4 <= rl[k] && v0[k] <= rl[k] - bs - 4;
            len[k] = src.u32(Src::kHbm && !p_ok ? 0 : ra[k] + bs + v0[k]);
        }
    }
    uint32_t nulls = 0;
#pragma unroll
    for (uint32_t k = 0; k < KMAX; k++) {
        const uint32_t i = k * kDT + tid;
        const bool isnull = !present[k] || ((nb[k] >> nbit) & 1);
        const uint64_t vm = __ballot(act[k] && !isnull);
        nulls += __popcll(__ballot(act[k] && isnull));
        const bool live = k * kDT + wave * 64 < T.nr;  // wave-uniform
        if (live && lane == 0) vwords[kDW * k] = vm;
        bool bad = rl[k] && !present[k];  // split_at panics on a row shorter than the bitset
        if constexpr (KIND == 0) {
            const uint32_t vlen = rl[k] - bs, prel = v0[k];
            const bool p_ok = !isnull && fo + 4 <= rl[k] && prel <= vlen - 4;
            const bool good = p_ok && len[k] <= vlen - 4 - prel;
            bad |= !isnull && !good;
            const uint32_t slen = good ? len[k] : 0;
            if (cell) cell[i] = ((uint64_t)slen << 32) | (ra[k] + bs + prel + 4);
            const uint32_t tot = wave_total_u32(slen);  // < tile span < 4 GiB
            if (live && lane == 0) pre_u[k * kDW + wave] = tot;
        } else if constexpr (KIND == 1) {
            const bool have = !isnull && fo + 1 <= rl[k];
            bad |= !isnull && !have;
            const uint64_t m = __ballot(act[k] && have && v0[k] != 0);
            if (live && lane == 0) gp((uint64_t*)o.values)[(T.r0 >> 6) + kDW * k + wave] = m;
        } else {
            constexpr uint32_t W = KIND == 3 ? 1 : KIND;  // KIND 3 = 1-byte values
            const bool have = !isnull && fo + W <= rl[k];
            bad |= !isnull && !have;
            if constexpr (KIND == 8) {
                if (act[k]) ((GAS uint64_t*)gp(o.values) + T.r0)[i] = have ? v8[k] : 0;
            } else if constexpr (KIND == 4) {
                if (act[k]) ((GAS uint32_t*)gp(o.values) + T.r0)[i] = have ? v0[k] : 0;
            } else if constexpr (KIND == 2) {
                if (act[k]) ((GAS uint16_t*)gp(o.values) + T.r0)[i] = have ? (uint16_t)v0[k] : 0;
            } else {
                if (act[k]) (gp((uint8_t*)o.values) + T.r0)[i] = have ? (uint8_t)v0[k] : 0;
            }
        }
        *badk |= (uint32_t)bad << k;
    }
    return nulls;
}

template <int KMAX, class Src>
__device__ __forceinline__ void decode_tile(const DecodeArgs& A, const Src& src, const DecTile& T,
                                            LAS uint8_t* buf, const DecLayout& L, const DecLds& S) {
    const uint32_t tid = tidx(), lane = tid & 63, wave = tid >> 6;
    const uint32_t bs = A.bs, R = A.rows_per_tile, nproj = A.nproj;
    // staged row offsets; their low dwords suffice (a tile spans < 4 GiB)
    const LAS uint32_t* ro = (const LAS uint32_t*)(buf + L.rowoff +
                                                   (((uintptr_t)(ldblk(A, T.b).row_off + T.r0)) & 15));
    const uint32_t abase = (uint32_t)T.abase;
    LAS uint32_t* pre = (LAS uint32_t*)(buf + L.pre);
    const uint32_t PS = R / 64 + 1;  // pre stride per utf8 column
    const uint32_t nchunk = (T.nr + 63) / 64;
    const uint32_t nk = (T.nr + kDT - 1) / kDT;
    LAS uint32_t* wnull = S.nulls + wave * nproj;  // this wave's null counters

    // ---- pass 1: column by column (descriptor loads and the dtype dispatch
    // once per column, straight-line row loops inside).
    uint32_t badk = 0;
#pragma unroll 1
    for (uint32_t p = 0; p < nproj; p++) {
        const DecProj pc = ldproj(A, p);
        const DecOut o = ldout(A, (uint64_t)T.b * nproj + p);
        uint32_t nn;
        if (pc.is_utf8) {
            LAS uint64_t* cell = pc.uslot < A.cell_cols ? S.cell + pc.uslot * R : nullptr;
            nn = dec_column<0, KMAX>(A, src, T, ro, nk, pc, o, cell, pre + pc.uslot * PS, &badk);
        } else if (pc.dtype == kBool) {
            nn = dec_column<1, KMAX>(A, src, T, ro, nk, pc, o, nullptr, nullptr, &badk);
        } else if (pc.width == 4) {
            nn = dec_column<4, KMAX>(A, src, T, ro, nk, pc, o, nullptr, nullptr, &badk);
        } else if (pc.width == 8) {
            nn = dec_column<8, KMAX>(A, src, T, ro, nk, pc, o, nullptr, nullptr, &badk);
        } else if (pc.width == 2) {
            nn = dec_column<2, KMAX>(A, src, T, ro, nk, pc, o, nullptr, nullptr, &badk);
        } else {
            nn = dec_column<3, KMAX>(A, src, T, ro, nk, pc, o, nullptr, nullptr, &badk);  // 1-byte values
        }
        if (lane == 0 && nn) wnull[p] += nn;
    }
    // Exact error reports, in the reference's order (projection order inside a
    // row; the packed key orders rows).  Cold: only rows the fast pass flagged.
    if (__ballot(badk != 0)) {
        for (uint32_t k = 0; k < nk; k++) {
            if (!((badk >> k) & 1)) continue;
            const uint32_t i = k * kDT + tid;
            const uint32_t ra = ro[2 * i] - abase, rl = ro[2 * i + 2] - ro[2 * i];
            const uint64_t row = T.r0 + i;
            if (rl < bs) { report(A.err, err_key(T.b, row, 0, kStMalformed)); continue; }
            for (uint32_t p = 0; p < nproj; p++) {
                const DecProj pc = ldproj(A, p);
                if ((src.u8(ra + (pc.bit >> 3)) >> (pc.bit & 7)) & 1) continue;
                const uint32_t fo = bs + pc.offset;
                bool bad = false;
                if (pc.is_utf8) {
                    uint32_t pay;
                    utf8_cell(src, ra, rl, bs, fo, true, &pay, &bad);
                } else {
                    bad = fo + pc.width > rl;
                }
                if (bad) { report(A.err, err_key(T.b, row, p, kStMalformed)); break; }
            }
        }
    }
    dstamp(A, S, 2);
    if (!A.nutf8) return;
    lds_barrier();  // every wave's chunk totals are in LDS
    dstamp(A, S, 5);

    // ---- pass 2: per utf8 column: cross-tile prefix, offsets, string bytes ----
#pragma unroll 1
    for (uint32_t p = 0; p < nproj; p++) {
        const DecProj pc = ldproj(A, p);
        if (!pc.is_utf8) continue;
        const DecOut o = ldout(A, (uint64_t)T.b * nproj + p);
        // Every wave scans the (<= 32) chunk totals itself: no further barrier.
        const LAS uint32_t* pu = pre + pc.uslot * PS;
        const uint32_t ctot = lane < nchunk ? pu[lane] : 0;
        const uint32_t cinc = wave_scan_u32(ctot);
        const uint32_t agg = __builtin_amdgcn_readlane(cinc, 63);
        if (!A.local && tid == 0) publish(A.lookback + (uint64_t)pc.uslot * A.total_tiles + T.t, (uint64_t)agg + 1);
        // Block-local mode: this workgroup decodes the whole block in tile
        // order, so the prefix is its own running sum.  Window mode: its own
        // inclusive prefix of tile t - G (same block) plus the aggregates of the
        // tiles between (window_prefix).  Each wave keeps its own copy.
        LAS uint64_t* mine = S.mine + wave * A.nutf8 + pc.uslot;
        uint64_t prefix;
        if (A.local) {
            prefix = T.t == T.tfirst ? 0 : sgpr64(*mine);
        } else {
            const uint64_t G = gridDim.x;
            const bool have_prev = T.t >= T.tfirst + G;
            const uint64_t lo = have_prev ? T.t - G + 1 : T.tfirst;
            const uint64_t* st = A.lookback + (uint64_t)pc.uslot * A.total_tiles;
            prefix = sgpr64((kDbg && (A.debug & 2)) ? 0 : window_prefix<kDW>(st, lo, T.t, have_prev ? *mine : 0, S.w, A.err,
                                                               err_key(T.b, T.r0, p, 0)));
        }
        if (lane == 0) *mine = prefix + agg;
        if (tid == 0) {
            if (T.t == T.tfirst) gp(o.offsets)[0] = 0;
            if (T.last) gp(A.lens)[(uint64_t)T.b * nproj + p] = prefix + agg;
        }
        GAS int32_t* ob = gp(o.offsets) + T.r0 + 1;  // uniform base
        const uint32_t fo = bs + pc.offset;
#pragma unroll 1
        for (uint32_t k = 0; k < nk; k++) {
            const uint32_t c = k * kDW + wave;
            if (c >= nchunk) break;  // wave-uniform
            const uint32_t i = k * kDT + tid;
            const bool act = i < T.nr;
            uint32_t slen, pay;
            if (pc.uslot < A.cell_cols) {
                const uint64_t cl = S.cell[pc.uslot * R + i];
                slen = (uint32_t)(cl >> 32);
                pay = (uint32_t)cl;
            } else {  // re-parse (more utf8 columns than the cell cache holds)
                const uint32_t ra = ro[2 * i] - abase;
                const uint32_t rl = act ? ro[2 * i + 2] - ro[2 * i] : 0;
                const bool present = rl >= bs && rl != 0;
                const bool nul = !present || ((src.u8(ra + (pc.bit >> 3)) >> (pc.bit & 7)) & 1);
                bool bad;
                slen = utf8_cell(src, ra, rl, bs, fo, !nul, &pay, &bad);
            }
            slen = act ? slen : 0;
            const uint32_t inc = wave_scan_u32(slen);  // < tile span < 4 GiB
            const uint32_t wn = __builtin_amdgcn_readlane(ctot, c);       // this chunk's bytes
            const uint64_t ws = prefix + (__builtin_amdgcn_readlane(cinc, c) - wn);  // and output start
            const bool fits = ws + wn <= 0x7FFFFFFFull;    // every i32 offset representable
            const bool room = ws + wn <= o.values_cap;
            if (fits) {
                if (act) ob[i] = (int32_t)((uint32_t)ws + inc);
            } else if (act) {
                const uint64_t end = ws + inc;
                if (end > 0x7FFFFFFFull) report(A.err, err_key(T.b, T.r0 + i, p, kStOverflow));
                else ob[i] = (int32_t)end;
            }
            if (!room && act && slen && ws + inc > o.values_cap)
                report(A.err, err_key(T.b, T.r0 + i, p, kStCapacity));
            // Each lane stores its own string straight to HBM: dword moves from
            // the stage (aligned reads + alignbyte) as unaligned global_store_dword
            // (gfx9 unaligned mode), then a 0-3 byte tail; the L2 merges the
            // wave's partial lines.  Any non-ASCII byte is noted for the DFA.
            dstamp(A, S, 3);
            uint32_t hi_bits = 0;
            if (fits && room && !(kDbg && (A.debug & 1))) {
                GAS uint8_t* dst = gp(o.values) + ws + (inc - slen);
                uint32_t q = 0;
#pragma unroll 1
                for (; q + 4 <= slen; q += 4) {
                    const uint32_t v = src.u32(pay + q);
                    *(GAS uint32_t*)(dst + q) = v;
                    hi_bits |= v;
                }
                const uint32_t n = slen - q;  // 0..3 tail bytes
                if (n) {
                    const uint32_t v = src.head(pay + q, n);
                    hi_bits |= v;
                    if (n & 2) *(GAS uint16_t*)(dst + q) = (uint16_t)v;
                    if (n & 1) dst[q + (n & 2)] = (uint8_t)(v >> (8 * (n & 2)));
                }
            } else if (slen) {
#pragma unroll 1
                for (uint32_t q = 0; q < slen; q += 4) hi_bits |= src.head(pay + q, slen - q);
            }
            dstamp(A, S, 6);
            if ((hi_bits & 0x80808080u) && !utf8_valid_slow(src, pay, slen))
                report(A.err, err_key(T.b, T.r0 + i, p, kStUtf8));
        }
    }
    dstamp(A, S, 4);
}

// A tile whose rows outgrew the stage: the same decoder over HBM.
template <int KMAX>
__device__ __forceinline__ void decode_tile_hbm(const DecodeArgs& A, const DecTile& T, LAS uint8_t* buf,
                                                          DecLayout L, DecLds S) {
    decode_tile<KMAX>(A, HbmSrc{gp(ldblk(A, T.b).data) + T.abase}, T, buf, L, S);
}

// LDS (dynamic): [buffer 0][buffer 1][nulls: nproj u32][w: 4 u64]
//                [mine: 4 x nutf8 u64][st: 8 u64][cell: cell_cols x R u64]
// The arguments are re-read from the kernarg segment every tile (s_load, K$
// hits) instead of being held in SGPRs across the loop: with ~30 argument
// words live, the tile code ran out of SGPRs and spilled to VGPR lanes.
__device__ __forceinline__ DecodeArgs load_args() {
    const CAS DecodeArgs* ap = (const CAS DecodeArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ap));  // opaque: no hoisting across the loop
    DecodeArgs A;
    A.blocks = ap->blocks; A.proj = ap->proj; A.outs = ap->outs; A.lookback = ap->lookback;
    A.prev = ap->prev; A.nulls = ap->nulls; A.lens = ap->lens; A.err = ap->err; A.stamps = ap->stamps;
    A.total_tiles = ap->total_tiles; A.nblocks = ap->nblocks; A.nproj = ap->nproj; A.nutf8 = ap->nutf8;
    A.bs = ap->bs; A.cap = ap->cap; A.stage = ap->stage; A.debug = ap->debug;
    A.rows_per_tile = ap->rows_per_tile; A.cell_cols = ap->cell_cols; A.local = ap->local;
    A.lds_rowoff = ap->lds_rowoff; A.lds_stage = ap->lds_stage; A.lds_buf = ap->lds_buf;
    A.lds_nulls = ap->lds_nulls; A.lds_w = ap->lds_w; A.lds_mine = ap->lds_mine; A.lds_st = ap->lds_st;
    A.lds_cell = ap->lds_cell; A.lds_total = ap->lds_total;
    // every field above: a new DecodeArgs member must be copied here too
    static_assert(sizeof(DecodeArgs) == 160, "load_args: copy every DecodeArgs field (10 x 8 B + 19 x 4 B)");
    return A;
}

__device__ __forceinline__ DecLayout dec_plan(const DecodeArgs& A) {
    DecLayout L;
    L.pre = 0;
    L.rowoff = A.lds_rowoff;
    L.stage = A.lds_stage;
    L.bytes = A.lds_buf;
    return L;
}

__device__ __forceinline__ DecLds dec_lds(const DecodeArgs& A, LAS uint8_t* lds, const DecLayout&) {
    DecLds S;
    S.nulls = (LAS uint32_t*)(lds + A.lds_nulls);
    S.w = (LAS uint64_t*)(lds + A.lds_w);
    S.mine = (LAS uint64_t*)(lds + A.lds_mine);
    S.st = (LAS uint64_t*)(lds + A.lds_st);
    S.cell = (LAS uint64_t*)(lds + A.lds_cell);
    return S;
}

// KMAX = rows_per_tile / kDT: 64-row chunks per wave per tile.
template <int KMAX>
__global__ void __launch_bounds__(kDT) decode_kernel(DecodeArgs A0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_[];
    LAS uint8_t* lds = (LAS uint8_t*)lds_;
    const uint32_t tid = tidx();
    TileRef cur, nxt;
    {
        const DecodeArgs A = load_args();
        const DecLayout L = dec_plan(A);
        const DecLds S = dec_lds(A, lds, L);
        if (tid < 8) S.st[tid] = tid == 7 ? __builtin_amdgcn_s_memtime() : 0;
        for (uint32_t p = tid; p < kDW * A.nproj; p += kDT) S.nulls[p] = 0;
        cur = first_ref(A);
        if (!cur.ok) return;  // uniform
        issue_stage(A, tile_of(A, cur), lds, L);
        nxt = next_ref(A, cur);
    }
    for (uint32_t i = 0; cur.ok; i++) {
        const DecodeArgs A = load_args();
        const DecLayout L = dec_plan(A);
        const DecLds S = dec_lds(A, lds, L);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA for `cur` landed
        __syncthreads();                                  // ... and every other wave's
        dstamp(A, S, 0);
        if (nxt.ok) issue_stage(A, tile_of(A, nxt), lds + ((i + 1) & 1) * L.bytes, L);
        const TileRef nn = next_ref(A, nxt);
        dstamp(A, S, 1);
        LAS uint8_t* buf = lds + (i & 1) * L.bytes;
        const DecTile T = tile_of(A, cur);
        const uint64_t span = ((T.end + 15) & ~15ull) - T.abase;
        if (T.end - T.abase > 0xFFFFFFF0ull) {  // > 4 GiB tile: unsupported
            if (tid == 0) {
                report(A.err, err_key(T.b, T.r0, 0, kStMalformed));
                for (uint32_t u = 0; u < A.nutf8; u++) publish(A.lookback + (uint64_t)u * A.total_tiles + T.t, 1);
            }
        } else if (kDbg && (A.debug & 4)) {
            // ablation: staging only
        } else if (span <= A.stage) {
            decode_tile<KMAX>(A, StageSrc{buf + L.stage}, T, buf, L, S);
        } else {
            decode_tile_hbm<KMAX>(A, T, buf, L, S);
        }
        // Each wave flushes its own null counters when its block changes (or
        // at the end): wave-private LDS, so no barrier.
        if (!nxt.ok || nxt.b != cur.b) {
            LAS uint32_t* wn = S.nulls + (tid >> 6) * A.nproj;
            for (uint32_t p = tid & 63; p < A.nproj; p += 64) {
                const uint32_t v = wn[p];
                if (v) {
                    __hip_atomic_fetch_add(gp(A.nulls) + (uint64_t)T.b * A.nproj + p, (unsigned long long)v,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    wn[p] = 0;
                }
            }
        }
        cur = nxt;
        nxt = nn;
    }
    const DecodeArgs A = load_args();
    const DecLds S = dec_lds(A, lds, dec_plan(A));
    if (kDbg && (A.debug & 8) && tid == 0)
        for (int j = 0; j < 7; j++) __hip_atomic_fetch_add(gp(A.stamps) + j, (unsigned long long)S.st[j],
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- encode ------------------------------------------------------------------
__device__ __forceinline__ bool in_valid(const EncCol& c, uint64_t i) {
    if (!c.validity) return true;
    uint64_t bit = c.offset + i;
    return (c.validity[bit >> 3] >> (bit & 7)) & 1;
}

template <class Dst>
__device__ __forceinline__ void put_w(Dst* d, uint64_t a, uint64_t v, uint32_t w) {
    for (uint32_t k = 0; k < w; k++) d[a + k] = (uint8_t)(v >> (8 * k));
}

// Assemble one row (WriteRow::new + write_to_row per column) at dst[0..size).
template <class Dst>
__device__ __forceinline__ void encode_row(const EncodeArgs& A, uint64_t row, Dst* dst) {
    const uint32_t bs = A.bs;
    // bitset: 0xFF then clear the bit of every non-null column (write.rs:20-35)
    for (uint32_t k = 0; k < bs; k++) {
        uint32_t byte = 0xFF;
        for (uint32_t c = 8 * k; c < min(A.ncols, 8 * k + 8); c++)
            if (in_valid(A.cols[c], row)) byte &= ~(1u << (c & 7));
        dst[k] = (uint8_t)byte;
    }
    uint64_t pos = (uint64_t)bs + A.cap;  // payload append position (write.rs:44-52)
    for (uint32_t c = 0; c < A.ncols; c++) {
        const EncCol col = A.cols[c];
        const bool v = in_valid(col, row);
        const uint64_t e = col.offset + row;
        const uint64_t fo = (uint64_t)bs + col.soff;
        if (col.dtype == kUtf8) {
            if (!v) { put_w(dst, fo, 0, 4); continue; }
            const int32_t a = col.offsets[e], z = col.offsets[e + 1];
            const uint32_t len = (uint32_t)(z - a);
            put_w(dst, fo, pos - bs, 4);
            put_w(dst, pos, len, 4);
            const uint8_t* s = col.values + a;
            for (uint32_t k = 0; k < len; k++) dst[pos + 4 + k] = s[k];
            pos += 4 + (uint64_t)len;
        } else if (col.dtype == kBool) {
            uint32_t bit = v ? ((col.values[e >> 3] >> (e & 7)) & 1) : 0;
            dst[fo] = (uint8_t)bit;
        } else {
            uint64_t x = 0;
            if (v) {
                const uint8_t* s = col.values + e * col.width;
                switch (col.width) {
                case 8: x = *reinterpret_cast<const uint64_t*>(s); break;
                case 4: x = *reinterpret_cast<const uint32_t*>(s); break;
                case 2: x = *reinterpret_cast<const uint16_t*>(s); break;
                default: x = *s; break;
                }
            }
            put_w(dst, fo, x, col.width);
        }
    }
}

__global__ void __launch_bounds__(256) encode_kernel(EncodeArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kStage + 32];
    __shared__ uint64_t s_w[4];
    const uint32_t tid = threadIdx.x;
    const uint64_t fixed = (uint64_t)A.bs + A.cap;
    uint64_t prev_incl = 0;

    for (uint64_t t = blockIdx.x; t < A.total_tiles; t += gridDim.x) {
        const uint64_t r0 = t * kTile;
        const uint32_t nr = (uint32_t)min((uint64_t)kTile, A.n_rows - r0);
        const bool active = tid < nr;
        const uint64_t row = r0 + tid;
        // Row size: bs + cap + sum over non-null utf8 of (4 + len).
        uint64_t size = active ? fixed : 0;
        if (A.nutf8 && active) {
            for (uint32_t c = 0; c < A.ncols; c++) {
                const EncCol col = A.cols[c];
                if (col.dtype == kUtf8 && in_valid(col, row)) {
                    const uint64_t e = col.offset + row;
                    size += 4 + (uint64_t)(uint32_t)(col.offsets[e + 1] - col.offsets[e]);
                }
            }
        }
        uint64_t start, tstart, span;
        if (A.nutf8 == 0) {
            start = row * fixed;
            tstart = r0 * fixed;
            span = (uint64_t)nr * fixed;
        } else {
            uint64_t agg;
            const uint64_t incl = block_incl_scan(size, s_w, &agg);
            if (tid == 0) publish(A.lookback + t, agg + 1);
            const uint64_t G = gridDim.x;
            const bool have_prev = t >= G;
            tstart = window_prefix<4>(A.lookback, have_prev ? t - G + 1 : 0, t, have_prev ? prev_incl : 0,
                                   (LAS uint64_t*)s_w, A.err, err_key(0, r0, 0, 0));
            prev_incl = tstart + agg;  // this workgroup's next tile is t + G
            start = tstart + incl - size;
            span = agg;
        }
        if (active) {
            A.row_off[row] = start;
            if (row + 1 == A.n_rows) A.row_off[row + 1] = start + size;
        }
        if (tstart + span > A.out_cap) {
            if (tid == 0) report(A.err, err_key(0, r0, 0, kStCapacity));
            continue;  // uniform: no tile-local barrier pending
        }
        if (span <= kStage) {
            if (active) encode_row(A, row, stage + (start - tstart));
            __syncthreads();
            write_out((const LAS uint8_t*)stage, gp(A.out), tstart, span, tid, 256);
            __syncthreads();
        } else if (active) {
            encode_row(A, row, A.out + start);
        }
    }
}

}  // namespace

// The LDS plan of a launch (DecodeArgs::lds_*): two tile buffers, then the
// per-wave null counters, the window scratch, the per-wave running prefixes,
// the diagnostic stamps and the utf8 cell cache.
void decode_lds_plan(DecodeArgs& a) {
    const DecLayout L = dec_layout(a.rows_per_tile, a.nutf8, a.stage);
    a.lds_rowoff = L.rowoff;
    a.lds_stage = L.stage;
    a.lds_buf = L.bytes;
    a.lds_nulls = 2 * L.bytes;
    a.lds_w = a.lds_nulls + ((4 * kDW * a.nproj + 15) & ~15u);
    a.lds_mine = a.lds_w + 8 * kDW;
    a.lds_st = a.lds_mine + 8 * kDW * a.nutf8;
    a.lds_cell = a.lds_st + 64;
    a.lds_total = a.lds_cell + 8 * a.rows_per_tile * a.cell_cols;
}

uint32_t decode_lds_bytes(uint32_t stage, uint32_t nproj, uint32_t nutf8, uint32_t rows_per_tile,
                          uint32_t cell_cols) {
    DecodeArgs a{};
    a.stage = stage;
    a.nproj = nproj;
    a.nutf8 = nutf8;
    a.rows_per_tile = rows_per_tile;
    a.cell_cols = cell_cols;
    decode_lds_plan(a);
    return a.lds_total;
}

hipError_t launch_decode(const DecodeArgs& a0, uint32_t grid, hipStream_t s) {
    DecodeArgs a = a0;
    decode_lds_plan(a);
    const uint32_t lds = a.lds_total;
    switch (a.rows_per_tile / kDT) {
    case 1: hipLaunchKernelGGL(decode_kernel<1>, dim3(grid), dim3(kDT), lds, s, a); break;
    case 2: hipLaunchKernelGGL(decode_kernel<2>, dim3(grid), dim3(kDT), lds, s, a); break;
    default: hipLaunchKernelGGL(decode_kernel<4>, dim3(grid), dim3(kDT), lds, s, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_encode(const EncodeArgs& a, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(encode_kernel, dim3(grid), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

int decode_blocks_per_cu(uint32_t lds, uint32_t rows_per_tile) {
    int n = 0;
    hipError_t e;
    switch (rows_per_tile / kDT) {
    case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_kernel<1>, kDT, lds); break;
    case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_kernel<2>, kDT, lds); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_kernel<4>, kDT, lds); break;
    }
    return e == hipSuccess ? n : 1;
}

int encode_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, encode_kernel, kTile, 0) != hipSuccess) return 1;
    return n;
}

}  // namespace murr
