// murr_jit_kernel.hip — schema-specialised decode kernel, compiled at run time
// (hiprtc, gfx950) once per (segment layout, projection, tile shape) and
// cached by the context (murr_jit.cpp).  The host prepends a prelude of
// #defines (MJ_*) that fixes the bitset size, every projected column's kind,
// field offset and null bit, and the tile shape, so the per-row code is
// straight-line: no descriptor loads, no dtype dispatch, no column loops.
//
// Same contract as the generic decode kernel (murr_decode.hip) and the
// reference path it replaces: ReadBatchBuilder::add_row / add_empty / build
// and the per-dtype ColumnEncoders (src/io/row/read.rs:62-110,
// src/io/codec/primitive.rs:38-61, bool_.rs:85-104, utf8.rs:85-105);
// bit-exact Arrow buffers (arrow-rs 58 builder layout).
//
// Shape (block-local): a persistent workgroup of MJ_NW waves owns whole
// blocks (order[w], order[w+G], ...) and walks each block in tiles of
// TR = 64*MJ_NW*MJ_R rows.  Tile i+1's row-offset slice and blob span stream
// into the other half of a two-slot LDS ring (global_load_lds_dwordx4, 1 KiB
// per wave-instruction) while tile i is decoded; tile i+2's span (two u64 row
// offsets) is fetched a tile ahead, so the only dependent HBM round trip per
// tile is hidden behind a whole tile of work.  One lane decodes one row per
// 64-row chunk; wave w owns rows [w*64*R, (w+1)*64*R) of the tile.  The utf8
// offset prefix is the workgroup's running sum over its block (no cross-
// workgroup protocol): a DPP wave scan per chunk, wave totals through LDS.
//
// Malformed rows (the reference panics) are flagged in the fast path and
// reported exactly, in row-major / projection order, by a cold path.  Errors
// are an atomicMax of ~key (murr_internal.h err_key).

#ifdef __HIPCC_RTC__
typedef unsigned char uint8_t;
typedef unsigned short uint16_t;
typedef unsigned int uint32_t;
typedef unsigned long long uint64_t;
typedef int int32_t;
typedef unsigned long long uintptr_t;
#else  // offline syntax/ISA check build (make jitcheck)
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#define GAS __attribute__((address_space(1)))
#define LAS __attribute__((address_space(3)))
#define CAS __attribute__((address_space(4)))
#define DEV __device__ __forceinline__

typedef uint16_t __attribute__((aligned(1))) u16u;
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;

namespace mj {

// ---- argument block (layout shared with murr_jit.cpp: JitArgs) -------------
struct Blk {  // = murr::DecBlock
    const uint8_t* data;
    const uint64_t* row_off;
    uint64_t n_rows;
    uint64_t tile_base;
};
struct Out {  // = murr::DecOut
    uint8_t* values;
    uint8_t* validity;
    int32_t* offsets;
    uint64_t values_cap;
};
struct Args {
    const Blk* blocks;
    const Out* outs;          // [nblocks][MJ_NPROJ]
    const uint32_t* order;    // non-empty blocks, in launch order
    unsigned long long* nulls;  // [nblocks][MJ_NPROJ]
    unsigned long long* lens;   // [nblocks][MJ_NPROJ] utf8 data bytes
    unsigned long long* err;    // max of ~key
    uint8_t* sink;              // 1 KiB the inactive lanes of unmasked stores write to
    uint32_t norder, pad;
};

// MJ_NW waves: NC = MJ_NW - 1 consumers decode, the last wave only loads.
constexpr uint32_t NW = MJ_NW, NC = MJ_NW - 1, R = MJ_R, TR = 64 * NC * MJ_R, BS = MJ_BS, NPROJ = MJ_NPROJ,
                   NUTF8 = MJ_NUTF8, STAGE = MJ_STAGE;
// LDS slot: [row offsets (TR+1)*8 + 16][blob stage STAGE + 64 pad]
constexpr uint32_t RO_BYTES = ((TR + 1) * 8 + 16 + 15) & ~15u;
constexpr uint32_t SLOT = RO_BYTES + STAGE + 64;
constexpr uint32_t RO_PIECES = (RO_BYTES + 1023) / 1024;
constexpr uint32_t ST_PIECES = STAGE / 1024;
#ifndef MJ_SLOTS
#define MJ_SLOTS 2
#endif
constexpr uint32_t NSLOT = MJ_SLOTS;                    // LDS ring slots (tiles in flight + 1)
static_assert(NSLOT >= 2 && NSLOT <= 4, "2..4 slots");
constexpr uint32_t LDS_SPAN = NSLOT * SLOT;             // [8][16 B] tile spans
constexpr uint32_t LDS_CNT = LDS_SPAN + 128;            // u32 prefix arrival counter (+ pad)
constexpr uint32_t LDS_WT = LDS_CNT + 16;               // [NUTF8][NC] u32 wave totals
constexpr uint32_t LDS_TOTAL = LDS_WT + 4 * (NUTF8 ? NUTF8 : 1) * NC;
static_assert(STAGE % 1024 == 0, "stage is whole 1 KiB pieces");

enum : uint32_t { kStUtf8 = 1, kStOverflow = 4, kStMalformed = 5, kStCapacity = 6, kStInternal = 10 };

DEV uint64_t err_key(uint64_t block, uint64_t row, uint32_t col, uint32_t status) {
    if (row > 0xFFFFFFFFull) row = 0xFFFFFFFFull;
    if (block > 0x3FFFFull) block = 0x3FFFFull;
    return (block << 46) | (row << 14) | ((uint64_t)(col & 0x3FF) << 4) | (status & 0xF);
}
DEV void report(unsigned long long* err, uint64_t key) {
    __hip_atomic_fetch_max((GAS unsigned long long*)err, (unsigned long long)~key, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
template <class T> DEV GAS T* gp(T* p) { return (GAS T*)p; }
template <class T> DEV const GAS T* gp(const T* p) { return (const GAS T*)p; }
DEV uint32_t sgpr(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
DEV uint64_t sgpr64(uint64_t v) { return ((uint64_t)sgpr((uint32_t)(v >> 32)) << 32) | sgpr((uint32_t)v); }
DEV uint32_t lane_id() {
    uint32_t t = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    return t;
}

// Wave64 inclusive scan on DPP (row_shr 1/2/4/8, row_bcast 15/31).
DEV uint32_t wave_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);
    return v;
}

// UTF-8 well-formedness (Unicode Table 3-7 = Rust core::str::from_utf8).
struct Utf8Dfa {
    uint32_t need = 0, lo = 0x80, hi = 0xBF;
    bool bad = false;
    DEV void step(uint32_t c) {
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
    DEV bool ok() const { return !bad && need == 0; }
};

// Tuning-only ablations (MURR_JIT_DEFS="MJ_ABLATE=n"; wrong outputs, never
// in a production prelude): 1 no string stores, 2 string stores 4-B aligned,
// 4 no fixed-width value stores, 8 no utf8 offset stores, 16 no validity
// stores, 32 fixed 4-B values stored by 16 lanes x 16 B.
#ifndef MJ_ABLATE
#define MJ_ABLATE 0
#endif

// ---- byte sources ------------------------------------------------------------
// Tile bytes staged in LDS (hot path).  Aligned dword reads + v_alignbyte (an
// unaligned ds_read_b32 is correct on gfx950 but far slower).  Reads are
// unguarded: the stage has 64 B of pad and an out-of-allocation LDS read
// returns 0; callers mask what they read for rows that fail validation.
struct StageSrc {
    static constexpr bool kHbm = false;
    const LAS uint8_t* s;
    DEV uint32_t u8(uint32_t a) const { return s[a]; }
    DEV uint32_t u32(uint32_t a) const {
        const LAS uint32_t* w = (const LAS uint32_t*)(s + (a & ~3u));
        return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
    }
    DEV uint32_t u16(uint32_t a) const { return u32(a) & 0xFFFFu; }
    DEV uint64_t u64(uint32_t a) const {
        const LAS uint32_t* w = (const LAS uint32_t*)(s + (a & ~3u));
        const uint32_t sh = a & 3u, w0 = w[0], w1 = w[1], w2 = w[2];
        return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) |
               ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    }
    // three aligned dwords covering [a & ~3, (a & ~3) + 12)
    DEV void win3(uint32_t a, uint32_t& w0, uint32_t& w1, uint32_t& w2) const {
        const LAS uint32_t* w = (const LAS uint32_t*)(s + (a & ~3u));
        w0 = w[0]; w1 = w[1]; w2 = w[2];
    }
};
// A tile whose span outgrew the stage is decoded from HBM: exact-width
// unaligned loads, never a byte past the field; unwanted reads are pointed at
// the tile's first byte by the caller (at()).
struct HbmSrc {
    static constexpr bool kHbm = true;
    const GAS uint8_t* g;
    DEV uint32_t u8(uint32_t a) const { return g[a]; }
    DEV uint32_t u16(uint32_t a) const { return *(const GAS u16u*)(g + a); }
    DEV uint32_t u32(uint32_t a) const { return *(const GAS u32u*)(g + a); }
    DEV uint64_t u64(uint32_t a) const { return *(const GAS u64u*)(g + a); }
};
template <class Src> DEV uint32_t at(bool ok, uint32_t a) { return Src::kHbm && !ok ? 0u : a; }

// ---- LDS-DMA (inline asm: kept out of the compiler's waitcnt bookkeeping;
// every wave drains its own with vmcnt(0) before the tile barrier) ----------
DEV void glds16(const GAS void* src, LAS void* dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst))
                 : "memory");
}
DEV void tile_barrier() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Phase stamps (MJ_STAMPS builds only, MURR_JIT_STAMPS=1): cycles per phase
// summed over waves into err[2..17].  Loader: issue, -, vmcnt wait, tile
// barrier.  Consumers: tile barrier, prefix wait, fixed columns, utf8 emit,
// row offsets, utf8 slots, utf8 lengths, windows, error check, tile setup.
#ifndef MJ_STAMPS
#define MJ_STAMPS 0
#endif
struct Stamps {
    uint64_t t = 0, acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    DEV void start() { if (MJ_STAMPS) t = __builtin_amdgcn_s_memtime(); }
    DEV void lap(int i) {
        if (MJ_STAMPS) { const uint64_t n = __builtin_amdgcn_s_memtime(); acc[i] += n - t; t = n; }
    }
    DEV void flush(unsigned long long* err, int base, int n, uint32_t lane) {
        if (MJ_STAMPS && lane == 0)
            for (int i = 0; i < n; i++)
                __hip_atomic_fetch_add((GAS unsigned long long*)err + 2 + base + i, (unsigned long long)acc[i],
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};

// ---- the workgroup's tile cursor (wave-uniform, every wave keeps a copy) -----
struct Cur {
    const uint8_t* data;
    const uint64_t* row_off;
    uint64_t n_rows, r0;
    uint32_t k, b, ok;
};
DEV const Args* args() {
    const CAS Args* ap = (const CAS Args*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ap));
    return (const Args*)ap;
}
DEV void cur_load(Cur& c, uint32_t k) {
    const CAS Args* A = (const CAS Args*)args();
    c.k = sgpr(k);
    c.r0 = 0;
    c.ok = c.k < A->norder;
    if (!c.ok) return;
    c.b = sgpr(((const CAS uint32_t*)A->order)[c.k]);
    const CAS Blk* bp = (const CAS Blk*)A->blocks + c.b;
    c.data = (const uint8_t*)sgpr64((uint64_t)bp->data);
    c.row_off = (const uint64_t*)sgpr64((uint64_t)bp->row_off);
    c.n_rows = sgpr64(bp->n_rows);
}
DEV void cur_next(Cur& c) {
    if (!c.ok) return;
    c.r0 += TR;
    if (c.r0 < c.n_rows) return;
    cur_load(c, c.k + gridDim.x);
}
DEV uint32_t cur_nr(const Cur& c) { return (uint32_t)min((uint64_t)TR, c.n_rows - c.r0); }

// Span of a tile (row_off[r0], row_off[r0 + nr]) into a 16-B LDS entry:
// wave 0, lanes 0-3, one LDS-DMA dword each (no register results, so the
// compiler never waits on it; the loop-top vmcnt(0) + barrier publish it).
DEV void glds4(const GAS void* src, LAS void* dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst))
                 : "memory");
}
DEV void span_issue(const Cur& c, LAS uint8_t* ent, uint32_t wave, uint32_t lane) {
    if (wave == 0 && c.ok && lane < 4) {
        const uint64_t r = c.r0 + (lane < 2 ? 0u : cur_nr(c));
        glds4((const GAS uint8_t*)(c.row_off + r) + (lane & 1) * 4, ent);
    }
}

// The staged tile: where its bytes are and how they map to LDS.
struct Tile {
    uint64_t r0, abase;
    const uint8_t* data;
    uint32_t b, nr, ro_shift, hbm, first, last, span;  // span: staged blob bytes (16-B granules)
};

// A tile's placement, from the cursor and its span (LDS entry `ent`).
DEV Tile tile_info(const Cur& c, const LAS uint8_t* ent) {
    Tile T;
    const uint64_t base = sgpr64(((const LAS uint64_t*)ent)[0]);
    const uint64_t end = sgpr64(((const LAS uint64_t*)ent)[1]);
    T.r0 = c.r0;
    T.nr = cur_nr(c);
    T.b = c.b;
    T.data = c.data;
    T.abase = base & ~15ull;
    T.first = c.r0 == 0;
    T.last = c.r0 + T.nr == c.n_rows;
    const uint64_t span = ((end + 15) & ~15ull) - T.abase;
    T.hbm = end < base || end - T.abase > 0xFFFFFF00ull ? 2u : span > STAGE ? 1u : 0u;
    T.span = T.hbm ? 0u : (uint32_t)span;
    const uintptr_t rp = (uintptr_t)(c.row_off + c.r0);
    T.ro_shift = (uint32_t)(rp & 15);
    return T;
}

// The loader wave's LDS-DMA of one tile: its row-offset slice, then (unless
// it outgrew the stage) its blob span, in 1 KiB pieces.
DEV uint32_t tile_dma(const Tile& T, const Cur& c, LAS uint8_t* slot, uint32_t lane) {
    const GAS uint8_t* s0 = (const GAS uint8_t*)((uintptr_t)(c.row_off + c.r0) & ~(uintptr_t)15);
    const uint32_t nb_ro = (T.ro_shift + (T.nr + 1) * 8 + 15) & ~15u;
    uint32_t n = 0;
    for (uint32_t q = 0; q * 1024 < nb_ro; q++, n++)  // lane 0 is always active: one instruction each
        if (q * 1024 + lane * 16 < nb_ro) glds16(s0 + q * 1024 + lane * 16, slot + q * 1024);
    if (T.hbm) return n;
    const GAS uint8_t* g = gp(c.data) + T.abase;
    for (uint32_t q = 0; q * 1024 < T.span; q++, n++)
        if (q * 1024 + lane * 16 < T.span) glds16(g + q * 1024 + lane * 16, slot + RO_BYTES + q * 1024);
    return n;
}

// s_waitcnt vmcnt(n) for a wave-uniform run-time n (clamped to the 6-bit
// field: a larger n waits for more than needed, never for less).
DEV void wait_vmcnt(uint32_t n) {
    switch (n < 63u ? n : 63u) {
#define W(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
        W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15)
        W(16) W(17) W(18) W(19) W(20) W(21) W(22) W(23) W(24) W(25) W(26) W(27) W(28) W(29) W(30) W(31)
        W(32) W(33) W(34) W(35) W(36) W(37) W(38) W(39) W(40) W(41) W(42) W(43) W(44) W(45) W(46) W(47)
        W(48) W(49) W(50) W(51) W(52) W(53) W(54) W(55) W(56) W(57) W(58) W(59) W(60) W(61) W(62) W(63)
#undef W
    }
}

DEV const Out* outs_of(uint32_t b) {
    const Out* o = args()->outs + (uint64_t)sgpr(b) * NPROJ;
    return (const Out*)sgpr64((uint64_t)o);
}
DEV Out ldout(const Out* base, uint32_t p) {
    const CAS Out* q = (const CAS Out*)base + p;
    Out r;
    r.values = q->values; r.validity = q->validity; r.offsets = q->offsets; r.values_cap = q->values_cap;
    return r;
}

// ---- per-row state of a wave's R chunks ----------------------------------------
struct Rows {
    uint32_t ra[R], rl[R], bits[R];
};

template <class Src> DEV bool null_bit(const Rows& W, int k, uint32_t bit, const Src& src) {
    if (BS <= 4) return W.rl[k] == 0 || ((W.bits[k] >> bit) & 1);
    const uint32_t b = src.u8(at<Src>(W.rl[k] != 0, W.ra[k] + (bit >> 3)));
    return W.rl[k] == 0 || ((b >> (bit & 7)) & 1);
}

// Rows of chunk k of this wave (wave-uniform).
DEV uint32_t chunk_rows(const Tile& T, uint32_t rbase, int k) {
    const uint32_t c0 = rbase + k * 64;
    return c0 < T.nr ? min(64u, T.nr - c0) : 0u;
}

// Stores are never exec-masked for inactive lanes in the hot path: those lanes
// write to a per-lane sink in the workspace instead, so no branch splits the
// wave's straight-line code (and the scheduler can overlap LDS reads across
// columns and chunks).
DEV GAS uint8_t* sink(uint32_t lane) { return gp(args()->sink) + lane * 16; }

// Validity / bool value words of the wave's chunks: lane k < R stores chunk
// k's word (one instruction per column).
DEV void store_words(uint8_t* base, const Tile& T, uint32_t rbase, const uint64_t (&w)[R], uint32_t lane) {
    uint64_t v = w[0];
#pragma unroll
    for (int k = 1; k < (int)R; k++) v = lane == (uint32_t)k ? w[k] : v;
    const bool act = lane < R && rbase + lane * 64 < T.nr;
    GAS uint64_t* dst = act ? gp((uint64_t*)base) + ((T.r0 + rbase) >> 6) + lane : (GAS uint64_t*)sink(lane);
    if (lane < R) *dst = v;
}

// ---- column descriptors (compile-time; the prelude lists them) ----------------
template <uint32_t P_, uint32_t KIND_, uint32_t FO_, uint32_t BIT_> struct FC {  // fixed width / bool
    static constexpr uint32_t P = P_, KIND = KIND_, FO = FO_, BIT = BIT_;
};
template <uint32_t P_, uint32_t U_, uint32_t FO_, uint32_t BIT_> struct UC {  // utf8
    static constexpr uint32_t P = P_, U = U_, FO = FO_, BIT = BIT_;
};
template <class... Cs> struct G {};    // a group of fixed columns: loads, then stores
template <class... Gs> struct GL {};   // the groups

// One fixed-width (KIND = 1/2/4/8 bytes) or bool (KIND = 0) column's values
// for the wave's chunks, loaded and masked (null / malformed -> 0).
template <class C> struct FV {
    uint32_t lo[R], hi[R];
    uint64_t vm[R], bm[R];
};

template <class C, class Src>
DEV void fixed_load(FV<C>& v, const Src& src, const Rows& W, const Tile& T, uint32_t rbase, uint32_t lane,
                    uint32_t& nn, uint32_t* badk) {
    constexpr uint32_t WID = C::KIND == 0 ? 1 : C::KIND;
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const bool isnull = null_bit(W, k, C::BIT, src);
        const bool have = !isnull && C::FO + WID <= W.rl[k];
        *badk |= (uint32_t)(!isnull && !have) << k;
        const uint32_t a = at<Src>(have, W.ra[k] + C::FO);
        v.vm[k] = __ballot(!isnull);  // lanes past the tile are null
        nn += chunk_rows(T, rbase, k) - (uint32_t)__popcll(v.vm[k]);
        v.hi[k] = 0;
        if constexpr (C::KIND == 0) {
            v.bm[k] = __ballot(have && src.u8(a) != 0);
            v.lo[k] = 0;
        } else if constexpr (C::KIND == 8) {
            const uint64_t x = src.u64(a);
            v.lo[k] = have ? (uint32_t)x : 0u;
            v.hi[k] = have ? (uint32_t)(x >> 32) : 0u;
        } else if constexpr (C::KIND == 4) {
            const uint32_t x = src.u32(a);
            v.lo[k] = have ? x : 0u;
        } else if constexpr (C::KIND == 2) {
            const uint32_t x = src.u16(a);
            v.lo[k] = have ? x : 0u;
        } else {
            const uint32_t x = src.u8(a);
            v.lo[k] = have ? x : 0u;
        }
    }
}

template <class C>
DEV void fixed_store(const FV<C>& v, const Out& o, const Tile& T, uint32_t rbase, uint32_t lane) {
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const uint32_t i = rbase + k * 64 + lane;
        const bool act = i < T.nr;
        if constexpr (C::KIND == 8) {
            GAS uint64_t* d = act ? gp((uint64_t*)o.values) + T.r0 + i : (GAS uint64_t*)sink(lane);
            *d = (uint64_t)v.lo[k] | ((uint64_t)v.hi[k] << 32);
        } else if constexpr (C::KIND == 4) {
            if (MJ_ABLATE & 32) {  // tuning only: 16 lanes x 16 B (wrong data)
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                if (lane < 16)
                    *(GAS u32x4*)(gp((uint32_t*)o.values) + T.r0 + (i - lane) + lane * 4) =
                        u32x4{v.lo[k], v.lo[k], v.lo[k], v.lo[k]};
                continue;
            }
            GAS uint32_t* d = act ? gp((uint32_t*)o.values) + T.r0 + i : (GAS uint32_t*)sink(lane);
            *d = v.lo[k];
        } else if constexpr (C::KIND == 2) {
            GAS uint16_t* d = act ? gp((uint16_t*)o.values) + T.r0 + i : (GAS uint16_t*)sink(lane);
            *d = (uint16_t)v.lo[k];
        } else if constexpr (C::KIND == 1) {
            GAS uint8_t* d = act ? gp(o.values) + T.r0 + i : sink(lane);
            *d = (uint8_t)v.lo[k];
        }
    }
    if constexpr (C::KIND == 0) store_words(o.values, T, rbase, v.bm, lane);
    store_words(o.validity, T, rbase, v.vm, lane);
}

// A group's columns: every load (and its LDS latency) ahead of every store.
template <class Src, class C, class... Rest>
DEV void fixed_chain(const Src& src, const Rows& W, const Tile& T, const Out* ob, uint32_t rbase, uint32_t lane,
                     uint32_t (&nn)[NPROJ], uint32_t* badk) {
    FV<C> v;
    fixed_load<C>(v, src, W, T, rbase, lane, nn[C::P], badk);
    if constexpr (sizeof...(Rest) > 0) fixed_chain<Src, Rest...>(src, W, T, ob, rbase, lane, nn, badk);
    fixed_store<C>(v, ldout(ob, C::P), T, rbase, lane);
}
template <class Src, class... Cs>
DEV void fixed_group(G<Cs...>, const Src& src, const Rows& W, const Tile& T, const Out* ob, uint32_t rbase,
                     uint32_t lane, uint32_t (&nn)[NPROJ], uint32_t* badk) {
    if constexpr (sizeof...(Cs) > 0) fixed_chain<Src, Cs...>(src, W, T, ob, rbase, lane, nn, badk);
}
template <class Src, class... Gs>
DEV void fixed_groups(GL<Gs...>, const Src& src, const Rows& W, const Tile& T, const Out* ob, uint32_t rbase,
                      uint32_t lane, uint32_t (&nn)[NPROJ], uint32_t* badk) {
    (fixed_group(Gs{}, src, W, T, ob, rbase, lane, nn, badk), ...);
}

// ---- utf8 columns ----------------------------------------------------------------
constexpr uint32_t NU = NUTF8 ? NUTF8 : 1;
struct UState {
    uint32_t pay[NU][R], len[NU][R], inc[NU][R], w0[NU][R], w1[NU][R], w2[NU][R];
    uint64_t vm[NU][R];
    uint32_t tot[NU];
};

// read_dynamic (read.rs:45-55), step 1: the slot (payload offset) of each row.
template <class C, class Src>
DEV void utf8_slot(UState& S, const Src& src, const Rows& W, const Tile& T, uint32_t rbase, uint32_t (&nn)[NPROJ]) {
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const bool isnull = null_bit(W, k, C::BIT, src);
        const bool s_ok = !isnull && C::FO + 4 <= W.rl[k];
        S.pay[C::U][k] = src.u32(at<Src>(s_ok, W.ra[k] + C::FO));
        S.vm[C::U][k] = __ballot(!isnull);
        nn[C::P] += chunk_rows(T, rbase, k) - (uint32_t)__popcll(S.vm[C::U][k]);
    }
}
// step 2: the length word, bounds (the reference would panic: flagged), the
// payload address, and the chunk scans of the lengths.
template <class C, class Src>
DEV void utf8_len(UState& S, const Src& src, const Rows& W, uint32_t* badk) {
    uint32_t wt = 0;
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const bool isnull = null_bit(W, k, C::BIT, src);
        const bool s_ok = !isnull && C::FO + 4 <= W.rl[k];
        const uint32_t slot = S.pay[C::U][k];
        const uint32_t vlen = W.rl[k] - BS;  // >= 4 when s_ok
        const bool p_ok = s_ok && slot <= vlen - 4;
        const uint32_t l = src.u32(at<Src>(p_ok, W.ra[k] + BS + slot));
        const bool good = p_ok && l <= vlen - 4 - slot;
        *badk |= (uint32_t)(!isnull && !good) << k;
        S.pay[C::U][k] = W.ra[k] + BS + slot + 4;
        S.len[C::U][k] = good ? l : 0u;
        S.inc[C::U][k] = wave_scan(S.len[C::U][k]) + wt;
        wt = __builtin_amdgcn_readlane(S.inc[C::U][k], 63);
    }
    S.tot[C::U] = wt;
}
// step 3 (stage only): the three aligned dwords around each string's start,
// which hold every string of up to 8 bytes.
template <class C, class Src> DEV void utf8_win(UState& S, const Src& src) {
    if constexpr (!Src::kHbm) {
#pragma unroll
        for (int k = 0; k < (int)R; k++) src.win3(S.pay[C::U][k], S.w0[C::U][k], S.w1[C::U][k], S.w2[C::U][k]);
    }
}

DEV uint32_t pick(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t x) {  // dword at byte x in [0, 8)
    return x < 4 ? __builtin_amdgcn_alignbyte(w1, w0, x) : __builtin_amdgcn_alignbyte(w2, w1, x - 4);
}

// Generic string copy (any length, stage or HBM): unaligned dword stores and a
// last overlapping dword of its own bytes; bytes below 4.  Returns the OR of
// its bytes (UTF-8 pre-check).
template <class Src> DEV uint32_t copy_str(const Src& src, GAS uint8_t* vb, uint32_t pay, uint32_t n) {
    uint32_t hib = 0, q = 0;
    if (n >= 4) {
#pragma unroll 1
        for (; q + 4 <= n; q += 4) {
            const uint32_t v = src.u32(pay + q);
            *(GAS u32u*)(vb + q) = v;
            hib |= v;
        }
        if (q < n) {
            const uint32_t v = src.u32(pay + n - 4);
            *(GAS u32u*)(vb + n - 4) = v;
            hib |= v;
        }
    } else {
        for (; q < n; q++) {
            const uint32_t v = src.u8(pay + q);
            vb[q] = (uint8_t)v;
            hib |= v;
        }
    }
    return hib;
}

template <class Src> DEV bool utf8_valid_slow(const Src& src, uint32_t a, uint32_t n) {
    Utf8Dfa dfa;
    for (uint32_t q = 0; q < n; q++) dfa.step(src.u8(a + q));
    return dfa.ok();
}

// step 4: offsets and string bytes of one utf8 column from the wave's prefix
// `base`; then its validity words.
template <class C, class Src>
DEV void utf8_emit(const UState& S, const Src& src, const Tile& T, uint32_t rbase, const Out& o, uint64_t base,
                   uint32_t lane, unsigned long long* err) {
    GAS int32_t* ob = gp(o.offsets) + T.r0 + 1;
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const uint32_t i = rbase + k * 64 + lane;
        const bool act = i < T.nr;
        const uint32_t n = S.len[C::U][k], pay = S.pay[C::U][k];
        const uint64_t e = base + S.inc[C::U][k];  // inc: inclusive over the wave's chunks
        const uint64_t cend = base + __builtin_amdgcn_readlane(S.inc[C::U][k], 63);
        uint32_t hib = 0;
        if (cend <= 0x7FFFFFFFull && cend <= o.values_cap) {  // wave-uniform fast path
            *(act ? ob + i : (GAS int32_t*)sink(lane)) = (int32_t)e;
            GAS uint8_t* vb = gp(o.values) + (e - n);
            bool slow = n != 0;
            if constexpr (!Src::kHbm) {
                // 4..8 bytes (the common case): head and tail dwords, unmasked
                const uint32_t w0 = S.w0[C::U][k], w1 = S.w1[C::U][k], w2 = S.w2[C::U][k], sh = pay & 3u;
                const uint32_t head = __builtin_amdgcn_alignbyte(w1, w0, sh);
                const uint32_t tail = pick(w0, w1, w2, sh + (n >= 4 ? n : 4u) - 4);
                const bool fast = n >= 4 && n <= 8;
                *(GAS u32u*)(fast ? vb : sink(lane)) = head;
                *(GAS u32u*)(fast ? vb + n - 4 : sink(lane) + 4) = tail;
                hib = fast ? head | tail : 0u;
                slow = n != 0 && !fast;
            }
            if (slow) hib = copy_str(src, vb, pay, n);
        } else {
            if (act) {
                if (e > 0x7FFFFFFFull) report(err, err_key(T.b, T.r0 + i, C::P, kStOverflow));
                else ob[i] = (int32_t)e;
                if (n && e > o.values_cap) report(err, err_key(T.b, T.r0 + i, C::P, kStCapacity));
            }
            for (uint32_t q = 0; q < n; q++) hib |= src.u8(pay + q);
        }
        if ((hib & 0x80808080u) && !utf8_valid_slow(src, pay, n)) report(err, err_key(T.b, T.r0 + i, C::P, kStUtf8));
    }
    store_words(o.validity, T, rbase, S.vm[C::U], lane);
}

template <class Src, class... Cs>
DEV void utf8_slots(G<Cs...>, UState& S, const Src& src, const Rows& W, const Tile& T, uint32_t rbase,
                    uint32_t (&nn)[NPROJ]) {
    (utf8_slot<Cs>(S, src, W, T, rbase, nn), ...);
}
template <class Src, class... Cs> DEV void utf8_lens(G<Cs...>, UState& S, const Src& src, const Rows& W, uint32_t* badk) {
    (utf8_len<Cs>(S, src, W, badk), ...);
}
template <class Src, class... Cs> DEV void utf8_wins(G<Cs...>, UState& S, const Src& src) { (utf8_win<Cs>(S, src), ...); }
// The block's first tile writes offsets[0] = 0 (StringBuilder); its last the
// block's utf8 byte total.
template <class C> DEV void firstlast(const Tile& T, const Out* ob, const uint64_t (&run)[NU]) {
    const Out o = ldout(ob, C::P);
    if (T.first) gp(o.offsets)[0] = 0;
    if (T.last) gp(args()->lens)[(uint64_t)T.b * NPROJ + C::P] = run[C::U];
}
template <class... Cs> DEV void utf8_firstlast(G<Cs...>, const Tile& T, const Out* ob, const uint64_t (&run)[NU]) {
    (firstlast<Cs>(T, ob, run), ...);
}
template <class Src, class... Cs>
DEV void utf8_emits(G<Cs...>, const UState& S, const Src& src, const Tile& T, uint32_t rbase, const Out* ob,
                    const uint64_t (&pre)[NU], uint32_t lane, unsigned long long* err) {
    (utf8_emit<Cs>(S, src, T, rbase, ldout(ob, Cs::P), pre[Cs::U], lane, err), ...);
}

// Exact error of a flagged row: the first projected column (projection order)
// whose cell the reference would reject (read.rs:39-55 bounds).
constexpr uint32_t kColFo[NPROJ] = {MJ_COL_FO};
constexpr uint32_t kColBit[NPROJ] = {MJ_COL_BIT};
constexpr uint32_t kColWid[NPROJ] = {MJ_COL_WID};  // 0 = utf8
template <class Src>
DEV void report_row(const Src& src, uint32_t ra, uint32_t rl, uint64_t b, uint64_t row, unsigned long long* err) {
    if (rl < BS) { report(err, err_key(b, row, 0, kStMalformed)); return; }
    for (uint32_t p = 0; p < NPROJ; p++) {
        const uint32_t bit = kColBit[p], fo = kColFo[p], wid = kColWid[p];
        if ((src.u8(ra + (bit >> 3)) >> (bit & 7)) & 1) continue;
        bool bad;
        if (wid == 0) {
            bad = fo + 4 > rl;
            if (!bad) {
                const uint32_t sv = src.u32(ra + fo);
                bad = sv > rl - BS - 4;
                if (!bad) bad = src.u32(ra + BS + sv) > rl - BS - 4 - sv;
            }
        } else {
            bad = fo + wid > rl;
        }
        if (bad) { report(err, err_key(b, row, p, kStMalformed)); return; }
    }
}

// Decode one staged tile.  run[u]: the block's utf8 bytes before this tile
// (updated to after it); nn[p]: this wave's null counts for the block.
using FixedGroups = GL<MJ_FIXED_GROUPS>;
using Utf8Cols = G<MJ_UTF8_COLS>;

template <class Src>
DEV void decode_tile(const Src& src, const Tile& T, const LAS uint32_t* ro, LAS uint32_t* wt, uint64_t (&run)[NU],
                     uint32_t (&nn)[NPROJ], uint32_t wave, uint32_t lane, Stamps& St, LAS uint32_t* pcnt,
                     uint32_t ptarget) {
    unsigned long long* err = args()->err;
    const uint32_t rbase = wave * 64 * R;
    const uint32_t abase = (uint32_t)T.abase;
    const Out* ob = outs_of(T.b);
    Rows W;
    uint32_t badk = 0;
    St.lap(9);
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const uint32_t i = rbase + k * 64 + lane;
        const uint32_t a0 = ro[2 * i], a1 = ro[2 * i + 2];
        const uint32_t rl = i < T.nr ? a1 - a0 : 0u;
        W.ra[k] = a0 - abase;
        badk |= (uint32_t)(rl != 0 && rl < BS) << k;
        W.rl[k] = rl >= BS ? rl : 0u;
        if (BS <= 4) {
            if constexpr (Src::kHbm) {
                uint32_t v = 0;
                for (uint32_t q = 0; q < BS; q++) v |= src.u8(at<Src>(W.rl[k] != 0, W.ra[k] + q)) << (8 * q);
                W.bits[k] = v;
            } else {
                W.bits[k] = src.u32(W.ra[k]);
            }
        } else {
            W.bits[k] = 0;
        }
    }

#if MJ_NUTF8 > 0
    // utf8 cells first: the wave totals go out before the fixed columns are
    // decoded, so the prefix wait below overlaps with them.
    UState U;
    if (MJ_STAMPS) asm volatile("" ::"v"(W.bits[0]), "v"(W.bits[R - 1]), "v"(W.rl[R - 1]));
    St.lap(4);
    utf8_slots(Utf8Cols{}, U, src, W, T, rbase, nn);
    if (MJ_STAMPS) asm volatile("" ::"v"(U.pay[0][0]), "v"(U.pay[NU - 1][R - 1]));
    St.lap(5);
    utf8_lens(Utf8Cols{}, U, src, W, &badk);
    St.lap(6);
    // Consumers only (the loader may still be issuing): each wave stores its
    // totals, then counts itself in; LDS operations of one wave complete in
    // order, so a count of NC * (tile + 1) means every total is in place.
    if (lane == 0) {
        for (uint32_t u = 0; u < NUTF8; u++) wt[u * NC + wave] = U.tot[u];
        __hip_atomic_fetch_add(pcnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    utf8_wins(Utf8Cols{}, U, src);
    if (MJ_STAMPS) asm volatile("" ::"v"(U.w0[0][0]), "v"(U.w2[NU - 1][R - 1]));
    St.lap(7);
#endif

    fixed_groups(FixedGroups{}, src, W, T, ob, rbase, lane, nn, &badk);
    St.lap(2);

    if (__ballot(badk != 0)) {  // cold: exact error reports
#pragma unroll
        for (int k = 0; k < (int)R; k++) {
            if (!((badk >> k) & 1)) continue;
            const uint32_t i = rbase + k * 64 + lane;
            report_row(src, W.ra[k], ro[2 * i + 2] - ro[2 * i], T.b, T.r0 + i, err);
        }
    }
    St.lap(8);

#if MJ_NUTF8 > 0
    {
        uint32_t spins = 0;
        while (__hip_atomic_load(pcnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < ptarget) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) { report(err, err_key(T.b, T.r0, 0, kStInternal)); break; }
        }
    }
    St.lap(1);
    uint64_t pre[NU];
#pragma unroll
    for (uint32_t u = 0; u < NUTF8; u++) {
        uint64_t before = 0, all = 0;
#pragma unroll
        for (uint32_t w = 0; w < NC; w++) {
            const uint32_t v = wt[u * NC + w];
            before += w < wave ? v : 0u;
            all += v;
        }
        pre[u] = run[u] + sgpr64(before);
        run[u] += sgpr64(all);
    }
    utf8_emits(Utf8Cols{}, U, src, T, rbase, ob, pre, lane, err);
    if (wave == 0 && lane == 0) utf8_firstlast(Utf8Cols{}, T, ob, run);
#endif
    St.lap(3);
}

DEV void flush_nulls(uint32_t b, uint32_t (&nn)[NPROJ], uint32_t lane) {
    unsigned long long* nulls = args()->nulls + (uint64_t)b * NPROJ;
#pragma unroll
    for (uint32_t p = 0; p < NPROJ; p++) {
        if (nn[p] && lane == 0)
            __hip_atomic_fetch_add(gp(nulls) + p, (unsigned long long)nn[p], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        nn[p] = 0;
    }
}

}  // namespace mj

extern "C" __global__ void __launch_bounds__(64 * MJ_NW) murr_jit_decode(mj::Args) {
    using namespace mj;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_[];
    LAS uint8_t* lds = (LAS uint8_t*)lds_;
    const uint32_t lane = lane_id();
    const uint32_t wave = sgpr(threadIdx.x >> 6);
    LAS uint32_t* wt = (LAS uint32_t*)(lds + LDS_WT);
    LAS uint32_t* pcnt = (LAS uint32_t*)(lds + LDS_CNT);
    if (threadIdx.x == 0) *pcnt = 0;

    LAS uint8_t* spans = lds + LDS_SPAN;

    Cur cur;
    cur_load(cur, blockIdx.x);
    if (!cur.ok) return;

    if (wave == NC) {
        // ---- loader: NSLOT-1 tiles in flight.  At iteration i (after tile
        // barrier B_i freed slot (i-1) % NSLOT) it DMAs tile i+NSLOT-1 and
        // the span of tile i+NSLOT+1.  It issues no other vector-memory
        // instruction, so its counted vmcnt waits for exactly the DMA it
        // needs (tile i+1, and the span of tile i+NSLOT it reads next), never
        // for the consumers' stores.
        Cur cs = cur;  // next tile whose span to fetch
        for (uint32_t k = 0; k <= NSLOT; k++) {
            span_issue(cs, spans + (k & 7) * 16, 0, lane);
            cur_next(cs);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        Cur cd = cur;  // next tile to DMA
        uint32_t after0 = 0;
        for (uint32_t j = 0; j + 1 < NSLOT; j++) {
            if (cd.ok) {
                const uint32_t n = tile_dma(tile_info(cd, spans + (j & 7) * 16), cd, lds + j * SLOT, lane);
                if (j) after0 += n;
            }
            cur_next(cd);
        }
        wait_vmcnt(after0);
        lds_barrier();  // B_0: tile 0 and the spans of tiles 0 .. NSLOT landed
        Stamps S;
        S.start();
        Cur cc = cur;  // the tile the consumers decode in this iteration
        for (uint32_t it = 0;; it++) {
            cur_next(cc);
            const uint32_t more = cc.ok;
            uint32_t nd = 0, ns = 0;
            if (cd.ok) {
                const uint32_t t = it + NSLOT - 1;
                nd = tile_dma(tile_info(cd, spans + (t & 7) * 16), cd, lds + (t % NSLOT) * SLOT, lane);
                cur_next(cd);
            }
            if (cs.ok) {
                span_issue(cs, spans + ((it + NSLOT + 1) & 7) * 16, 0, lane);
                ns = 1;
                cur_next(cs);
            }
            S.lap(0);
            wait_vmcnt(NSLOT == 2 ? ns : nd + ns);
            S.lap(2);
            lds_barrier();  // B_i+1: tile i+1 landed, tile i decoded
            S.lap(3);
            if (!more) break;
        }
        S.flush(args()->err, 0, 4, lane);
        return;
    }

    // ---- consumers ----
    uint64_t run[NUTF8 ? NUTF8 : 1];
    for (uint32_t u = 0; u < (NUTF8 ? NUTF8 : 1); u++) run[u] = 0;
    uint32_t nn[NPROJ];
    for (uint32_t p = 0; p < NPROJ; p++) nn[p] = 0;
    lds_barrier();  // B_0
    Stamps S;
    S.start();
    for (uint32_t it = 0;; it++) {
        LAS uint8_t* slot = lds + (it % NSLOT) * SLOT;
        const Tile T = tile_info(cur, spans + (it & 7) * 16);
        const LAS uint32_t* ro = (const LAS uint32_t*)(slot + T.ro_shift);
        if (T.hbm == 2) {  // a tile over 4 GiB of blob bytes (unsupported): report; prefixes undefined
            if (wave == 0 && lane == 0) report(args()->err, err_key(T.b, T.r0, 0, kStMalformed));
            if (NUTF8 && lane == 0) __hip_atomic_fetch_add(pcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (T.hbm) {
            decode_tile(HbmSrc{gp(T.data) + T.abase}, T, ro, wt, run, nn, wave, lane, S, pcnt, NC * (it + 1));
            // drain the cold path's loads here (a compiler-visible vmcnt(0)),
            // so none is pending into a register the hot path reuses
            __builtin_amdgcn_s_waitcnt(0x0F70);
        } else {
            decode_tile(StageSrc{slot + RO_BYTES}, T, ro, wt, run, nn, wave, lane, S, pcnt, NC * (it + 1));
        }
        if (T.last) {
            flush_nulls(T.b, nn, lane);
            for (uint32_t u = 0; u < (NUTF8 ? NUTF8 : 1); u++) run[u] = 0;
        }
        cur_next(cur);
        S.lap(3);
        lds_barrier();  // B_it+1
        S.lap(0);
        if (!cur.ok) break;
    }
    S.flush(args()->err, 4, 12, lane);
}
