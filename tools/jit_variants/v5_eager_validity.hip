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
// A segment: rows [r_begin, r_end) of block b, decoded by one workgroup.  A
// block is one segment unless the launch has fewer blocks than CUs; then its
// segments' utf8 byte counts come from a length pass (murr_jit_lengths) and
// segment k starts at the sum over segments first .. k-1 of its block.
struct Seg {
    uint32_t b, first;
    uint64_t r_begin, r_end;
};
struct Args {
    const Blk* blocks;
    const Out* outs;          // [nblocks][MJ_NPROJ]
    const void* segs;         // Seg[norder]: row ranges of non-empty blocks, in launch order
    unsigned long long* seg_tot;  // [norder][NU] utf8 bytes per segment (length pass)
    unsigned long long* nulls;  // [nblocks][MJ_NPROJ]
    unsigned long long* lens;   // [nblocks][MJ_NPROJ] utf8 data bytes
    unsigned long long* err;    // max of ~key
    uint8_t* sink;
    uint32_t norder, pad;
};

// MJ_NW waves: NC = MJ_NW - 1 consumers decode, the last wave only loads.
constexpr uint32_t NW = MJ_NW, NC = MJ_NW - 1, R = MJ_R, TR = 64 * NC * MJ_R, BS = MJ_BS, NPROJ = MJ_NPROJ,
                   NUTF8 = MJ_NUTF8, STAGE = MJ_STAGE;
// LDS slot: [row offsets (TR+1)*8 + 16][blob stage STAGE + 64 pad]
// Row offsets are staged packed: the low dword of each u64 (a gather DMA),
// 4 B per row; tiles never span 4 GiB of blob bytes.  MJ_RO8 (tuning): stage
// the u64 slice as is, 1 KiB per DMA instruction.
#ifndef MJ_RO8
#define MJ_RO8 0
#endif
constexpr uint32_t RO_W = MJ_RO8 ? 2 : 1;  // dwords per staged row offset
constexpr uint32_t RO_BYTES = ((TR + 1) * 4 * RO_W + 16 + 15) & ~15u;
constexpr uint32_t SLOT = RO_BYTES + STAGE + 64;
constexpr uint32_t ST_PIECES = STAGE / 1024;
#ifndef MJ_SLOTS
#define MJ_SLOTS 3
#endif
constexpr uint32_t NSLOT = MJ_SLOTS;                    // LDS ring slots (tiles in flight + 1)
static_assert(NSLOT >= 2 && NSLOT <= 4, "2..4 slots");
constexpr uint32_t LDS_SPAN = NSLOT * SLOT;             // [8][16 B] tile spans
constexpr uint32_t LDS_CNT = LDS_SPAN + 128;
constexpr uint32_t LDS_WT = LDS_CNT + 16;              // [NUTF8][NC] u32 wave totals
constexpr uint32_t LDS_TOTAL = LDS_WT + 4 * (NUTF8 ? NUTF8 : 1) * NC;
static_assert(STAGE % 1024 == 0, "stage is whole 1 KiB pieces");

constexpr uint32_t NU = NUTF8 ? NUTF8 : 1;
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

// ---- the workgroup's tile cursor (wave-uniform, every wave keeps a copy) -----
struct Cur {
    const uint8_t* data;
    const uint64_t* row_off;
    uint64_t n_rows, r0, r_begin, r_end;
    uint32_t k, b, first, ok;
};
DEV const Args* args() {
    const CAS Args* ap = (const CAS Args*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ap));
    return (const Args*)ap;
}
DEV void cur_load(Cur& c, uint32_t k) {
    const CAS Args* A = (const CAS Args*)args();
    c.k = sgpr(k);
    c.ok = c.k < A->norder;
    if (!c.ok) return;
    const CAS Seg* sp = (const CAS Seg*)A->segs + c.k;
    c.b = sgpr(sp->b);
    c.first = sgpr(sp->first);
    c.r_begin = sgpr64(sp->r_begin);
    c.r_end = sgpr64(sp->r_end);
    c.r0 = c.r_begin;
    const CAS Blk* bp = (const CAS Blk*)A->blocks + c.b;
    c.data = (const uint8_t*)sgpr64((uint64_t)bp->data);
    c.row_off = (const uint64_t*)sgpr64((uint64_t)bp->row_off);
    c.n_rows = sgpr64(bp->n_rows);
}
DEV void cur_next(Cur& c) {
    if (!c.ok) return;
    c.r0 += TR;
    if (c.r0 < c.r_end) return;
    cur_load(c, c.k + gridDim.x);
}
DEV uint32_t cur_nr(const Cur& c) { return (uint32_t)min((uint64_t)TR, c.r_end - c.r0); }

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
    uint32_t seg_first, seg_last;  // first / last tile of its segment
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
    T.seg_first = c.r0 == c.r_begin;
    T.seg_last = c.r0 + T.nr == c.r_end;
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
    // row offsets: lane j of piece q fetches the low dword of row_off[r0 + 64q + j]
    uint32_t n = 0;
    if (MJ_RO8) {
        const GAS uint8_t* s0 = (const GAS uint8_t*)((uintptr_t)(c.row_off + c.r0) & ~(uintptr_t)15);
        const uint32_t nb_ro = (T.ro_shift + (T.nr + 1) * 8 + 15) & ~15u;
        for (uint32_t q = 0; q * 1024 < nb_ro; q++, n++)
            if (q * 1024 + lane * 16 < nb_ro) glds16(s0 + q * 1024 + lane * 16, slot + q * 1024);
    } else {
        const GAS uint32_t* ro = (const GAS uint32_t*)(c.row_off + c.r0);
        for (uint32_t q = 0; q * 64 <= T.nr; q++, n++)  // lane 0 is always active: one instruction each
            if (q * 64 + lane <= T.nr) glds4(ro + 2 * (q * 64 + lane), slot + q * 256);
    }
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

// ---- per-row state of a wave's R chunks ----------------------------------------
struct Rows {
    uint32_t ra[R], rl[R], bits[R];
};

template <class Src> DEV bool null_bit(const Rows& W, int k, uint32_t bit, const Src& src) {
    if (BS <= 4) return W.rl[k] == 0 || ((W.bits[k] >> bit) & 1);
    const uint32_t b = src.u8(at<Src>(W.rl[k] != 0, W.ra[k] + (bit >> 3)));
    return W.rl[k] == 0 || ((b >> (bit & 7)) & 1);
}

// One fixed-width (KIND = 1/2/4/8 bytes) or bool (KIND = 0) column over the
// wave's chunks.  Returns its nulls.
template <int KIND, uint32_t FO, uint32_t BIT, class Src>
DEV uint32_t fixed_col(const Src& src, const Rows& W, const Tile& T, uint32_t rbase, const Out& o,
                       uint32_t* badk, uint32_t lane) {
    constexpr uint32_t WID = KIND == 0 ? 1 : KIND;
    uint32_t nn = 0;
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const uint32_t i = rbase + k * 64 + lane;
        const uint32_t nk = i - lane < T.nr ? min(64u, T.nr - (i - lane)) : 0u;
        const bool isnull = null_bit(W, k, BIT, src);
        const bool have = !isnull && FO + WID <= W.rl[k];
        *badk |= (uint32_t)(!isnull && !have) << k;
        const uint32_t a = at<Src>(have, W.ra[k] + FO);
        const uint64_t vm = __ballot(!isnull);
        nn += nk - (uint32_t)__popcll(vm);
        const uint64_t word = (T.r0 + i - lane) >> 6;
        if (nk && lane == 0) gp((uint64_t*)o.validity)[word] = vm;
        const bool act = lane < nk;
        if constexpr (KIND == 0) {
            const uint32_t v = src.u8(a);
            const uint64_t m = __ballot(have && v != 0);
            if (nk && lane == 0) gp((uint64_t*)o.values)[word] = m;
        } else if constexpr (KIND == 8) {
            const uint64_t v = src.u64(a);
            if (act) gp((uint64_t*)o.values)[T.r0 + i] = have ? v : 0;
        } else if constexpr (KIND == 4) {
            const uint32_t v = src.u32(a);
            if (act) gp((uint32_t*)o.values)[T.r0 + i] = have ? v : 0;
        } else if constexpr (KIND == 2) {
            const uint32_t v = src.u16(a);
            if (act) gp((uint16_t*)o.values)[T.r0 + i] = have ? (uint16_t)v : 0;
        } else {
            const uint32_t v = src.u8(a);
            if (act) gp(o.values)[T.r0 + i] = have ? (uint8_t)v : 0;
        }
    }
    return nn;
}

// Cells of one utf8 column (ReadRow::read_dynamic, read.rs:45-55): payload
// address and length per row (0 for null / missing / malformed), chunk
// inclusive scans, validity words.  Returns its nulls; *tot = wave total.
template <uint32_t FO, uint32_t BIT, bool STORE, class Src>
DEV uint32_t utf8_cells(const Src& src, const Rows& W, const Tile& T, uint32_t rbase, const Out& o,
                        uint32_t* badk, uint32_t lane, uint32_t (&pay)[R], uint32_t (&len)[R],
                        uint32_t (&inc)[R], uint32_t* tot) {
    uint32_t nn = 0, wt = 0;
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const uint32_t i = rbase + k * 64 + lane;
        const uint32_t nk = i - lane < T.nr ? min(64u, T.nr - (i - lane)) : 0u;
        const bool isnull = null_bit(W, k, BIT, src);
        const bool s_ok = !isnull && FO + 4 <= W.rl[k];
        const uint32_t slot = src.u32(at<Src>(s_ok, W.ra[k] + FO));
        const uint32_t vlen = W.rl[k] - BS;  // >= 4 when s_ok
        const bool p_ok = s_ok && slot <= vlen - 4;
        const uint32_t l = src.u32(at<Src>(p_ok, W.ra[k] + BS + slot));
        const bool good = p_ok && l <= vlen - 4 - slot;
        *badk |= (uint32_t)(!isnull && !good) << k;
        pay[k] = W.ra[k] + BS + slot + 4;
        len[k] = good ? l : 0u;
        inc[k] = wave_scan(len[k]) + wt;
        wt = __builtin_amdgcn_readlane(inc[k], 63);
        const uint64_t vm = __ballot(!isnull);
        nn += nk - (uint32_t)__popcll(vm);
        if (STORE && nk && lane == 0) gp((uint64_t*)o.validity)[(T.r0 + i - lane) >> 6] = vm;
    }
    *tot = wt;
    return nn;
}

// Copy one string from the stage to vb[d .. d+n): overlapping unaligned dword
// stores of its own bytes (head and tail), short/byte stores below 4 bytes.
// Returns the OR of its bytes (UTF-8 pre-check).
DEV uint32_t pick(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t x) {  // dword at byte x in [0, 8)
    return x < 4 ? __builtin_amdgcn_alignbyte(w1, w0, x) : __builtin_amdgcn_alignbyte(w2, w1, x - 4);
}
template <class Src>
DEV uint32_t copy_str(const Src& src, GAS uint8_t* vb, uint32_t pay, uint32_t n) {
    if constexpr (!Src::kHbm) {
        if (n <= 8) {
            uint32_t w0, w1, w2;
            src.win3(pay, w0, w1, w2);
            const uint32_t sh = pay & 3u;
            const uint32_t head = __builtin_amdgcn_alignbyte(w1, w0, sh);
            if (n >= 4) {
                const uint32_t tail = pick(w0, w1, w2, sh + n - 4);
                *(GAS u32u*)vb = head;
                *(GAS u32u*)(vb + n - 4) = tail;
                return head | tail;
            }
            if (n >= 2) {
                const uint32_t t2 = pick(w0, w1, w2, sh + n - 2) & 0xFFFFu;
                *(GAS u16u*)vb = (uint16_t)head;
                *(GAS u16u*)(vb + n - 2) = (uint16_t)t2;
                return (head & 0xFFFFu) | t2;
            }
            if (n == 1) {
                *vb = (uint8_t)head;
                return head & 0xFFu;
            }
            return 0u;
        }
    }
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

// Offsets and string bytes of one utf8 column (projection index P) for the
// wave's chunks, from the wave's prefix `base`.
template <uint32_t P, class Src>
DEV void utf8_emit(const Src& src, const Tile& T, uint32_t rbase, const Out& o, uint64_t base,
                   const uint32_t (&pay)[R], const uint32_t (&len)[R], const uint32_t (&inc)[R], uint32_t lane,
                   unsigned long long* err) {
    GAS int32_t* ob = gp(o.offsets) + T.r0 + 1;
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const uint32_t i = rbase + k * 64 + lane;
        const bool act = i < T.nr;
        const uint32_t n = len[k];
        const uint64_t e = base + inc[k];
        const uint64_t cend = base + __builtin_amdgcn_readlane(inc[k], 63);
        uint32_t hib = 0;
        if (cend <= 0x7FFFFFFFull && cend <= o.values_cap) {  // wave-uniform fast path
            if (act) ob[i] = (int32_t)e;
            if (n) hib = copy_str(src, gp(o.values) + (e - n), pay[k], n);
        } else {
            if (act) {
                if (e > 0x7FFFFFFFull) report(err, err_key(T.b, T.r0 + i, P, kStOverflow));
                else ob[i] = (int32_t)e;
                if (n && e > o.values_cap) report(err, err_key(T.b, T.r0 + i, P, kStCapacity));
            }
            for (uint32_t q = 0; q < n; q++) hib |= src.u8(pay[k] + q);
        }
        if ((hib & 0x80808080u) && !utf8_valid_slow(src, pay[k], n))
            report(err, err_key(T.b, T.r0 + i, P, kStUtf8));
    }
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

DEV const Out* outs_of(uint32_t b) {
    const Out* o = args()->outs + (uint64_t)sgpr(b) * NPROJ;
    return (const Out*)sgpr64((uint64_t)o);
}
DEV Out ldout(const Out* base, uint32_t p) {
    // opaque per use: the compiler would otherwise hoist every column's
    // descriptor into SGPRs up front (spills on wide projections)
    asm volatile("" : "+s"(base));
    const CAS Out* q = (const CAS Out*)base + p;
    Out r;
    r.values = q->values; r.validity = q->validity; r.offsets = q->offsets; r.values_cap = q->values_cap;
    return r;
}

// Null counts of a wave: column p's count in lane p % 64 of nn[p / 64]
// (VGPRs, not an SGPR per column).
constexpr uint32_t NNV = (NPROJ + 63) / 64;
template <uint32_t P> DEV void add_nulls(uint32_t (&nn)[NNV], uint32_t lane, uint32_t v) {
    // readlane / writelane: no per-column lane compare (those masks would be
    // hoisted out of the tile loop into SGPR pairs)
    const uint32_t t = __builtin_amdgcn_readlane(nn[P / 64], P % 64) + v;
    asm("v_writelane_b32 %0, %1, %2" : "+v"(nn[P / 64]) : "s"(t), "i"(P % 64));
}

// Decode one staged tile.  run[u]: the block's utf8 bytes before this tile
// (updated to after it); nn: this wave's null counts for the segment.
// LEN (the length pass): utf8 cells only; each wave adds its utf8 bytes to
// run[] (no prefix, no stores).
template <bool LEN, class Src>
DEV void decode_tile(const Src& src, const Tile& T, const LAS uint32_t* ro, LAS uint32_t* wt, uint64_t (&run)[NUTF8 ? NUTF8 : 1],
                     uint32_t (&nn)[NNV], uint32_t wave, uint32_t lane, LAS uint32_t* pcnt, uint32_t ptarget) {
    unsigned long long* err = args()->err;
    const uint32_t rbase = wave * 64 * R;
    const uint32_t abase = (uint32_t)T.abase;
    const Out* ob = outs_of(T.b);
    Rows W;
    uint32_t badk = 0;
#pragma unroll
    for (int k = 0; k < (int)R; k++) {
        const uint32_t i = rbase + k * 64 + lane;
        const uint32_t a0 = ro[RO_W * i], a1 = ro[RO_W * (i + 1)];
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

    if constexpr (!LEN) {
#define MJ_DO_FIXED(P, KIND, FO, BIT) \
    add_nulls<P>(nn, lane, fixed_col<KIND, FO, BIT>(src, W, T, rbase, ldout(ob, P), &badk, lane));
        MJ_FIXED(MJ_DO_FIXED)
#undef MJ_DO_FIXED
    }

#if MJ_NUTF8 > 0
    uint32_t upay[NUTF8][R], ulen[NUTF8][R], uinc[NUTF8][R], utot[NUTF8];
#define MJ_DO_CELLS(P, U, FO, BIT) \
    add_nulls<P>(nn, lane, utf8_cells<FO, BIT, !LEN>(src, W, T, rbase, ldout(ob, P), &badk, lane, upay[U], ulen[U], uinc[U], &utot[U]));
    MJ_UTF8(MJ_DO_CELLS)
#undef MJ_DO_CELLS
    if constexpr (LEN) {
        for (uint32_t u = 0; u < NUTF8; u++) run[u] += utot[u];
        return;
    }
#endif
    if constexpr (LEN) return;

    if (__ballot(badk != 0)) {  // cold: exact error reports
#pragma unroll
        for (int k = 0; k < (int)R; k++) {
            if (!((badk >> k) & 1)) continue;
            const uint32_t i = rbase + k * 64 + lane;
            report_row(src, W.ra[k], ro[RO_W * (i + 1)] - ro[RO_W * i], T.b, T.r0 + i, err);
        }
    }

#if MJ_NUTF8 > 0
    // wave totals -> LDS; every wave derives its prefix and the tile total
    if (lane == 0) {
        for (uint32_t u = 0; u < NUTF8; u++) wt[u * NC + wave] = utot[u];
        __hip_atomic_fetch_add(pcnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    {
        uint32_t spins = 0;
        while (__hip_atomic_load(pcnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < ptarget) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) { report(err, err_key(T.b, T.r0, 0, kStInternal)); break; }
        }
    }
    uint64_t pre[NUTF8];
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
#define MJ_DO_EMIT(P, U, FO, BIT)                                                                      \
    {                                                                                                  \
        const Out o = ldout(ob, P);                                                                    \
        if (T.first && wave == 0 && lane == 0) gp(o.offsets)[0] = 0;                                   \
        if (T.last && wave == 0 && lane == 0) gp(args()->lens)[(uint64_t)T.b * NPROJ + P] = run[U];    \
        utf8_emit<P>(src, T, rbase, o, pre[U], upay[U], ulen[U], uinc[U], lane, err);                  \
    }
    MJ_UTF8(MJ_DO_EMIT)
#undef MJ_DO_EMIT
#endif
}

DEV void flush_nulls(uint32_t b, uint32_t (&nn)[NNV], uint32_t lane) {
    unsigned long long* nulls = args()->nulls + (uint64_t)b * NPROJ;
#pragma unroll
    for (uint32_t j = 0; j < NNV; j++) {
        if (j * 64 + lane < NPROJ && nn[j])
            __hip_atomic_fetch_add(gp(nulls) + j * 64 + lane, (unsigned long long)nn[j], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        nn[j] = 0;
    }
}

}  // namespace mj

namespace mj {

// utf8 bytes of block rows before segment c (the sum of the length pass's
// totals of the block's earlier segments), per utf8 column.
DEV void seg_prefix(const Cur& c, uint64_t (&run)[NU], uint32_t lane) {
    const unsigned long long* st = args()->seg_tot;
#pragma unroll
    for (uint32_t u = 0; u < NUTF8; u++) {
        uint64_t v = 0;
        for (uint32_t j = c.first + lane; j < c.k; j += 64) v += __hip_atomic_load(gp(st) + (uint64_t)j * NU + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int m = 32; m >= 1; m >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, m, 64);
        run[u] = sgpr64(v);
    }
}

template <bool LEN>
DEV void kernel_body() {
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
        Cur cc = cur;  // the tile the decode waves work on in this iteration
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
            wait_vmcnt(NSLOT == 2 ? ns : nd + ns);
            lds_barrier();  // B_i+1: tile i+1 landed, tile i decoded
            if (!more) break;
        }
        return;
    }

    // ---- consumers ----
    uint64_t run[NUTF8 ? NUTF8 : 1];
    for (uint32_t u = 0; u < (NUTF8 ? NUTF8 : 1); u++) run[u] = 0;
    uint32_t nn[NNV];
    for (uint32_t j = 0; j < NNV; j++) nn[j] = 0;
    lds_barrier();  // B_0
    for (uint32_t it = 0;; it++) {
        LAS uint8_t* slot = lds + (it % NSLOT) * SLOT;
        const Tile T = tile_info(cur, spans + (it & 7) * 16);
        const LAS uint32_t* ro = (const LAS uint32_t*)(slot + (MJ_RO8 ? T.ro_shift : 0u));
        if (!LEN && NUTF8 && T.seg_first && !T.first) seg_prefix(cur, run, lane);
        if (T.hbm == 2) {  // a tile over 4 GiB of blob bytes (unsupported): report; prefixes undefined
            if (wave == 0 && lane == 0) report(args()->err, err_key(T.b, T.r0, 0, kStMalformed));
            if (!LEN && NUTF8 && lane == 0) __hip_atomic_fetch_add(pcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (T.hbm) {
            decode_tile<LEN>(HbmSrc{gp(T.data) + T.abase}, T, ro, wt, run, nn, wave, lane, pcnt, NC * (it + 1));
            __builtin_amdgcn_s_waitcnt(0x0F70);
            // drain the cold path's loads here (a compiler-visible vmcnt(0)),
            // so none is pending into a register the hot path reuses
            __builtin_amdgcn_s_waitcnt(0x0F70);
        } else {
            decode_tile<LEN>(StageSrc{slot + RO_BYTES}, T, ro, wt, run, nn, wave, lane, pcnt, NC * (it + 1));
        }
        if (T.seg_last) {
            if (LEN) {  // this wave's share of the segment's utf8 bytes
                for (uint32_t u = 0; u < NUTF8; u++)
                    if (lane == 0 && run[u])
                        __hip_atomic_fetch_add(gp(args()->seg_tot) + (uint64_t)cur.k * NU + u, (unsigned long long)run[u],
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                flush_nulls(T.b, nn, lane);
            }
            for (uint32_t u = 0; u < (NUTF8 ? NUTF8 : 1); u++) run[u] = 0;
        }
        cur_next(cur);
        lds_barrier();  // B_it+1
        if (!cur.ok) break;
    }
}

}  // namespace mj

extern "C" __global__ void __launch_bounds__(64 * MJ_NW) murr_jit_decode(mj::Args) { mj::kernel_body<false>(); }
extern "C" __global__ void __launch_bounds__(64 * MJ_NW) murr_jit_lengths(mj::Args) { mj::kernel_body<true>(); }
