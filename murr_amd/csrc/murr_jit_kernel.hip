// murr_jit_kernel.hip — layout-specialised decode kernel, compiled at run time
// (hiprtc, gfx950) once per segment layout and cached by murr_jit.cpp (in
// memory and on disk).  The host prepends a prelude of #defines (MJ_*) that
// fixes the bitset size, the fixed row size and every column's kind, field
// offset and utf8 ordinal.  The projection is a run-time argument: a column
// is decoded when args.slot[c] names its output position, so every
// projection of a table runs the same code object (no compile on the read
// path).
//
// Same contract as the generic decode kernel (murr_decode.hip) and the
// reference path it replaces: ReadBatchBuilder::add_row / add_empty / build
// and the per-dtype ColumnEncoders (src/io/row/read.rs:62-110,
// src/io/codec/primitive.rs:38-61, bool_.rs:85-104, utf8.rs:85-105);
// bit-exact Arrow buffers (arrow-rs 58 builder layout).
//
// Shape: a workgroup of NW waves; NC = NW - 1 decode waves, the last wave only
// loads.  Tiles of TR = 64 * NC * R rows stream through an LDS ring of two
// slots (row-offset slice + blob span by global_load_lds, 1 KiB per
// wave-instruction); one lane decodes one row of a 64-row chunk.  Per row the
// bitset and the static region are read once as aligned dwords and realigned
// to the row (v_alignbyte), so every field is a compile-time register pick.
// Validity and bool words are ballots stashed in lane c of a VGPR and stored
// by one instruction per chunk for all columns.
//
// Two work modes (args.mode):
//  * local: a workgroup owns whole blocks (the launch has at least as many
//    blocks as workgroups); the utf8 offset prefix is a running sum in SGPRs.
//  * split: few blocks.  Blocks are cut into segments of a few tiles, dealt
//    round-robin over a co-resident grid (segment s -> workgroup s mod G).  A
//    workgroup streams a segment twice: the first pass decodes the fixed-width
//    columns and validity and sums the utf8 lengths; a decoupled look-back
//    over the segments before it (one 8-byte {status, value} granule per
//    segment and utf8 column) gives the segment's utf8 starting offsets; the
//    second pass re-reads the segment -- about G segments ago, so it is still
//    in the 256 MiB Infinity Cache -- and writes offsets and strings.  HBM sees
//    the blobs once.  Every wait is bounded in time; one that expires aborts
//    the launch and the host re-runs it in local mode, so a grid that was not
//    co-resident costs time, never a hang.
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
    const uint64_t* row_off;  // u64 offsets, or (ro32) u32 ones
    uint64_t n_rows;
    uint64_t tile_base;    // first global tile of this block (stream mode)
    const uint64_t* uidx;  // utf8 index (murr_utf8_index) or null: [row / 2^ulog][NU] starting offsets
    uint32_t ro32, pad;    // row_off holds u32 offsets (murr_block_t.row_off32)
};
// A segment: rows [r_begin, r_end) of block b; `first` is the index of the
// block's first segment (split mode).  Local mode walks a table of them too:
// whole blocks, or virtual blocks of an indexed block (their utf8 offsets
// start at the index's entry for r_begin).
struct Seg {  // = murr::JitSeg
    uint32_t b, first;
    uint64_t r_begin, r_end;
};
struct Out {  // = murr::DecOut
    uint8_t* values;
    uint8_t* validity;
    int32_t* offsets;
    uint64_t values_cap;
};
constexpr uint32_t NCOLS = MJ_NCOLS, BS = MJ_BS, FIX = MJ_FIX, NUTF8 = MJ_NUTF8;
constexpr uint32_t NU = NUTF8 ? NUTF8 : 1;
constexpr uint32_t NCW = (NCOLS + 63) / 64;  // 64-column lane groups
struct Args {
    const Blk* blocks;
    const Out* outs;              // [nblocks][nproj]
    const uint32_t* order;        // unused
    const void* segs;             // Seg[nseg] (split mode) or Seg[norder] (local mode)
    const uint16_t* slot_tab;     // = slot[], in memory (per-lane reads)
    const uint16_t* projcols;     // [nproj]: segment column of projection position p
    unsigned long long* nulls;    // [nblocks][nproj]
    unsigned long long* lens;     // [nblocks][nproj] utf8 data bytes
    unsigned long long* err;      // max of ~key
    unsigned long long* flags;    // split mode: [nseg][NU] look-back granules, then the segment claim word
    uint8_t* sink;
    uint64_t nseg;                // split mode: segments
    uint32_t nblocks, nproj, norder, mode;
    uint32_t stage;               // stage bytes per ring slot (multiple of 1 KiB)
    uint32_t report;              // report malformed rows (the first projection round)
    uint32_t emit;                // split mode: some utf8 column is projected (second pass)
    uint32_t ulog;                // log2 of the utf8 index stride
    unsigned int* abort_word;     // split mode: set when a wait timed out (every wait then gives up)
    unsigned int* zero_next;      // prepared launches: the other counter set, zeroed for the next run
    uint32_t zero_words, rb_words;  // ... its dwords; counter words the epilogue copies to rb_host
    unsigned int* ticket;         // prepared launches: workgroups finished (in the counter set)
    unsigned long long* rb_host;  // prepared launches: pinned host read-back ([rb_words] + done flag)
    uint32_t fast;                // the loader's fast start (MJ_FASTSTART builds): cut and split launches
    uint32_t pad_;
    uint16_t slot[(NCOLS + 1) & ~1u];  // output position of column c, 0xFFFF = not decoded
};
constexpr uint16_t kNone = 0xFFFF;

enum : uint32_t { kStUtf8 = 1, kStOverflow = 4, kStMalformed = 5, kStCapacity = 6, kStInternal = 10 };
// Phase stamps of tuning builds (MURR_JIT_DEFS=MJ_STAMPS): shader cycles
// summed over waves into err[2 + k] (murr_abi.cpp prints them with
// MURR_DECODE_VERBOSE).  k: 0 decode-wave tile barrier, 1 wave-total wait,
// 2 segment-prefix wait, 3 look-back, 4 first-pass tiles, 5 second-pass
// tiles, 6 local tiles, 7 loader waits, 8 loader total, 9 decode-wave total,
// 10 the loader's vmcnt waits (part of 7).
#ifdef MJ_STAMPS
#define MJ_TIC const uint64_t mj_t0_ = __builtin_amdgcn_s_memtime();
#define MJ_TOC(k)                                                                                             \
    if (lane_id() == 0)                                                                                       \
        __hip_atomic_fetch_add((GAS unsigned long long*)args()->err + 2 + (k),                              \
                               (unsigned long long)(__builtin_amdgcn_s_memtime() - mj_t0_), __ATOMIC_RELAXED, \
                               __HIP_MEMORY_SCOPE_AGENT);
#else
#define MJ_TIC
#define MJ_TOC(k)
#endif

// Waits are bounded in wall time (s_memrealtime, 100 MHz): 50 ms.
constexpr uint64_t kWaitTicks = 5000000;

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
// by value (HIP's min/max of mixed temporaries bind references, which ends
// up as a stack slot)
DEV uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
DEV uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }
DEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
DEV const CAS Args* args() {
    const CAS Args* ap = (const CAS Args*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ap));
    return ap;
}
// Output position of column c (compile-time c): one scalar dword load of the
// kernel arguments (a 16-bit load would be a vector load and a vmcnt wait).
DEV uint32_t slot_of(uint32_t c) {
    const CAS uint32_t* w = (const CAS uint32_t*)args()->slot;
    return (w[c >> 1] >> (16 * (c & 1))) & 0xFFFFu;
}

// A bounded wait.  `expired()` once the deadline passed or another wave of
// the launch gave up (the abort word; stream mode only), after reporting.
struct Wait {
    uint64_t t0 = 0;
    uint32_t n = 0;
    DEV bool expired(uint64_t block, uint64_t row) {
        __builtin_amdgcn_s_sleep(1);
        if ((++n & 63) != 1) return false;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (n == 1) t0 = now;
        unsigned int* ab = args()->abort_word;
        const bool late = now - t0 > kWaitTicks;
        const bool gave_up = ab && __hip_atomic_load((const GAS unsigned int*)ab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!late && !gave_up) return false;
        if (late) {
            report(args()->err, err_key(block, row, 0, kStInternal));
            if (ab) __hip_atomic_store((GAS unsigned int*)ab, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return true;
    }
};

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

// ---- layout tables (cold paths, run-time column index) ----------------------
constexpr uint32_t kColFo[NCOLS] = {
#define MJ_X(C, W, FO, U) FO,
    MJ_COLS(MJ_X)
#undef MJ_X
};
constexpr uint32_t kColW[NCOLS] = {  // 0 = utf8, 9 = bool
#define MJ_X(C, W, FO, U) W,
    MJ_COLS(MJ_X)
#undef MJ_X
};

// Word lanes per chunk (see store_words).
#ifndef MJ_FOLDB
#define MJ_FOLDB 1
#endif
constexpr bool has_bool() {
    for (uint32_t c = 0; c < NCOLS; c++)
        if (kColW[c] == 9) return true;
    return false;
}
constexpr bool FOLDB = MJ_FOLDB && has_bool() && 2 * NCOLS <= 64;
constexpr uint32_t WL = FOLDB ? 2 * NCOLS : NCOLS;
// ---- byte sources ------------------------------------------------------------
// Tile bytes staged in LDS (hot path).  Aligned dword reads + v_alignbyte (an
// unaligned ds_read_b32 is correct on gfx950 but far slower).  Reads are
// unguarded: the stage has 64 B of pad and an out-of-allocation LDS read
// returns 0; callers mask what they read for rows that fail validation.
struct StageSrc {
    static constexpr bool kHbm = false;
    const LAS uint8_t* s;
    DEV uint32_t u8(uint32_t a) const { return s[a]; }
    DEV uint32_t w(uint32_t a4) const { return ((const LAS uint32_t*)s)[a4]; }  // aligned dword a4
    DEV uint32_t u32(uint32_t a) const {
        const LAS uint32_t* p = (const LAS uint32_t*)(s + (a & ~3u));
        return __builtin_amdgcn_alignbyte(p[1], p[0], a & 3u);
    }
    DEV void win3(uint32_t a, uint32_t& w0, uint32_t& w1, uint32_t& w2) const {
        const LAS uint32_t* p = (const LAS uint32_t*)(s + (a & ~3u));
        w0 = p[0]; w1 = p[1]; w2 = p[2];
    }
};
// A tile whose span outgrew the stage is decoded from HBM: aligned dword loads
// that never leave the row's own dwords (callers point unwanted reads at the
// tile's first byte).
struct HbmSrc {
    static constexpr bool kHbm = true;
    const GAS uint8_t* g;
    DEV uint32_t u8(uint32_t a) const { return g[a]; }
    DEV uint32_t w(uint32_t a4) const { return ((const GAS uint32_t*)g)[a4]; }
    DEV uint32_t u32(uint32_t a) const { return *(const GAS u32u*)(g + a); }
};

// Projection slots loaded once per tile (MJ_HOIST >= 1) and output
// descriptors kept in per-lane registers (>= 2) instead of kernel-argument
// and descriptor loads at every use (0; tuning).
#ifndef MJ_HOIST
#define MJ_HOIST 2
#endif
// Ablations (tuning only, MURR_JIT_DEFS): skip the string byte stores / the
// fixed-width value stores, to price them.
#ifndef MJ_ABL_NOSTR
#define MJ_ABL_NOSTR 0
#endif
#ifndef MJ_ABL_NOFIX
#define MJ_ABL_NOFIX 0
#endif
// Output stores (written once, read by the caller later): plain, or
// non-temporal (MJ_OUT_NT 1: fixed-width values and utf8 offsets; the host
// picks it per layout, murr_jit.cpp prelude; 2: every output store, tuning).
#ifndef MJ_OUT_NT
#ifdef MJ_OUT_NT_LAYOUT
#define MJ_OUT_NT MJ_OUT_NT_LAYOUT
#else
#define MJ_OUT_NT 0
#endif
#endif
template <class T> DEV void ost(GAS T* p, T v) {
#if defined(MJ_OUT_NT) && MJ_OUT_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
// The other output stores (string bytes at any alignment, validity and bool
// words): non-temporal from MJ_OUT_NT 2.
template <class T> DEV void ostu(GAS uint8_t* p, T v) {
    typedef T __attribute__((aligned(1))) TU;
#if defined(MJ_OUT_NT) && MJ_OUT_NT >= 2
    __builtin_nontemporal_store(v, (GAS TU*)p);
#else
    *(GAS TU*)p = v;
#endif
}
// 1-byte values (a wave's store is half a line): like the wider ones
// (MJ_OUT_NT_W1 1), or plain (0; tuning).
#ifndef MJ_OUT_NT_W1
#define MJ_OUT_NT_W1 1
#endif
// Validity and bool words: non-temporal with MJ_OUT_NT 2 or MJ_OUT_NT_VAL (tuning).
#ifndef MJ_OUT_NT_VAL
#define MJ_OUT_NT_VAL 0
#endif
DEV void ostw(GAS uint64_t* p, uint64_t v) {
#if (defined(MJ_OUT_NT) && MJ_OUT_NT >= 2) || MJ_OUT_NT_VAL
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// ---- LDS-DMA (inline asm: kept out of the compiler's waitcnt bookkeeping;
// the loader wave waits for exactly its own DMA with counted vmcnt) ----------
// Cache policy of the blob stream (read once): MJ_BLOB_POL, e.g. " nt"
// (tuning: MURR_JIT_DEFS=MJ_BLOB_NT=1).
#if defined(MJ_BLOB_NT) && MJ_BLOB_NT
#define MJ_BLOB_POL " nt"
#else
#define MJ_BLOB_POL ""
#endif
DEV void glds16(const GAS void* src, LAS void* dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" MJ_BLOB_POL "\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst))
                 : "memory");
}
DEV void glds4(const GAS void* src, LAS void* dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off" MJ_BLOB_POL "\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst))
                 : "memory");
}
DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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

// Row offsets in the ring slot: 4 B per row.  u64 offsets: their low dwords
// gathered 64 per LDS-DMA instruction (only the low dwords are read: a tile's
// span is below 4 GiB).  u32 offsets (murr_block_t.row_off32): loaded
// linearly, 256 per dwordx4 instruction from the 16-B aligned group at or
// below the tile's first offset; the tile's offsets start `lead` dwords into
// the slot.  (Round 2 also measured whole u64s by dwordx4, 128 per
// instruction: neutral on B, and twice the LDS.)
// Early release of ring slots in local mode (decode_tile, kernel_body); 0 =
// one workgroup barrier per tile (tuning A/B).
#ifndef MJ_ER
#define MJ_ER 0
#endif
// Fast start (2-slot rings): the loader DMAs its first tile as soon as that
// tile's span is in and announces the next ones behind the DMA, with the
// scalar cache warmed for their cursors first; 0 = announce four tiles, then
// DMA (tuning A/B).
#ifndef MJ_FASTSTART
#define MJ_FASTSTART 1
#endif

// ---- shape ---------------------------------------------------------------------
template <uint32_t NW_, uint32_t R_, uint32_t NSLOT_>
struct Shape {
    static constexpr uint32_t NW = NW_, NC = NW_ - 1, R = R_, TR = 64 * (NW_ - 1) * R_;
    // LDS slot: [row offsets, u32: (TR+1)*4 + 16][stage + 64 pad].  A u32
    // block's slice lands 16-B groups whole: up to 3 dwords before the tile's
    // first offset and 3 after its last, (TR + 7) * 4 <= RO_BYTES.
    static constexpr uint32_t RO_BYTES = ((TR + 1) * 4 + 16 + 15) & ~15u;
    static_assert((TR + 7) * 4 <= RO_BYTES, "u32 offset groups fit the slot");
    // ring slots: 2 (one tile in flight while one decodes) or 3 (two in flight)
    static constexpr uint32_t NSLOT = NSLOT_;
    static_assert(NSLOT == 2 || NSLOT == 3, "ring of 2 or 3 slots");
    // after the slots: span ring [8][16 B] | tile ring [8][32 B] | counters
    // (8 words: wave totals published, segment prefix ready, epilogue count,
    // -, slot landed [2], slot released [2]) | tile prefixes [NU] u64 | wave
    // totals [2 (tile parity)][NU][NC] u32 | prefetch scratch 1 KiB
    static constexpr uint32_t SPAN_B = 128, INFO_B = 256, CNT_B = 32, PF_B = 1024;
    DEV static uint32_t slot_bytes(uint32_t stage) { return RO_BYTES + stage + 64; }
};

#ifndef MJ_LOADER_PRIO
#define MJ_LOADER_PRIO 0
#endif
// One tile as the loader dealt it (tile ring entry, 32 B).
struct TileInfo {
    uint32_t b, nr;
    uint64_t r0;
    uint64_t t;       // split mode: segment index (look-back granules)
    uint32_t flags;   // bit 0: first tile of its block, 1: last, 2: valid, 3: first of its segment
                      // (this pass), 4: last of its segment (this pass), 5-6: pass (0 local, 1, 2)
    uint32_t first;   // split mode: the block's first segment
};

// ---- the loader's tile cursor (wave-uniform) -------------------------------------
struct Cur {
    const uint8_t* data;
    const uint64_t* row_off;
    const uint64_t* uidx;
    uint64_t n_rows, r0, r_begin, r_end;
    uint32_t k, b, first, phase, ok, ro32;
};
// Cursors are built whole by value (every field assigned on every path: a
// conditionally stored field would keep the struct on the stack, and stack
// traffic would disturb the loader's counted vmcnt waits).
DEV Cur cur_make(uint32_t ok, uint32_t k, uint32_t b, uint32_t first, uint32_t phase, uint64_t r_begin, uint64_t r_end,
                 uint64_t r0) {
    Cur c;
    const CAS Blk* bp = (const CAS Blk*)args()->blocks + (ok ? b : 0u);
    c.ok = ok;
    c.k = k;
    c.b = b;
    c.first = first;
    c.phase = phase;
    c.r0 = r0;
    c.data = ok ? (const uint8_t*)sgpr64((uint64_t)bp->data) : nullptr;
    c.row_off = ok ? (const uint64_t*)sgpr64((uint64_t)bp->row_off) : nullptr;
    c.n_rows = ok ? sgpr64(bp->n_rows) : 0;
    c.uidx = ok ? (const uint64_t*)sgpr64((uint64_t)bp->uidx) : nullptr;
    c.ro32 = ok ? sgpr(bp->ro32) : 0u;
    c.r_begin = r_begin;
    c.r_end = ok && r_end == ~0ull ? c.n_rows : r_end;
    return c;
}
// local mode: the k-th (virtual) block of the launch
DEV Cur cur_local(uint32_t k) {
    k = sgpr(k);
    const uint32_t ok = k < args()->norder;
    const CAS Seg* sp = (const CAS Seg*)args()->segs + (ok ? k : 0u);
    const uint64_t rb = ok ? sgpr64(sp->r_begin) : 0, re = ok ? sgpr64(sp->r_end) : 0;
    return cur_make(ok, k, ok ? sgpr(sp->b) : 0u, 0, 0, rb, re, rb);
}
// split mode: segment k, first pass
DEV Cur cur_seg(uint32_t k) {
    k = sgpr(k);
    const uint32_t ok = k < args()->nseg;
    const CAS Seg* sp = (const CAS Seg*)args()->segs + (ok ? k : 0u);
    const uint64_t rb = ok ? sgpr64(sp->r_begin) : 0, re = ok ? sgpr64(sp->r_end) : 0;
    return cur_make(ok, k, ok ? sgpr(sp->b) : 0u, ok ? sgpr(sp->first) : 0u, 1, rb, re, rb);
}
// Split mode with more segments than workgroups: segments are claimed from a
// counter (the word after the look-back granules, zeroed with them) in the
// order workgroups actually run, so a segment's predecessors are always held
// by running workgroups.  A static deal (g, g + G, ...) makes workgroup 0's
// second segment wait on workgroup G - 1's first, and when other streams'
// kernels hold CUs that workgroup may not be resident: every resident
// workgroup waits until the bounded wait aborts the launch (three overlapped
// split launches measured 21 ms a step instead of 0.43).  One round of
// segments (nseg <= G) needs no claims: workgroup g's predecessors are
// workgroups < g, dispatched before it.  Only launches with a second pass
// wait on other workgroups (emit), so only those claim.
DEV bool seg_claims() { return args()->emit && args()->nseg > gridDim.x; }
DEV uint32_t seg_claim() {
    unsigned int* w = (unsigned int*)(args()->flags + (uint64_t)NU * args()->nseg);
    uint32_t k = 0;
    if (lane_id() == 0) k = __hip_atomic_fetch_add(gp(w), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return sgpr(k);
}
template <uint32_t MODE> DEV Cur cur_first() {
    if constexpr (MODE == 0) return cur_local(blockIdx.x);
    return cur_seg(seg_claims() ? seg_claim() : blockIdx.x);
}
// Fast start: the scalar loads behind the first cursors (the segment entries
// g, g + G, g + 2G, g + 3G, then their block entries) issued side by side, so
// the dependent chain of cursor loads that follows hits the scalar cache
// instead of paying two L2 round trips per tile.
template <uint32_t MODE> DEV void warm_scalar() {
    const uint32_t G = gridDim.x, n = MODE == 0 ? args()->norder : args()->nseg;
    if (!n) return;
    uint32_t b[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t k = blockIdx.x + j * G;
        b[j] = sgpr(((const CAS Seg*)args()->segs)[k < n ? k : n - 1].b);
    }
    uint64_t acc = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const CAS Blk* bp = (const CAS Blk*)args()->blocks + b[j];
        acc += sgpr64((uint64_t)bp->data) ^ sgpr64((uint64_t)bp->uidx);
    }
    asm volatile("; warm %0" ::"s"(acc));
}
// Local mode deals statically: workgroup g takes (virtual) blocks g, g + G,
// ...  Rounds 3 and 4 measured dynamic deals against it and dropped them: one
// queue counter (the D shard's first tiles waited 13-52 us), per-XCD pools
// claimed a tile ahead with the rest of a launch's blocks (every workgroup's
// tiles got slower, 0.104-0.112 vs 0.085 ms), and per-position claim words
// (0.078 vs 0.075 ms); DESIGN.md §7.
// The next tile: local mode walks the block, then the next block of the
// order; split mode walks the segment, then walks it again (second pass,
// when there are utf8 cells to write), then takes segment k + G.
template <uint32_t TR> DEV Cur cur_next(const Cur& c) {
    if (!c.ok) return c;
    if (c.r0 + TR < c.r_end) {
        Cur n = c;
        n.r0 = c.r0 + TR;
        return n;
    }
    if (c.phase == 0) return cur_local(c.k + gridDim.x);
    if (c.phase == 1 && args()->emit) {
        Cur n = c;
        n.phase = 2;
        n.r0 = c.r_begin;
        return n;
    }
    return cur_seg(seg_claims() ? seg_claim() : c.k + gridDim.x);
}
template <uint32_t TR> DEV uint32_t cur_nr(const Cur& c) { return (uint32_t)umin64((uint64_t)TR, c.r_end - c.r0); }

// The loader publishes tile i's identity (ring entry i & 7, lane 0) and
// fetches its span (row_off[r0], row_off[r0 + nr]) by LDS-DMA (lanes 0-3).
// Local mode: the utf8 index entry that starts a (virtual) block, fetched by
// the loader with the tile's announcement into a ring beside the tile ring
// (the prefetch scratch), so the decode waves read it from LDS instead of two
// dependent scalar loads at the block's first tile.
#ifndef MJ_PREFETCH
#define MJ_PREFETCH 0
#endif
#if MJ_PREFETCH || MJ_NUTF8 == 0 || MJ_NUTF8 > 16
constexpr bool UPRE = false;
#else
constexpr bool UPRE = true;
#endif
template <uint32_t TR>
DEV uint32_t tile_announce(const Cur& c, LAS uint8_t* span_ent, LAS uint8_t* info_ent, uint32_t lane,
                           LAS uint8_t* upre_ent) {
    if (lane == 0) {
        LAS TileInfo* ti = (LAS TileInfo*)info_ent;
        if (c.ok) {
            const uint32_t nr = cur_nr<TR>(c);
            ti->b = c.b;
            ti->nr = nr;
            ti->r0 = c.r0;
            ti->t = c.k;
            ti->first = c.first;
            // bit 7: u32 offsets; bits 8-9: the dwords before the tile's
            // first offset in its aligned 16-B group (tile_dma)
            const uint32_t lead = c.ro32 ? (uint32_t)(((uintptr_t)((const uint32_t*)c.row_off + c.r0) >> 2) & 3u) : 0u;
            ti->flags = (c.r0 == 0 ? 1u : 0u) | (c.r0 + nr == c.n_rows ? 2u : 0u) | 4u |
                        (c.r0 == c.r_begin ? 8u : 0u) | (c.r0 + nr == c.r_end ? 16u : 0u) | (c.phase << 5) |
                        (c.ro32 << 7) | (lead << 8);
        } else {
            ti->flags = 0;
        }
    }
    if (!c.ok) return 0;
    if (c.ro32) {
        // the span's two u32 offsets into the low dwords of the two u64
        // entries (lanes 0 and 2; tile_read masks the high dwords)
        if (lane == 0 || lane == 2) glds4((const GAS uint32_t*)c.row_off + c.r0 + (lane ? cur_nr<TR>(c) : 0u), span_ent);
    } else if (lane < 4) {
        const uint64_t r = c.r0 + (lane < 2 ? 0u : cur_nr<TR>(c));
        glds4((const GAS uint8_t*)(c.row_off + r) + (lane & 1) * 4, span_ent);
    }
    if constexpr (UPRE) {
        if (c.phase == 0 && c.r0 == c.r_begin && c.r0 != 0 && c.uidx) {
            const GAS uint32_t* ux = (const GAS uint32_t*)(c.uidx + (c.r0 >> args()->ulog) * NU);
            if (lane < 2 * NU) glds4(ux + lane, upre_ent);
            return 2;
        }
    }
    return 1;
}

// The staged tile: where its bytes are and how they map to LDS.
struct Tile {
    uint64_t r0, abase, t;
    const uint8_t* data;
    const uint64_t* row_off;
    uint32_t b, nr, hbm, span, first, last, seg_first, seg_last, first_seg;
    uint32_t ro32, lead;  // u32 offsets; the tile's first offset is dword `lead` of the slot
};
DEV Tile tile_read(const LAS uint8_t* span_ent, const LAS uint8_t* info_ent, uint32_t stage) {
    const LAS TileInfo* ti = (const LAS TileInfo*)info_ent;
    Tile T;
    T.b = sgpr(ti->b);
    T.nr = sgpr(ti->nr);
    T.r0 = sgpr64(ti->r0);
    T.t = sgpr64(ti->t);
    const uint32_t f = sgpr(ti->flags);
    T.first = f & 1u;
    T.last = (f >> 1) & 1u;
    T.seg_first = (f >> 3) & 1u;
    T.seg_last = (f >> 4) & 1u;
    T.ro32 = (f >> 7) & 1u;
    T.lead = (f >> 8) & 3u;
    T.first_seg = sgpr(ti->first);
    const uint64_t m = T.ro32 ? 0xFFFFFFFFull : ~0ull;  // (u32 offsets: the high dwords are stale)
    const uint64_t base = sgpr64(((const LAS uint64_t*)span_ent)[0]) & m;
    const uint64_t end = sgpr64(((const LAS uint64_t*)span_ent)[1]) & m;
    T.abase = base & ~15ull;
    const uint64_t span = ((end + 15) & ~15ull) - T.abase;
    T.hbm = end < base || end - T.abase > 0xFFFFFF00ull ? 2u : span > stage ? 1u : 0u;
    T.span = T.hbm ? 0u : (uint32_t)span;
    T.data = nullptr;
    T.row_off = nullptr;
    return T;
}
// The block's blob and row-offset pointers: the loader needs them for every
// tile, the decode waves only for a tile decoded from HBM (two dependent
// scalar loads kept off their per-tile path).
DEV void tile_ptrs(Tile& T) {
    const CAS Blk* bp = (const CAS Blk*)args()->blocks + T.b;
    T.data = (const uint8_t*)sgpr64((uint64_t)bp->data);
    T.row_off = (const uint64_t*)sgpr64((uint64_t)bp->row_off);
}
DEV Tile tile_read_ptrs(const LAS uint8_t* span_ent, const LAS uint8_t* info_ent, uint32_t stage) {
    Tile T = tile_read(span_ent, info_ent, stage);
    tile_ptrs(T);
    return T;
}
DEV uint32_t tile_valid(const LAS uint8_t* info_ent) { return sgpr(((const LAS TileInfo*)info_ent)->flags) & 4u; }
DEV uint32_t tile_phase(const LAS uint8_t* info_ent) { return (sgpr(((const LAS TileInfo*)info_ent)->flags) >> 5) & 3u; }

// The loader wave's LDS-DMA of one tile: its row-offset slice, then (unless
// it outgrew the stage) its blob span in 1 KiB pieces.  u64 offsets: their
// low dwords, a gather (lane j of piece q fetches row_off[r0 + 64q + j]).
// u32 offsets: the aligned 16-B groups that cover row_off32[r0 .. r0 + nr],
// a linear dwordx4 stream (lane j of piece q: group 64q + j).  The groups at
// either end hold only whole dwords of the same 16 B, so they never leave the
// pages the offsets live in.
template <uint32_t TR, uint32_t RO_BYTES>
DEV uint32_t tile_dma(const Tile& T, LAS uint8_t* slot, uint32_t lane) {
    uint32_t n = 0;
    if (T.ro32) {
        const GAS uint8_t* g = (const GAS uint8_t*)((uintptr_t)((const uint32_t*)T.row_off + T.r0) & ~(uintptr_t)15);
        const uint32_t groups = (T.lead + T.nr + 1 + 3) >> 2;
        for (uint32_t q = 0; q * 64 < groups; q++, n++)  // lane 0 is always active: one instruction each
            if (q * 64 + lane < groups) glds16(g + (q * 64 + lane) * 16, slot + q * 1024);
    } else {
        const GAS uint32_t* ro = (const GAS uint32_t*)(T.row_off + T.r0);
        for (uint32_t q = 0; q * 64 <= T.nr; q++, n++)  // lane 0 is always active: one instruction each
            if (q * 64 + lane <= T.nr) glds4(ro + 2 * (q * 64 + lane), slot + q * 256);
    }
    if (T.hbm) return n;
    const GAS uint8_t* g = gp(T.data) + T.abase;
    for (uint32_t q = 0; q * 1024 < T.span; q++, n++)
        if (q * 1024 + lane * 16 < T.span) glds16(g + q * 1024 + lane * 16, slot + RO_BYTES + q * 1024);
    return n;
}

// L2 prefetch of a later tile's blob span: the same LDS-DMA pieces, all
// landing in one 1 KiB scratch slot of LDS (the data is dropped; the lines
// stay in L2), so a second tile is in flight without a second ring slot.
// Returns the instructions issued.
DEV uint32_t tile_prefetch(const Tile& T, LAS uint8_t* scratch, uint32_t lane) {
    if (T.hbm) return 0;
    uint32_t n = 0;
    const GAS uint8_t* g = gp(T.data) + T.abase;
    for (uint32_t q = 0; q * 1024 < T.span; q++, n++)
        if (q * 1024 + lane * 16 < T.span) glds16(g + q * 1024 + lane * 16, scratch);
    return n;
}

// ---- row windows -----------------------------------------------------------------
// NRA dwords of the row's fixed part (bitset + static region) realigned to
// the row start: r[j] = row bytes [4j, 4j + 4).  Wide layouts (more than
// MJ_WINMAX dwords) read each field on its own instead.
constexpr uint32_t NRA = (FIX + 3) / 4;
#ifndef MJ_PREFETCH
#define MJ_PREFETCH 0
#endif
#ifndef MJ_WINMAX
#define MJ_WINMAX 32
#endif
constexpr bool WIN = NRA <= MJ_WINMAX;
constexpr uint32_t NBW = (BS + 3) / 4;              // bitset dwords
// Extended window (round 6, narrow layouts with a utf8 column): the window
// also covers the first utf8 payload's length word and 8 string bytes (row
// bytes [0, FIX + 12)).  A row whose first utf8 column is not null has its
// payload right after the static region (write.rs:40-49: payloads in column
// order), so for such a row the length and a string of up to 8 bytes come out
// of the window's registers: two dependent LDS round trips per chunk fewer
// (length after window, string after the tile's prefix wait) and 6 instead of
// 9 strided dword reads per row on config B (each a 2-way bank conflict at
// its 18-B row stride).  Other rows (nulls, longer strings, later utf8
// columns) read the stage as before.  Measured (round 6, interleaved A/Bs on
// one box, config B): SQ_LDS_BANK_CONFLICT 31.2 M -> 20.8 M per dispatch and
// LDS instructions -21 %, but the kernel 0.7225 -> 0.7271 ms and 0.7141 ->
// 0.7178 ms (4 reps): neutral to 0.5 % slower (more SALU and VALU per chunk),
// so off by default (tuning: MURR_JIT_DEFS=MJ_XWIN=1; the GPU suite passed
// on it).  DESIGN.md §7.
#ifndef MJ_XWIN
#define MJ_XWIN 0
#endif
#ifndef MJ_XWMAX
#define MJ_XWMAX 12
#endif
// Ablations (tuning only): MJ_ABL_LDSX re-reads the window (read_window);
// MJ_ABL_LOADONLY skips the decode, so the decode waves only pass the tile
// barriers behind the loader (the production ring's own ceiling).
#ifndef MJ_ABL_LDSX
#define MJ_ABL_LDSX 0
#endif
#ifndef MJ_ABL_LOADONLY
#define MJ_ABL_LOADONLY 0
#endif
#ifndef MJ_FULLFAST
#define MJ_FULLFAST 0
#endif
constexpr uint32_t S0 = FIX + 4;         // row byte of the first payload's string (when it is first)
constexpr uint32_t NRX = S0 / 4 + 3;     // realigned dwords that hold row bytes [0, S0 + 8)
constexpr bool XW = MJ_XWIN && WIN && NUTF8 >= 1 && NRX <= MJ_XWMAX;
constexpr uint32_t NRW0 = WIN ? NRA : NBW;  // the fixed part's dwords (the window proper)
constexpr uint32_t NRW = XW ? NRX : NRW0;   // dwords kept per row
// row bytes the window must hold, and the aligned dwords that cover them at any shift
constexpr uint32_t NBYTES = XW ? S0 + 8 : 4 * NRW0;
constexpr uint32_t NRAW = (NBYTES + 3 + 3) / 4;

template <class Src> DEV void read_window(const Src& src, uint32_t ra, bool ok, uint32_t (&r)[NRW]) {
    // aligned dwords [ra & ~3, (ra & ~3) + 4 NRAW) cover the row's first
    // NBYTES bytes (with ok, every one of the window proper's holds a byte of
    // the row).  From HBM only the window proper (never past the row's own
    // dwords); the extension is a stage-only read (64 B of pad behind a tile).
    const uint32_t a4 = (Src::kHbm && !ok ? 0u : ra) >> 2, sh = ra & 3u;
    uint32_t w[NRAW];
#pragma unroll
    for (uint32_t j = 0; j < NRAW; j++) {
        if constexpr (Src::kHbm) {
            // the last dword only when the row reaches into it
            w[j] = j <= NRW0 && (j < NRW0 || sh) && ok ? src.w(a4 + j) : 0u;
        } else {
            w[j] = src.w(a4 + j);
        }
    }
#if MJ_ABL_LDSX
    // LDS sensitivity ablation (tuning only): every strided window dword read
    // a second time (volatile: neither merged nor dropped) and folded in with
    // a min of two equal values -- the window's bank conflicts and LDS cycles
    // doubled, both reads on the chain, the data and the rest of the tile
    // unchanged
    if constexpr (!Src::kHbm) {
        const volatile LAS uint32_t* vp = (const volatile LAS uint32_t*)src.s + a4;
#pragma unroll
        for (uint32_t j = 0; j < NRAW; j++) {
            const uint32_t x = vp[j];
            w[j] = w[j] < x ? w[j] : x;
        }
    }
#endif
#pragma unroll
    for (uint32_t j = 0; j < NRW; j++) r[j] = __builtin_amdgcn_alignbyte(j + 1 < NRAW ? w[j + 1] : 0u, w[j], sh);
}
// Field at compile-time row byte FO (realigned window).
template <uint32_t FO> DEV uint32_t get32(const uint32_t (&r)[NRW]) {
    if constexpr (FO % 4 == 0) return r[FO / 4];
    else return __builtin_amdgcn_alignbyte(r[FO / 4 + 1], r[FO / 4], FO % 4);
}
template <uint32_t FO> DEV uint32_t get16(const uint32_t (&r)[NRW]) {
    if constexpr (FO % 4 <= 2) return __builtin_amdgcn_ubfe(r[FO / 4], 8 * (FO % 4), 16);
    else return __builtin_amdgcn_alignbyte(r[FO / 4 + 1], r[FO / 4], 3) & 0xFFFFu;
}
template <uint32_t FO> DEV uint32_t get8(const uint32_t (&r)[NRW]) { return __builtin_amdgcn_ubfe(r[FO / 4], 8 * (FO % 4), 8); }

// Field of width W at row byte FO: from the window, or (wide layouts) read on
// its own from the source.
template <uint32_t W, uint32_t FO, class Src>
DEV void field(const Src& src, const uint32_t (&r)[NRW], uint32_t ra, bool ok, uint32_t& lo, uint32_t& hi) {
    if constexpr (WIN) {
        if constexpr (W == 8) { lo = get32<FO>(r); hi = get32<FO + 4>(r); }
        else if constexpr (W == 4) lo = get32<FO>(r);
        else if constexpr (W == 2) lo = get16<FO>(r);
        else lo = get8<FO>(r);
    } else {
        const uint32_t a = Src::kHbm && !ok ? 0u : ra + FO;
        if constexpr (Src::kHbm) {
            const GAS uint8_t* p = src.g + a;
            if constexpr (W == 8) { lo = *(const GAS u32u*)p; hi = *(const GAS u32u*)(p + 4); }
            else if constexpr (W == 4) lo = *(const GAS u32u*)p;
            else if constexpr (W == 2) lo = *(const GAS u16u*)p;
            else lo = *p;
        } else {
            if constexpr (W == 8) { lo = src.u32(a); hi = src.u32(a + 4); }
            else if constexpr (W == 4) lo = src.u32(a);
            else if constexpr (W == 2) lo = src.u32(a) & 0xFFFFu;
            else lo = src.u8(a);
        }
    }
}

// Ballot of `b` stashed in lane C % 64 of the pair (lo, hi) of lane group
// C / 64 (v_writelane with a compile-time lane).  The ballot's SGPRs come
// straight from a v_cmp: the nop covers the VALU-writes-SGPR ->
// v_writelane-reads-it hazard, which the compiler cannot see inside asm
// (without it the lane is written with a stale mask).
template <uint32_t C> DEV void stash(uint32_t (&lo)[NCW], uint32_t (&hi)[NCW], bool b) {
    const uint64_t m = __ballot(b);
    asm volatile("s_nop 4\n\tv_writelane_b32 %0, %2, %4\n\tv_writelane_b32 %1, %3, %4"
                 : "+v"(lo[C / 64]), "+v"(hi[C / 64])
                 : "s"((uint32_t)m), "s"((uint32_t)(m >> 32)), "i"(C % 64));
}
// Merged words: chunk k's ballot of word lane C into lane k * WL + C (k is a
// constant once the chunk loop is unrolled, but not a C++ constant, so the
// lane select goes through M0: an SGPR value and an SGPR lane select in one
// VOP3 would break the constant-bus limit).  M0 is saved and restored (the
// loader's LDS-DMA relies on it the same way); the nop covers both the
// SALU-writes-M0 and the VALU-writes-SGPR (ballot) hazards.
template <uint32_t C> DEV void stash_k(uint32_t& lo, uint32_t& hi, bool b, uint32_t k) {
    const uint64_t m = __ballot(b);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %5\n\ts_nop 4\n\tv_writelane_b32 %1, %3, m0\n\t"
                 "v_writelane_b32 %2, %4, m0\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep), "+v"(lo), "+v"(hi)
                 : "s"((uint32_t)m), "s"((uint32_t)(m >> 32)), "s"(k * WL + C));
}

// ---- per-wave state of a tile --------------------------------------------------
template <uint32_t R> struct Rows {
    uint32_t ra[R], rl[R];          // stage offset and length of the row (0 = missing / past the tile)
    uint32_t vb[R][NBW];            // valid bits (~bitset; 0 for a missing row)
    uint32_t r[R][NRW];             // realigned window
};

// Per-lane per-column state (lane c % 64 of group c / 64).
struct Lanes {
    uint64_t vptr[NCW], bptr[NCW];  // validity / bool values pointer of column c for the current block
    uint32_t proj[NCW];             // column c decoded (0/1)
    uint32_t isbool[NCW];
    uint32_t nacc[NCW];             // nulls of column c since the last flush
    uint32_t blk;                   // block the pointers belong to (~0 = none)
#if MJ_HOIST >= 2
    uint64_t optr[NCW], ocap[NCW];  // utf8 offsets pointer / values capacity of column c
#endif
};

DEV const Out* outs_of(uint32_t b) {
    const Out* o = args()->outs + (uint64_t)sgpr(b) * sgpr(args()->nproj);
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

// Column C's output descriptor for the current block from the lane table
// (v_readlane, no memory round trip; MJ_HOIST >= 2), or from memory.
template <uint32_t C> DEV Out lane_out(const Lanes& L, const Out* ob, uint32_t p) {
#if MJ_HOIST >= 2
    auto rl64 = [](uint64_t v) {
        // (readlane returns int: cast before widening, or the low word sign-extends)
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), C % 64) << 32) |
               (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, C % 64);
    };
    Out r;
    r.values = (uint8_t*)rl64(L.bptr[C / 64]);
    r.validity = nullptr;  // (validity words go through store_words)
    r.offsets = (int32_t*)rl64(L.optr[C / 64]);
    r.values_cap = rl64(L.ocap[C / 64]);
    return r;
#else
    return ldout(ob, p);
#endif
}

// Word lanes.  A chunk's validity words (and the bool columns' value words)
// go out as one wave store: lane c writes column c's validity word and, with
// MJ_FOLDB, lane NCOLS + c column c's bool value word (WL = 2 NCOLS word
// lanes when the layout has a bool column), instead of a second store for the
// bools.  A wave store instruction costs about the same whatever it writes
// (the store-shape probe: ~30 cycles of the CU's memory pipeline up to 256 B).
//
// Merged validity words (tiles of R > 1 chunks per wave, R x WL <= 64
// lanes): the words of all R chunks of a wave go out in ONE store -- lane
// k * WL + c holds chunk k's word c -- instead of one store per chunk (config
// B ablation, round 5: its two-lane validity store per chunk was 7.5 % of the
// kernel).  The per-lane tables then hold word lane (lane % WL).
template <uint32_t R> DEV constexpr bool merged_words() { return R > 1 && R * WL <= 64; }
// Lane `lane` of lane group j: its column c and whether it is a bool value
// word (bw); false for a lane with no word.
template <uint32_t R> DEV bool lane_word(uint32_t j, uint32_t lane, uint32_t& c, uint32_t& bw) {
    uint32_t x;
    if constexpr (merged_words<R>()) {
        if (lane >= R * WL) return false;
        x = lane % WL;
    } else if constexpr (FOLDB) {
        if (lane >= WL) return false;
        x = lane;
    } else {
        x = j * 64 + lane;
        if (x >= NCOLS) return false;
    }
    bw = x >= NCOLS;
    c = bw ? x - NCOLS : x;
    return true;
}

// Per-lane output pointers of block b (word lane c: column c's validity, or
// a bool column's values), reloaded when the block changes; null counts of
// the previous block flushed first.
template <uint32_t R> DEV void lanes_flush(Lanes& L, uint32_t lane) {
    if (L.blk == ~0u) return;
    unsigned long long* nulls = args()->nulls + (uint64_t)L.blk * args()->nproj;
#pragma unroll
    for (uint32_t j = 0; j < NCW; j++) {
        uint32_t c = 0, bw = 0;
        if (lane_word<R>(j, lane, c, bw) && L.proj[j] && L.nacc[j])  // (nacc stays 0 on bool value lanes)
            __hip_atomic_fetch_add(gp(nulls) + gp(args()->slot_tab)[c], (unsigned long long)L.nacc[j], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        L.nacc[j] = 0;
    }
}
template <uint32_t R> DEV void lanes_block(Lanes& L, uint32_t b, uint32_t lane) {
    if (L.blk == b) return;
    lanes_flush<R>(L, lane);
    L.blk = b;
    const Out* ob = outs_of(b);
#pragma unroll
    for (uint32_t j = 0; j < NCW; j++) {
        uint32_t c = 0, bw = 0;
        const bool ok = lane_word<R>(j, lane, c, bw);
        const uint32_t s = ok ? (uint32_t)gp(args()->slot_tab)[c] : (uint32_t)kNone;
        const bool isb = ok && kColW[ok ? c : 0] == 9;
        L.proj[j] = s != kNone && (!bw || isb);
        L.isbool[j] = isb && !bw;  // (a separate bool store: layouts without FOLDB)
        const GAS Out* o = (const GAS Out*)ob + (s != kNone ? s : 0u);
        L.vptr[j] = s != kNone ? (uint64_t)(bw ? (void*)o->values : (void*)o->validity) : 0;
        L.bptr[j] = s != kNone ? (uint64_t)o->values : 0;
#if MJ_HOIST >= 2
        L.optr[j] = s != kNone ? (uint64_t)o->offsets : 0;
        L.ocap[j] = s != kNone ? (uint64_t)o->values_cap : 0;
#endif
    }
    // Wait for these loads here, on the (rare) block-change path.  Left
    // pending, they make the compiler put a vmcnt(0) where this path rejoins
    // the tile loop -- every tile would then wait for all of the previous
    // tile's stores to be acknowledged.
    __builtin_amdgcn_s_waitcnt(0x0F70);
}

// Validity (and bool values) words of one chunk for every decoded column: one
// store per lane group, lane c writes word c.
template <uint32_t R>
DEV void store_words(Lanes& L, const uint32_t (&vlo)[NCW], const uint32_t (&vhi)[NCW], const uint32_t (&blo)[NCW],
                     const uint32_t (&bhi)[NCW], uint64_t word, uint32_t nk, uint32_t lane) {
#pragma unroll
    for (uint32_t j = 0; j < NCW; j++) {
        if (L.proj[j]) {
            const uint64_t v = ((uint64_t)vhi[j] << 32) | vlo[j];
            ostw(gp((uint64_t*)L.vptr[j]) + word, v);
            if constexpr (!FOLDB)
                if (L.isbool[j]) ostw(gp((uint64_t*)L.bptr[j]) + word, ((uint64_t)bhi[j] << 32) | blo[j]);
            if (!FOLDB || lane < NCOLS) L.nacc[j] += nk - (uint32_t)__popcll(v);
        }
    }
}
// The merged form: lane k * WL + c stores chunk k's word c.
DEV void store_words_merged(Lanes& L, uint32_t vlo, uint32_t vhi, uint64_t r0, uint32_t rbase, uint32_t nr,
                            uint32_t lane) {
    const uint32_t c0 = rbase + (lane / WL) * 64;
    const uint32_t nk = c0 < nr ? umin32(64u, nr - c0) : 0u;
    if (L.proj[0] && nk) {
        const uint64_t v = ((uint64_t)vhi << 32) | vlo, word = (r0 + c0) >> 6;
        ostw(gp((uint64_t*)L.vptr[0]) + word, v);
        if (lane % WL < NCOLS) L.nacc[0] += nk - (uint32_t)__popcll(v);
    }
}

// Copy one string from the stage to vb[0 .. n): overlapping unaligned stores
// of its own bytes (head and tail).  Returns the OR of its bytes (UTF-8
// pre-check).
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
                ostu<uint32_t>(vb, head);
                ostu<uint32_t>(vb + n - 4, tail);
                return head | tail;
            }
            if (n >= 2) {
                const uint32_t t2 = pick(w0, w1, w2, sh + n - 2) & 0xFFFFu;
                ostu<uint16_t>(vb, (uint16_t)head);
                ostu<uint16_t>(vb + n - 2, (uint16_t)t2);
                return (head & 0xFFFFu) | t2;
            }
            if (n == 1) {
                ostu<uint8_t>(vb, (uint8_t)head);
                return head & 0xFFu;
            }
            return 0u;
        }
        // 8-byte steps from realigned dword pairs, the last one overlapping;
        // two steps per iteration with their LDS reads issued together (one
        // LDS round trip per 16 bytes)
        uint32_t hib = 0;
        const uint32_t sh = pay & 3u;
        const LAS uint32_t* p = (const LAS uint32_t*)(src.s + (pay & ~3u));
#pragma unroll 1
        for (uint32_t q = 0;; q += 16) {
            const bool two = q + 8 < n;  // a second step in this iteration
            const uint32_t at0 = q + 8 <= n ? q : n - 8;
            const uint32_t at1 = q + 16 <= n ? q + 8 : n - 8;
            const uint32_t b0 = sh + at0, d0 = b0 >> 2, s0 = b0 & 3u;
            const uint32_t b1 = sh + at1, d1 = b1 >> 2, s1 = b1 & 3u;
            const uint32_t x0 = p[d0], x1 = p[d0 + 1], x2 = p[d0 + 2];
            const uint32_t y0 = p[d1], y1 = p[d1 + 1], y2 = p[d1 + 2];
            const uint32_t lo0 = __builtin_amdgcn_alignbyte(x1, x0, s0), hi0 = __builtin_amdgcn_alignbyte(x2, x1, s0);
            const uint32_t lo1 = __builtin_amdgcn_alignbyte(y1, y0, s1), hi1 = __builtin_amdgcn_alignbyte(y2, y1, s1);
            ostu<uint64_t>(vb + at0, ((uint64_t)hi0 << 32) | lo0);
            hib |= lo0 | hi0;
            if (two) {
                ostu<uint64_t>(vb + at1, ((uint64_t)hi1 << 32) | lo1);
                hib |= lo1 | hi1;
            }
            if (q + 16 >= n) break;
        }
        return hib;
    }
    uint32_t hib = 0, q = 0;
    if (n >= 4) {
#pragma unroll 1
        for (; q + 4 <= n; q += 4) {
            const uint32_t v = src.u32(pay + q);
            ostu<uint32_t>(vb + q, v);
            hib |= v;
        }
        if (q < n) {
            const uint32_t v = src.u32(pay + n - 4);
            ostu<uint32_t>(vb + n - 4, v);
            hib |= v;
        }
    } else {
        for (; q < n; q++) {
            const uint32_t v = src.u8(pay + q);
            ostu<uint8_t>(vb + q, (uint8_t)v);
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

// Exact error of a flagged row: the first projected column (projection order)
// whose cell the reference would reject (read.rs:39-55 bounds).
template <class Src>
DEV void report_row(const Src& src, uint32_t ra, uint32_t rl, uint64_t b, uint64_t row, unsigned long long* err) {
    if (rl < BS) { report(err, err_key(b, row, 0, kStMalformed)); return; }
    const uint32_t np = args()->nproj;
    for (uint32_t p = 0; p < np; p++) {
        const uint32_t c = gp(args()->projcols)[p];
        const uint32_t fo = kColFo[c], wid = kColW[c] == 9 ? 1u : kColW[c];
        if ((src.u8(ra + (c >> 3)) >> (c & 7)) & 1) continue;
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

// ---- decoupled look-back (stream mode) -----------------------------------------
// Granule = status (2 bits: 0 none, 1 aggregate, 2 inclusive prefix) | value.
constexpr uint64_t kAgg = 1ull << 62, kPre = 2ull << 62, kValMask = (1ull << 62) - 1;
DEV void publish(unsigned long long* g, uint64_t v) {
    __hip_atomic_store((GAS unsigned long long*)g, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV uint64_t peek(const unsigned long long* g) {
    return __hip_atomic_load((const GAS unsigned long long*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Exclusive prefix of segment t (first segment of its block t0) for utf8
// column u: 512 predecessors per round (8 per lane, lane l holds t-1-8l-q),
// newest first, summed back to the nearest inclusive prefix (or the block's
// first segment).  The segments of one round of the grid all publish their
// aggregates at about the same time, so one round usually ends at the
// previous round's prefixes.
constexpr uint32_t kLbPer = 8;
DEV uint64_t look_back(uint64_t t, uint64_t t0, uint32_t u, uint32_t lane, uint64_t b) {
    const unsigned long long* fl = args()->flags;
    uint64_t sum = 0;
    uint64_t j = t;  // segments [t0, j) remain
    Wait w;
    while (j > t0) {
        uint64_t g[kLbPer];
        bool in[kLbPer];
#pragma unroll
        for (uint32_t q = 0; q < kLbPer; q++) {
            const uint64_t back = 1 + kLbPer * lane + q;  // segment j - back
            in[q] = j >= t0 + back;
            g[q] = in[q] ? peek(fl + (j - back) * NU + u) : kPre;  // past the block: prefix 0
        }
        // predecessors with nothing published yet: re-read (bounded)
        for (;;) {
            bool pend = false;
#pragma unroll
            for (uint32_t q = 0; q < kLbPer; q++) pend |= in[q] && (g[q] >> 62) == 0;
            if (!__ballot(pend)) break;
            if (w.expired(b, 0)) return sum;
#pragma unroll
            for (uint32_t q = 0; q < kLbPer; q++)
                if (in[q] && (g[q] >> 62) == 0) g[q] = peek(fl + (j - 1 - kLbPer * lane - q) * NU + u);
        }
        // the nearest prefix: lowest lane holding one, lowest q in it
        uint32_t qp = kLbPer;
#pragma unroll
        for (uint32_t q = kLbPer; q-- > 0;)
            if ((g[q] >> 62) == 2) qp = q;
        const uint64_t pm = __ballot(qp < kLbPer);
        const uint32_t stop = pm ? (uint32_t)__builtin_ctzll(pm) : 64u;
        const uint32_t qstop = __builtin_amdgcn_readlane(qp, stop < 64 ? stop : 0);
        uint64_t v = 0;
#pragma unroll
        for (uint32_t q = 0; q < kLbPer; q++) {
            const bool take = in[q] && (lane < stop || (lane == stop && q <= qstop));
            v += take ? (g[q] & kValMask) : 0;
        }
        for (int m = 32; m >= 1; m >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, m, 64);
        sum += sgpr64(v);
        if (pm) break;
        j = j > 64 * kLbPer ? j - 64 * kLbPer : 0;
    }
    return sum;
}

// ---- one tile of one decode wave ---------------------------------------------------
// PH 0: everything (local mode); 1: first pass of a split segment (fixed
// columns, validity, utf8 lengths); 2: second pass (utf8 offsets and bytes).
// Early release (ER, local mode): the ring slot is handed back (`rel`, an LDS
// counter the loader polls) as soon as this wave holds in registers all it
// still needs of the tile -- its row windows, and each utf8 cell's string
// bytes when the cell is at most 8 bytes, with their OR for the UTF-8 check --
// so the loader refills the slot while the wave computes and stores.  A wave
// that would still read the slot (a longer string, a byte >= 0x80 to check,
// a malformed row, a layout whose fields are not all in the window) hands it
// back at the end of the tile instead.
DEV void release_slot(LAS uint32_t* rel, uint32_t lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot have returned
    if (lane == 0) __hip_atomic_fetch_add(rel, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The n <= 8 case of copy_str from the string's three aligned dwords in registers.
DEV void copy_str_regs(GAS uint8_t* vb, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t sh, uint32_t n) {
    const uint32_t head = __builtin_amdgcn_alignbyte(w1, w0, sh);
    if (n >= 4) {
        ostu<uint32_t>(vb, head);
        ostu<uint32_t>(vb + n - 4, pick(w0, w1, w2, sh + n - 4));
    } else if (n >= 2) {
        ostu<uint16_t>(vb, (uint16_t)head);
        ostu<uint16_t>(vb + n - 2, (uint16_t)(pick(w0, w1, w2, sh + n - 2) & 0xFFFFu));
    } else if (n == 1) {
        ostu<uint8_t>(vb, (uint8_t)head);
    }
}
// OR of a string's bytes (n <= 8) from its three aligned dwords (copy_str's return value).
DEV uint32_t hib_regs(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t sh, uint32_t n) {
    const uint32_t head = __builtin_amdgcn_alignbyte(w1, w0, sh);
    if (n >= 4) return head | pick(w0, w1, w2, sh + n - 4);
    if (n >= 2) return (head & 0xFFFFu) | (pick(w0, w1, w2, sh + n - 2) & 0xFFFFu);
    return n == 1 ? head & 0xFFu : 0u;
}

// Column C's fixed-width value of chunk k (width WW at row byte FO), 0 for a
// null or short cell; a valid cell the row is too short for is flagged in badk
// (primitive.rs:43-56: a null reads as the default value).
template <uint32_t C, uint32_t WW, uint32_t FO, class Src, uint32_t R>
DEV uint32_t fixed_val(const Src& src, const Rows<R>& W, uint32_t k, bool safe, uint32_t& badk, uint32_t& hi) {
    bool valid = (W.vb[k][C / 32] >> (C % 32)) & 1u;
    if (safe) {
        const bool have = FO + WW <= W.rl[k];
        badk |= (uint32_t)(valid && !have) << k;
        valid = valid && have;
    }
    uint32_t lo = 0;
    hi = 0;
    field<WW, FO>(src, W.r[k], W.ra[k], valid || !Src::kHbm, lo, hi);
    const uint32_t m = valid ? ~0u : 0u;
    hi &= m;
    return lo & m;
}

template <class SH, uint32_t PH, class Src, bool ER = false>
DEV void decode_tile(const Src& src, const Tile& T, const LAS uint32_t* ro, LAS uint8_t* ctl, uint64_t (&run)[NU],
                     Lanes& L, uint32_t wave, uint32_t lane, uint32_t it, LAS uint32_t* rel = nullptr) {
    constexpr uint32_t R = SH::R, NC = SH::NC;
    unsigned long long* err = args()->err;
    const uint32_t rbase = wave * 64 * R;
    const uint32_t abase = (uint32_t)T.abase;
    const Out* ob = outs_of(T.b);
    LAS uint32_t* pcnt = (LAS uint32_t*)ctl;         // wave totals published (monotone)
    LAS uint32_t* pready = (LAS uint32_t*)ctl + 1;   // segments whose prefix is in tpre (split mode)
    LAS uint64_t* tpre = (LAS uint64_t*)(ctl + SH::CNT_B);
    // wave totals of this tile: one buffer per tile parity (with early
    // release a wave may publish tile it+1's totals while another still reads
    // tile it's; it cannot get further ahead, since tile it+1's prefix wait
    // needs every wave's tile it+1 totals)
    LAS uint32_t* wt = (LAS uint32_t*)(ctl + SH::CNT_B + 8 * NU) + (it & 1) * NU * NC;
    lanes_block<R>(L, T.b, lane);
    constexpr bool MV = merged_words<R>();
#define MJ_STASH(C, LO, HI, K, B)                        \
    do {                                                 \
        if constexpr (MV) stash_k<C>(LO[0][0], HI[0][0], (B), (K)); \
        else stash<C>(LO[K], HI[K], (B));               \
    } while (0)
    // a bool column's value word: word lane NCOLS + C of the validity store
#define MJ_STASHB(C, K, B)                                                   \
    do {                                                                     \
        if constexpr (FOLDB) MJ_STASH(NCOLS + C, vlo, vhi, K, B);            \
        else MJ_STASH(C, blo, bhi, K, B);                                    \
    } while (0)
#if MJ_HOIST
    // the projection's slot words, once per tile (one batched scalar load;
    // slot_of would wait on a kernel-argument load per use)
    uint32_t slw[(NCOLS + 1) / 2];
    {
        const CAS uint32_t* w = (const CAS uint32_t*)args()->slot;
#pragma unroll
        for (uint32_t j = 0; j < (NCOLS + 1) / 2; j++) slw[j] = w[j];
    }
#define MJ_SLOT(C) ((slw[(C) >> 1] >> (16 * ((C) & 1))) & 0xFFFFu)
#else
#define MJ_SLOT(C) slot_of(C)
#endif

    Rows<R> W;
    uint32_t badk = 0, partial = 0;
    // MJ_FULLFAST (tuning A/B): a chunk whose 64 rows are all in the tile
    // (wave-uniform) stores without the per-lane row guard, so no exec-mask
    // save / restore per column and chunk
    bool fullk[R];
#pragma unroll
    for (uint32_t k = 0; k < R; k++) fullk[k] = rbase + (k + 1) * 64 <= T.nr;
#define MJ_IFROW(K, I, ...)                                   \
    do {                                                      \
        if (MJ_FULLFAST && fullk[K]) { __VA_ARGS__ }          \
        else if ((I) < T.nr) { __VA_ARGS__ }                  \
    } while (0)
#pragma unroll
    for (uint32_t k = 0; k < R; k++) {
        const uint32_t i = rbase + k * 64 + lane;
        const uint32_t a0 = ro[i], a1 = ro[i + 1];
        const uint32_t rl = i < T.nr ? a1 - a0 : 0u;
        W.ra[k] = a0 - abase;
        W.rl[k] = rl;
        const bool full = rl >= FIX;
        partial |= (uint32_t)(rl != 0 && !full) << k;
        read_window(src, W.ra[k], full, W.r[k]);
        if (!full) {
            // a short row: only the bytes it has (the cold path reports it)
#pragma unroll
            for (uint32_t j = 0; j < NRW; j++) {
                const uint32_t have = rl > 4 * j ? umin32(rl - 4 * j, 4u) : 0u;
                uint32_t v = 0;
                if (!Src::kHbm || have) {
                    for (uint32_t q = 0; q < have; q++) v |= src.u8(W.ra[k] + 4 * j + q) << (8 * q);
                }
                W.r[k][j] = v;
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < NBW; j++) {
            uint32_t bits = W.r[k][j];
            if (BS - 4 * j < 4) bits |= ~0u << (8 * (BS - 4 * j));  // padding bytes read as null
            W.vb[k][j] = rl >= BS ? ~bits : 0u;
        }
        badk |= (uint32_t)(rl != 0 && rl < BS) << k;
    }
    const bool safe = __ballot(partial != 0) != 0;  // some row shorter than the fixed part

    uint32_t vlo[R][NCW], vhi[R][NCW], blo[R][NCW], bhi[R][NCW];
#pragma unroll
    for (uint32_t k = 0; k < R; k++)
#pragma unroll
        for (uint32_t j = 0; j < NCW; j++) vlo[k][j] = vhi[k][j] = blo[k][j] = bhi[k][j] = 0;

    // ---- utf8 cells: payload position and length, chunk scans (read.rs:45-55)
    uint32_t upay[NU][R], ulen[NU][R], uinc[NU][R], utot[NU];
#pragma unroll
    for (uint32_t u = 0; u < NU; u++) utot[u] = 0;
    // extended window (XW): bit k = this lane's first utf8 payload sits right
    // after the static region, so its length and first 8 bytes are in W.r[k]
    constexpr bool XWS = XW && !Src::kHbm;
    uint32_t xin = 0;
#define MJ_U(C, W_, FO, U)                                                                              \
    if constexpr (W_ == 0) {                                                                            \
        if (MJ_SLOT(C) != kNone) {                                                                      \
            uint32_t wtot = 0;                                                                          \
            _Pragma("unroll") for (uint32_t k = 0; k < R; k++) {                                        \
                const uint32_t rl = W.rl[k];                                                            \
                const bool valid = (W.vb[k][C / 32] >> (C % 32)) & 1u;                                  \
                const bool s_ok = valid && FO + 4 <= rl;                                                \
                uint32_t sl, dummy = 0;                                                                 \
                field<4, FO>(src, W.r[k], W.ra[k], s_ok, sl, dummy);                                    \
                const uint32_t vlen = rl - BS; /* >= 4 when s_ok */                                     \
                const bool p_ok = s_ok && sl <= vlen - 4;                                               \
                const uint32_t pa = W.ra[k] + BS + sl;                                                  \
                uint32_t l;                                                                             \
                if constexpr (XWS && U == 0) {                                                          \
                    const bool xf = sl == FIX - BS; /* the first payload: in the window */              \
                    xin |= (uint32_t)xf << k;                                                           \
                    l = get32<FIX>(W.r[k]);                                                             \
                    if (s_ok && !xf) l = src.u32(pa);                                                   \
                } else {                                                                                \
                    l = src.u32(Src::kHbm && !p_ok ? 0u : pa);                                          \
                }                                                                                       \
                const bool good = p_ok && l <= vlen - 4 - sl;                                           \
                badk |= (uint32_t)(valid && !good) << k;                                                \
                upay[U][k] = pa + 4;                                                                    \
                ulen[U][k] = good ? l : 0u;                                                             \
                uinc[U][k] = wave_scan(ulen[U][k]) + wtot;                                              \
                wtot = (uint32_t)__builtin_amdgcn_readlane(uinc[U][k], 63);                                       \
                if constexpr (PH != 2) MJ_STASH(C, vlo, vhi, k, valid);                                 \
            }                                                                                           \
            utot[U] = wtot;                                                                             \
        }                                                                                               \
    }
    MJ_COLS(MJ_U)
#undef MJ_U

    // early release: strings of <= 8 bytes into registers, then the slot back
    constexpr bool ERS = ER && PH == 0 && !Src::kHbm;  // (a tile decoded from HBM: its slot held only offsets)
    uint32_t sw[NU][R][3], shib[NU][R];
    bool late = false;
    if constexpr (ER && PH == 0) {
        if constexpr (Src::kHbm) {
            release_slot(rel, lane);
        } else {
            bool lng = false;
            uint32_t hi = 0;
#pragma unroll
            for (uint32_t u = 0; u < NU; u++)
#pragma unroll
                for (uint32_t k = 0; k < R; k++) sw[u][k][0] = sw[u][k][1] = sw[u][k][2] = shib[u][k] = 0;
#define MJ_P(C, W_, FO, U)                                                                              \
            if constexpr (W_ == 0) {                                                                    \
                if (MJ_SLOT(C) != kNone) {                                                              \
                    _Pragma("unroll") for (uint32_t k = 0; k < R; k++) {                                \
                        const uint32_t n = ulen[U][k], pay = upay[U][k];                                \
                        if (n > 8) lng = true;                                                          \
                        if (n && n <= 8) {                                                              \
                            src.win3(pay, sw[U][k][0], sw[U][k][1], sw[U][k][2]);                       \
                            shib[U][k] = hib_regs(sw[U][k][0], sw[U][k][1], sw[U][k][2], pay & 3u, n);  \
                            hi |= shib[U][k];                                                           \
                        }                                                                               \
                    }                                                                                   \
                }                                                                                       \
            }
            MJ_COLS(MJ_P)
#undef MJ_P
            late = !WIN || __ballot(lng || (hi & 0x80808080u) || badk || partial) != 0;
            if (!late) release_slot(rel, lane);
        }
    }
    (void)sw;
    (void)shib;

    // wave totals -> LDS; the tile total and every wave's prefix follow
    if (NUTF8) {
        if (lane == 0) {
            for (uint32_t u = 0; u < NU; u++) wt[u * NC + wave] = utot[u];
            __hip_atomic_fetch_add(pcnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }

    // ---- fixed-width and bool columns (primitive.rs:43-56, bool_.rs:86-99)
#define MJ_F(C, W_, FO, U)                                                                              \
    if constexpr (W_ != 0 && PH != 2) {                                                                 \
        if (MJ_SLOT(C) != kNone) {                                                                      \
            constexpr uint32_t WW = W_ == 9 ? 1u : W_;                                                  \
            const Out o = lane_out<C>(L, ob, MJ_SLOT(C));                                               \
            _Pragma("unroll") for (uint32_t k = 0; k < R; k++) {                                        \
                const uint32_t i = rbase + k * 64 + lane;                                               \
                uint32_t hi = 0;                                                                        \
                const uint32_t lo = fixed_val<C, WW, FO>(src, W, k, safe, badk, hi);                    \
                MJ_STASH(C, vlo, vhi, k, (W.vb[k][C / 32] >> (C % 32)) & 1u);                           \
                if constexpr (W_ == 9) {                                                                \
                    MJ_STASHB(C, k, lo != 0);                                                           \
                } else if (!MJ_ABL_NOFIX) {                                                             \
                    const uint64_t row = T.r0 + i;                                                      \
                    MJ_IFROW(k, i, {                                                                    \
                        if constexpr (W_ == 8) ost(gp((uint64_t*)o.values) + row, ((uint64_t)hi << 32) | lo); \
                        else if constexpr (W_ == 4) ost(gp((uint32_t*)o.values) + row, lo);             \
                        else if constexpr (W_ == 2) ost(gp((uint16_t*)o.values) + row, (uint16_t)lo);   \
                        else if constexpr (MJ_OUT_NT_W1) ost(gp((uint8_t*)o.values) + row, (uint8_t)lo); \
                        else gp((uint8_t*)o.values)[row] = (uint8_t)lo;                                 \
                    });                                                                                 \
                }                                                                                       \
            }                                                                                           \
        }                                                                                               \
    }
    MJ_COLS(MJ_F)
#undef MJ_F

    if constexpr (PH != 2 && MV) {
        store_words_merged(L, vlo[0][0], vhi[0][0], T.r0, rbase, T.nr, lane);
    } else if constexpr (PH != 2) {
#pragma unroll
        for (uint32_t k = 0; k < R; k++) {
            const uint32_t c0 = rbase + k * 64;
            const uint32_t nk = c0 < T.nr ? umin32(64u, T.nr - c0) : 0u;
            if (nk) store_words<R>(L, vlo[k], vhi[k], blo[k], bhi[k], (T.r0 + c0) >> 6, nk, lane);
        }
    }
#undef MJ_STASHB
#undef MJ_STASH

    if (PH != 2 && args()->report && __ballot(badk != 0)) {  // cold: exact error reports
#pragma unroll
        for (uint32_t k = 0; k < R; k++) {
            if (!((badk >> k) & 1)) continue;
            const uint32_t i = rbase + k * 64 + lane;
            report_row(src, W.ra[k], W.rl[k], T.b, T.r0 + i, err);
        }
    }
    if (!NUTF8) {
        if (ERS && late) release_slot(rel, lane);
        return;
    }

    // ---- the tile's utf8 prefix
    {
        MJ_TIC
        Wait w;
        while (__hip_atomic_load(pcnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < NC * (it + 1))
            if (w.expired(T.b, T.r0)) break;
        MJ_TOC(1)
    }
    uint64_t tot[NU], before[NU];
#pragma unroll
    for (uint32_t u = 0; u < NU; u++) {
        uint64_t bf = 0, all = 0;
#pragma unroll
        for (uint32_t w = 0; w < NC; w++) {
            const uint32_t v = wt[u * NC + w];
            bf += w < wave ? v : 0u;
            all += v;
        }
        tot[u] = sgpr64(all);
        before[u] = sgpr64(bf);
    }
    uint64_t tile_pre[NU];
    if constexpr (PH == 0) {
#pragma unroll
        for (uint32_t u = 0; u < NU; u++) {
            tile_pre[u] = run[u];
            run[u] += tot[u];
        }
    } else if constexpr (PH == 1) {
        // the segment's utf8 bytes; after its last tile, wave 0 publishes the
        // aggregate, looks back, publishes the inclusive prefix and leaves the
        // exclusive one in LDS for the second pass
#pragma unroll
        for (uint32_t u = 0; u < NU; u++) run[u] = (T.seg_first ? 0 : run[u]) + tot[u];
        if (T.seg_last && wave == 0 && args()->emit) {
            unsigned long long* fl = args()->flags + T.t * NU;
            const bool head = T.t == T.first_seg;
#pragma unroll
            for (uint32_t u = 0; u < NU; u++)
                if (lane == 0) publish(fl + u, (head ? kPre : kAgg) | run[u]);
#pragma unroll
            for (uint32_t u = 0; u < NU; u++) {
                MJ_TIC
                const uint64_t ex = head ? 0 : look_back(T.t, T.first_seg, u, lane, T.b);
                MJ_TOC(3)
                if (!head && lane == 0) publish(fl + u, kPre | ((ex + run[u]) & kValMask));
                if (lane == 0) tpre[u] = ex;
            }
            if (lane == 0) __hip_atomic_store(pready, (uint32_t)T.t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return;
    } else {
        if (T.seg_first) {
            MJ_TIC
            Wait w;
            while (__hip_atomic_load(pready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != (uint32_t)T.t + 1)
                if (w.expired(T.b, T.r0)) break;
            MJ_TOC(2)
#pragma unroll
            for (uint32_t u = 0; u < NU; u++) run[u] = sgpr64(tpre[u]);
        }
#pragma unroll
        for (uint32_t u = 0; u < NU; u++) {
            tile_pre[u] = run[u];
            run[u] += tot[u];
        }
    }

    // ---- offsets and string bytes (utf8.rs:86-96 append_value)
#define MJ_E(C, W_, FO, U)                                                                              \
    if constexpr (W_ == 0 && PH != 1) {                                                                 \
        if (MJ_SLOT(C) != kNone) {                                                                      \
            const uint32_t P = MJ_SLOT(C);                                                              \
            const Out o = lane_out<C>(L, ob, P);                                                        \
            const uint64_t base = tile_pre[U] + before[U];                                              \
            if (T.first && wave == 0 && lane == 0) gp(o.offsets)[0] = 0;                                \
            if (T.last && wave == 0 && lane == 0)                                                       \
                __hip_atomic_store(gp(args()->lens) + (uint64_t)T.b * args()->nproj + P,             \
                                   (unsigned long long)(tile_pre[U] + tot[U]), __ATOMIC_RELAXED,        \
                                   __HIP_MEMORY_SCOPE_AGENT); /* write-through: read by the epilogue */ \
            GAS int32_t* obf = gp(o.offsets) + T.r0 + 1;                                                \
            _Pragma("unroll") for (uint32_t k = 0; k < R; k++) {                                        \
                const uint32_t i = rbase + k * 64 + lane;                                               \
                const bool act = i < T.nr;                                                              \
                const uint32_t n = ulen[U][k];                                                          \
                const uint64_t e = base + uinc[U][k];                                                   \
                const uint64_t cend = base + (uint32_t)__builtin_amdgcn_readlane(uinc[U][k], 63);                 \
                uint32_t hib = 0;                                                                       \
                const bool regs = ERS && !late; /* the bytes are in sw (the slot is gone) */            \
                /* XW: the string is in the window's registers (row bytes S0 ..) */                    \
                const bool inw = XWS && U == 0 && ((xin >> k) & 1u) && n <= 8;                          \
                if (cend <= 0x7FFFFFFFull && cend <= o.values_cap) { /* wave-uniform fast path */       \
                    MJ_IFROW(k, i, { ost(obf + i, (int32_t)e); });                                     \
                    if (regs) {                                                                         \
                        if (n && !MJ_ABL_NOSTR)                                                         \
                            copy_str_regs(gp(o.values) + (e - n), sw[U][k][0], sw[U][k][1], sw[U][k][2], \
                                          upay[U][k] & 3u, n);                                          \
                        hib = shib[U][k];                                                               \
                    } else if (inw) {                                                                   \
                        const uint32_t x0 = W.r[k][XW ? S0 / 4 : 0], x1 = W.r[k][XW ? S0 / 4 + 1 : 0];  \
                        const uint32_t x2 = W.r[k][XW ? S0 / 4 + 2 : 0];                                \
                        if (!MJ_ABL_NOSTR) copy_str_regs(gp(o.values) + (e - n), x0, x1, x2, S0 % 4, n); \
                        hib = hib_regs(x0, x1, x2, S0 % 4, n);                                          \
                    } else if (n && !MJ_ABL_NOSTR) {                                                    \
                        hib = copy_str(src, gp(o.values) + (e - n), upay[U][k], n);                     \
                    }                                                                                   \
                } else {                                                                                \
                    if (act) {                                                                          \
                        if (e > 0x7FFFFFFFull) report(err, err_key(T.b, T.r0 + i, P, kStOverflow));     \
                        else obf[i] = (int32_t)e;                                                       \
                        if (n && e > o.values_cap) report(err, err_key(T.b, T.r0 + i, P, kStCapacity)); \
                    }                                                                                   \
                    if (regs) hib = shib[U][k];                                                         \
                    else for (uint32_t q = 0; q < n; q++) hib |= src.u8(upay[U][k] + q);                \
                }                                                                                       \
                if ((hib & 0x80808080u) && !utf8_valid_slow(src, upay[U][k], n)) /* (never when regs) */ \
                    report(err, err_key(T.b, T.r0 + i, P, kStUtf8));                                    \
            }                                                                                           \
        }                                                                                               \
    }
    MJ_COLS(MJ_E)
#undef MJ_E
#undef MJ_SLOT
#undef MJ_IFROW
    if (ERS && late) release_slot(rel, lane);
}

// ---- read-back epilogue (prepared launches) ---------------------------------------
// The counters (error word, null counts, utf8 byte totals) are written only by
// agent-scope atomics and write-through stores, so once every workgroup has
// drained them the last one to finish can hand them to the host: each decode
// wave waits for its own memory operations, the workgroup's last decode wave
// (an LDS count) takes a ticket, and the workgroup holding the last ticket
// copies the counters into pinned host memory and then sets the done flag the
// host polls.  Replaces the read-back copy and the stream synchronisation of
// a run (MI355X_MICROARCH.md, inter-workgroup visibility: one agent-scope add
// per storing workgroup after its waits; the last adder reads).  Relaxed
// atomics throughout: everything handed over is already coherent (atomics,
// write-through stores), and a release / acquire here would write back and
// invalidate the L2 at the end of every workgroup.
template <uint32_t NC> DEV void epilogue(LAS uint8_t* ctl, uint32_t lane) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // this wave's stores and atomics landed
    uint32_t last = 0;
    if (lane == 0)
        last = __hip_atomic_fetch_add((LAS uint32_t*)ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == NC - 1;
    if (!__builtin_amdgcn_readfirstlane(last)) return;
    uint32_t t = 0;
    if (lane == 0)
        t = __hip_atomic_fetch_add(gp(args()->ticket), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_amdgcn_readfirstlane(t) != gridDim.x - 1) return;
    const uint32_t words = args()->rb_words;
    const GAS unsigned long long* __restrict__ src = (const GAS unsigned long long*)args()->err;
    GAS unsigned long long* __restrict__ dst = gp(args()->rb_host);
    for (uint32_t base = 0; base < words; base += 64 * 8) {
        unsigned long long v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            const uint32_t i = base + 64 * k + lane;
            v[k] = i < words ? __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        }
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            const uint32_t i = base + 64 * k + lane;
            if (i < words) dst[i] = v[k];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(dst + words, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- kernel body ---------------------------------------------------------------------
// MODE 0: local, 1: split (separate kernels: the split path's look-back
// registers would otherwise cost the local kernel occupancy).
template <uint32_t NW, uint32_t R, uint32_t NS, uint32_t MODE>
DEV void kernel_body() {
    using SH = Shape<NW, R, NS>;
    constexpr uint32_t NC = SH::NC, TR = SH::TR, NSLOT = SH::NSLOT;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_[];
    LAS uint8_t* lds = (LAS uint8_t*)lds_;
    const uint32_t lane = lane_id();
    const uint32_t wave = sgpr(threadIdx.x >> 6);
    const uint32_t stage = sgpr(args()->stage);
    const uint32_t SLOT = SH::slot_bytes(stage);
    LAS uint8_t* spans = lds + NSLOT * SLOT;
    LAS uint8_t* infos = spans + SH::SPAN_B;
    LAS uint8_t* ctl = infos + SH::INFO_B;
    LAS uint8_t* pf = ctl + SH::CNT_B + 8 * NU + ((8 * NU * NC + 15) & ~15u);
    if (threadIdx.x < 8) ((LAS uint32_t*)ctl)[threadIdx.x] = 0;
    // early release (local mode): slots handed over by LDS counters instead of
    // a workgroup barrier per tile
    constexpr bool ER = MODE == 0 && MJ_ER && NSLOT == 2;
    constexpr bool FAST = MJ_FASTSTART && NSLOT == 2;
    LAS uint32_t* full = (LAS uint32_t*)ctl + 4;  // [2]: number + 1 of the tile landed in slot s
    LAS uint32_t* freec = full + 2;               // [2]: decode-wave releases of slot s (cumulative)
    // A prepared launch (murr_decode_run) alternates two counter sets: this
    // launch counts into one and zeroes the other for the next run, so a run
    // needs no memset of its own.
    if (blockIdx.x == 0 && args()->zero_next) {
        GAS unsigned int* z = gp(args()->zero_next);
        for (uint32_t i = threadIdx.x; i < args()->zero_words; i += blockDim.x) z[i] = 0u;
    }

    if (wave == NC) {
        // (MJ_LOADER_PRIO: the loader wave's issue priority, s_setprio 0-3;
        // tuning)
        if constexpr (MJ_LOADER_PRIO > 0) __builtin_amdgcn_s_setprio(MJ_LOADER_PRIO);
        // ---- loader: NSLOT - 1 tiles in flight.  At iteration i (after
        // barrier B_i freed the slot of tile i - 1) it DMAs tile i + NSLOT - 1
        // and announces tile i + NSLOT + 2 (its identity and span), then waits
        // for tile i + 1.  It issues no other vector-memory instruction, so
        // its counted vmcnt waits for exactly the DMA it needs.
        // Fast start for cut and split launches only (args.fast): with many
        // short virtual blocks per workgroup it took the D shard 0.0866 ->
        // 0.0852 ms, while whole-block launches (config B) ran 0.758 -> 0.771.
        const bool fast = ER ? FAST : FAST && args()->fast != 0;
        if (fast && !(MODE == 1 && seg_claims())) warm_scalar<MODE>();  // (claimed segments: unknown yet)
        Cur cs = cur_first<MODE>();  // next tile to announce
        // tiles announced before the first DMA: 0 .. 3, or (fast start) 0 .. 1 / 0
        constexpr uint32_t NPRE_ER = FAST ? 1u : NSLOT + 1;
        const uint32_t npre = ER ? NPRE_ER : fast ? 0u : NSLOT + 1;
#pragma unroll
        for (uint32_t k = 0; k <= NSLOT + 1; k++) {
            if (k > npre) break;
            tile_announce<TR>(cs, spans + (k & 7) * 16, infos + (k & 7) * 32, lane, pf + (k & 7) * 8 * NU);
            cs = cur_next<TR>(cs);
        }
#ifdef MJ_STAMPS
        const uint64_t lt0 = __builtin_amdgcn_s_memtime();
        uint64_t lwait = 0, lvm = 0;  // loader waits: all / the vmcnt part (slot 10)
#endif
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if constexpr (ER) {
            // Up to two tiles in flight: tile t goes into slot t % 2 once every
            // decode wave has released tile t - 2 from it (freec), lands, and
            // is published (full).  Between those steps the loader waits only
            // on its own counted vmcnt and polls one LDS word, never on a
            // barrier, so a slot is refilled while the decode waves are still
            // computing and storing the tile it held.
            lds_barrier();  // B_0: counters zeroed, tiles 0 .. 3 (FAST: 0 .. 1) announced
            uint32_t ti = 0, tl = 0;        // next tile to DMA / to land
            uint32_t ops[2] = {0, 0}, ann[2] = {0, 0};  // vmem ops issued with tile j % 2: all, its announce part
            if constexpr (FAST) {
                // Fast start: tiles 0 and 1 go into their slots as soon as
                // their spans are in, and tiles 2 and 3 are announced behind
                // those DMAs.  Their spans are younger than tile 1's DMA, so
                // tile 1 lands with a full wait (ann[1] = 0), and tiles 2 and 3
                // are not issued before it has.
                uint32_t nd1 = 0;
                if (tile_valid(infos)) {
                    tile_dma<TR, SH::RO_BYTES>(tile_read_ptrs(spans, infos, stage), lds, lane);
                    ti = 1;
                    if (tile_valid(infos + 32)) {
                        nd1 = tile_dma<TR, SH::RO_BYTES>(tile_read_ptrs(spans + 16, infos + 32, stage), lds + SLOT, lane);
                        ti = 2;
                    }
                }
                uint32_t na = 0;
#pragma unroll
                for (uint32_t k = 2; k <= NSLOT + 1; k++) {
                    na += tile_announce<TR>(cs, spans + (k & 7) * 16, infos + (k & 7) * 32, lane, pf + (k & 7) * 8 * NU);
                    cs = cur_next<TR>(cs);
                }
                ops[1] = nd1 + na;  // landing tile 0: everything younger than its DMA (or a full wait)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            Wait w;
            for (;;) {
                const bool more = tile_valid(infos + (ti & 7) * 32);
                bool can = more && ti < tl + 2;
                if (FAST && ti < 4) can = can && tl >= 2;  // (tile 1 landed: the spans of tiles 2, 3 with it)
                if (can && ti >= 2)
                    can = __hip_atomic_load(freec + (ti & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= NC * (ti >> 1);
                if (can) {
                    const uint32_t nd = tile_dma<TR, SH::RO_BYTES>(
                        tile_read_ptrs(spans + (ti & 7) * 16, infos + (ti & 7) * 32, stage), lds + (ti & 1) * SLOT, lane);
                    const uint32_t k = ti + NSLOT + 2;
                    const uint32_t na = tile_announce<TR>(cs, spans + (k & 7) * 16, infos + (k & 7) * 32, lane,
                                                          pf + (k & 7) * 8 * NU);
                    cs = cur_next<TR>(cs);
                    ops[ti & 1] = nd + na;
                    ann[ti & 1] = na;
                    ti++;
                    w = Wait{};
                    continue;
                }
                if (tl < ti) {
                    // tile tl's DMA: its announce and the later tile's ops are younger
                    wait_vmcnt(ann[tl & 1] + (ti - tl == 2 ? ops[(tl + 1) & 1] : 0u));
                    __hip_atomic_store(full + (tl & 1), tl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    tl++;
                    w = Wait{};
                    continue;
                }
                if (!more) {  // the end: the decode waves see tile ti invalid and leave
                    __hip_atomic_store(full + (ti & 1), ti + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                if (w.expired(0, ti)) break;  // (bounded: the decode waves stopped releasing)
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return;
        }
        if (fast) {
            // fast start: tile 0's DMA, then the announcements of tiles 1 .. 3 behind it
            if (tile_valid(infos)) tile_dma<TR, SH::RO_BYTES>(tile_read_ptrs(spans, infos, stage), lds, lane);
#pragma unroll
            for (uint32_t k = 1; k <= NSLOT + 1; k++) {
                tile_announce<TR>(cs, spans + (k & 7) * 16, infos + (k & 7) * 32, lane, pf + (k & 7) * 8 * NU);
                cs = cur_next<TR>(cs);
            }
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        } else {
            // tiles 0 .. NSLOT - 2 into their slots; B_0 once tile 0 landed
            uint32_t after0 = 0;  // ops issued after tile 0's DMA
#pragma unroll
            for (uint32_t j = 0; j + 1 < NSLOT; j++) {
                uint32_t n = 0;
                if (tile_valid(infos + j * 32))
                    n = tile_dma<TR, SH::RO_BYTES>(tile_read_ptrs(spans + j * 16, infos + j * 32, stage), lds + j * SLOT, lane);
                after0 += j ? n : 0;
            }
            wait_vmcnt(after0);
        }
        lds_barrier();  // B_0: tile 0 and the spans of tiles 0 .. NSLOT + 1 landed
        uint32_t pend = 0;  // NSLOT 3: ops issued after tile it+1's DMA before this iteration
        for (uint32_t it = 0;; it++) {
            if (!tile_valid(infos + (it & 7) * 32)) break;  // the decode waves leave too
            const uint32_t tn = it + NSLOT - 1, k = it + NSLOT + 2;
            uint32_t nd = 0;
            if (tile_valid(infos + (tn & 7) * 32))
                nd = tile_dma<TR, SH::RO_BYTES>(tile_read_ptrs(spans + (tn & 7) * 16, infos + (tn & 7) * 32, stage),
                                                lds + (tn % NSLOT) * SLOT, lane);
            // tile it+2 into L2 (tuning: MJ_PREFETCH=1; measured slower on configs C/D)
            uint32_t np = 0;
#if MJ_PREFETCH
            const uint32_t t2 = it + 2;
            if (tile_valid(infos + (t2 & 7) * 32))
                np = tile_prefetch(tile_read_ptrs(spans + (t2 & 7) * 16, infos + (t2 & 7) * 32, stage), pf, lane);
#endif
            const uint32_t ns = tile_announce<TR>(cs, spans + (k & 7) * 16, infos + (k & 7) * 32, lane,
                                                  pf + (k & 7) * 8 * NU) + np;
            cs = cur_next<TR>(cs);
#ifdef MJ_STAMPS
            const uint64_t w0 = __builtin_amdgcn_s_memtime();
#endif
            // tile it+1's DMA: the one just issued (NSLOT 2), or the one issued
            // an iteration ago, with `pend` ops behind it then (NSLOT 3)
            wait_vmcnt((NSLOT == 2 ? 0u : pend + nd) + ns);
            pend = ns;
#ifdef MJ_STAMPS
            const uint64_t w1 = __builtin_amdgcn_s_memtime();
            lvm += w1 - w0;
#endif
            lds_barrier();  // B_it+1: tile it+1 landed, tile it decoded
#ifdef MJ_STAMPS
            lwait += __builtin_amdgcn_s_memtime() - w0;
#endif
        }
#ifdef MJ_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
            __hip_atomic_fetch_add((GAS unsigned long long*)args()->err + 2 + 7, (unsigned long long)lwait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add((GAS unsigned long long*)args()->err + 2 + 10, (unsigned long long)lvm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add((GAS unsigned long long*)args()->err + 2 + 8, (unsigned long long)(__builtin_amdgcn_s_memtime() - lt0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#endif
        return;
    }

    // ---- decode waves ----
    uint64_t run[NU];
#pragma unroll
    for (uint32_t u = 0; u < NU; u++) run[u] = 0;
    Lanes L;
    L.blk = ~0u;
#pragma unroll
    for (uint32_t j = 0; j < NCW; j++) L.nacc[j] = 0, L.proj[j] = 0, L.isbool[j] = 0, L.vptr[j] = 0, L.bptr[j] = 0;
#ifdef MJ_STAMPS
    const uint64_t ct0 = __builtin_amdgcn_s_memtime();
#endif
#ifdef MJ_TIMELINE
    const uint64_t tl0 = __builtin_amdgcn_s_memrealtime();
    uint32_t tl_tiles = 0;
#endif
    lds_barrier();  // B_0
#ifdef MJ_TIMELINE
    const uint64_t tl_b0 = __builtin_amdgcn_s_memrealtime();
#endif
    for (uint32_t it = 0;; it++) {
        if constexpr (ER) {  // tile it landed in its slot (or the loader says there is none)
            Wait w;
            bool gone = false;
            while (__hip_atomic_load(full + (it & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < it + 1)
                if (w.expired(0, it)) { gone = true; break; }
            if (gone) break;
        }
        const LAS uint8_t* info = infos + (it & 7) * 32;
        if (!tile_valid(info)) break;
#ifdef MJ_TIMELINE
        tl_tiles++;
#endif
        LAS uint8_t* slot = lds + (it % NSLOT) * SLOT;
        const Tile T = tile_read(spans + (it & 7) * 16, info, stage);
        const LAS uint32_t* ro = (const LAS uint32_t*)slot + T.lead;
        const uint32_t ph = tile_phase(info);
        if (MODE == 0 && T.seg_first) {
            // local mode: a (virtual) block starts at 0, or at its utf8 index
            // entry (in LDS, fetched by the loader with the announcement)
            if constexpr (UPRE) {
                const LAS uint64_t* up = (const LAS uint64_t*)(pf + (it & 7) * 8 * NU);
#pragma unroll
                for (uint32_t u = 0; u < NU; u++) run[u] = T.r0 ? sgpr64(up[u]) : 0;
            } else {
                const uint64_t* ux = (const uint64_t*)sgpr64((uint64_t)((const CAS Blk*)args()->blocks + T.b)->uidx);
#pragma unroll
                for (uint32_t u = 0; u < NU; u++)
                    run[u] = NUTF8 && T.r0 ? sgpr64(((const CAS uint64_t*)ux)[(T.r0 >> args()->ulog) * NU + u]) : 0;
            }
        }
        if (MJ_ABL_LOADONLY) {
            // ablation: no decode; the totals the prefix protocol counts are
            // still published so nothing waits on them
            if (NUTF8 && lane == 0) __hip_atomic_fetch_add((LAS uint32_t*)ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (T.hbm == 2) {  // a tile over 4 GiB of blob bytes (unsupported): report; keep the protocol going
            if (wave == 0 && lane == 0) report(args()->err, err_key(T.b, T.r0, 0, kStMalformed));
            if constexpr (ER) release_slot(freec + (it & 1), lane);
            if (NUTF8) {
                if (lane == 0) __hip_atomic_fetch_add((LAS uint32_t*)ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (MODE == 1 && ph == 1 && T.seg_last && wave == 0 && args()->emit) {
                    for (uint32_t u = 0; u < NU; u++)
                        if (lane == 0) publish(args()->flags + T.t * NU + u, kPre);
                    if (lane == 0) __hip_atomic_store((LAS uint32_t*)ctl + 1, (uint32_t)T.t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        } else if (T.hbm) {
            Tile Th = T;
            tile_ptrs(Th);
            const HbmSrc src{gp(Th.data) + Th.abase};
            if (MODE == 0) decode_tile<SH, 0, HbmSrc, ER>(src, T, ro, ctl, run, L, wave, lane, it, freec + (it & 1));
            else if (ph == 1) decode_tile<SH, 1>(src, T, ro, ctl, run, L, wave, lane, it);
            else decode_tile<SH, 2>(src, T, ro, ctl, run, L, wave, lane, it);
            // drain the cold path's loads here (a compiler-visible vmcnt(0)),
            // so none is pending into a register the hot path reuses
            __builtin_amdgcn_s_waitcnt(0x0F70);
        } else {
            const StageSrc src{slot + SH::RO_BYTES};
            MJ_TIC
            if (MODE == 0) decode_tile<SH, 0, StageSrc, ER>(src, T, ro, ctl, run, L, wave, lane, it, freec + (it & 1));
            else if (ph == 1) decode_tile<SH, 1>(src, T, ro, ctl, run, L, wave, lane, it);
            else decode_tile<SH, 2>(src, T, ro, ctl, run, L, wave, lane, it);
            MJ_TOC(ph == 0 ? 6 : ph == 1 ? 4 : 5)
        }
        if constexpr (!ER) {
            MJ_TIC
            lds_barrier();  // B_it+1
            MJ_TOC(0)
        }
    }
    lanes_flush<R>(L, lane);
#ifdef MJ_STAMPS
    if (lane == 0)
        __hip_atomic_fetch_add((GAS unsigned long long*)args()->err + 2 + 9, (unsigned long long)(__builtin_amdgcn_s_memtime() - ct0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
#ifdef MJ_TIMELINE
    // timeline (MURR_JIT_DEFS=MJ_TIMELINE=1, tuning builds) (100 MHz realtime): decode wave 0's start, first tile, end,
    // tiles, and where the workgroup ran (HW_ID, XCC_ID)
    if (wave == 0 && lane < 4) {
        const uint64_t hw = ((uint64_t)__builtin_amdgcn_s_getreg(20 | (15 << 11)) << 32) | __builtin_amdgcn_s_getreg(4 | (31 << 11));
        const uint64_t tl_end = __builtin_amdgcn_s_memrealtime();
        const uint64_t v = lane == 0 ? tl0 : lane == 1 ? tl_b0 : lane == 2 ? tl_end : ((uint64_t)tl_tiles | (hw << 16));
        ((GAS uint64_t*)args()->sink)[(uint64_t)blockIdx.x * 4 + lane] = v;
    }
#endif
    if (args()->rb_host) epilogue<NC>(ctl, lane);
}

}  // namespace mj

// Local-mode kernels may ask the compiler for a register budget that admits
// MJ_WPE waves per SIMD (SGPRs: 7 waves at <= 96, 8 at <= 80; tuning).
#if defined(MJ_WPE) && MJ_WPE
#define MJ_WPE_ATTR __attribute__((amdgpu_waves_per_eu(MJ_WPE)))
#else
#define MJ_WPE_ATTR
#endif
#define MJ_KERNEL(NW, R, NS, SFX)                                                                         \
    extern "C" __global__ void __launch_bounds__(64 * NW) MJ_WPE_ATTR murr_jit_decode_##NW##x##R##SFX(mj::Args) { \
        mj::kernel_body<NW, R, NS, 0>();                                                                   \
    }                                                                                                      \
    extern "C" __global__ void __launch_bounds__(64 * NW) murr_jit_decode_split_##NW##x##R##SFX(mj::Args) {\
        mj::kernel_body<NW, R, NS, 1>();                                                                   \
    }
MJ_KERNEL(5, 2, 2, )
MJ_KERNEL(5, 1, 2, )
MJ_KERNEL(3, 1, 2, )
MJ_KERNEL(5, 3, 2, )
