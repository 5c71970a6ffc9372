// murr_decode.hip — gfx950 decode kernel: row blobs -> Arrow buffers.
//
// Replaces ReadBatchBuilder::add_row / add_empty / build and the per-dtype
// ColumnEncoders (src/io/row/read.rs:62-110, src/io/codec/primitive.rs:38-61,
// bool_.rs:85-104, utf8.rs:85-105) for K blocks (batch reads) in one launch.
//
// Byte movement, HBM-bound, no MFMA.  A persistent workgroup is one LOADER
// wave and NC = NW-1 CONSUMER waves around a ring of S LDS slots:
//  * A fill is F = 64*KC*NC consecutive rows of one block; its row-offset
//    slice and its blob bytes are contiguous in HBM.  The loader streams fills
//    into the ring with LDS-DMA (global_load_lds_dwordx4, 1 KiB per
//    instruction), P fills deep.  It issues no stores, and every fill costs it
//    the same number E of vector-memory instructions (unused ones load 16 B
//    into a scratch slot), so `s_waitcnt vmcnt((P-1)*E)` is exactly "the fill
//    issued P-1 steps ago has landed"; it then raises that slot's ready flag.
//    Its block cursors live in registers: no scalar-memory round trip per fill.
//  * Consumer wave w decodes sub-tile w (KC 64-row chunks) of every fill, one
//    row per lane, straight out of the slot (aligned ds_read + alignbyte), and
//    writes Arrow buffers to HBM; the slot is free once all NC counted off.
//    No workgroup barrier anywhere: slots are handed over by LDS flags and
//    counters, and the utf8 offset prefix is a decoupled look-back over the
//    workgroup's sub-tile sequence in LDS (block-local mode), to which window
//    mode (a block spread over workgroups) adds, at each fill's first
//    sub-tile, a one-hop window sum of the other workgroups' fill aggregates.
//  * Per sub-tile: row offsets, null bits, fixed-width and bool values and the
//    validity words (from __ballot) go out first (pass A); utf8 cells (payload
//    address, length, wave-inclusive scan) stay in registers across the prefix
//    look-back, then offsets and string bytes go out (pass B).
// Errors are flagged per row in the fast path and re-derived exactly, in the
// reference's row-major / projection order, by a cold path.
#include "murr_device.h"

namespace murr {

namespace {

using namespace dev;

// Ablation switches for tuning builds only (`make ablate`, loaded with
// MURR_LIB); 0 in the production library, where their branches compile away.
//   1: no string byte copy   2: no fixed-width value stores   4: no pass B
//   8: phase stamps
#ifndef MURR_ABLATE
#define MURR_ABLATE 0
#endif

// Phase stamps (MURR_ABLATE & 8, tuning builds only): cycles per phase summed
// over waves into err[2..9] (loader: free-spin, issue, vmcnt wait, other;
// consumer: ready-spin, pass A, look-back, pass B).
constexpr bool kStamps = (MURR_ABLATE & 8) != 0;
struct Stamp {
    uint64_t t = 0, acc[4] = {0, 0, 0, 0};
    __device__ __forceinline__ void start() { if (kStamps) t = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void lap(int i) {
        if (kStamps) { const uint64_t n = __builtin_amdgcn_s_memtime(); acc[i] += n - t; t = n; }
    }
    __device__ __forceinline__ void flush(unsigned long long* err, int base) {
        if (kStamps && (threadIdx.x & 63) == 0)
            for (int i = 0; i < 4; i++)
                __hip_atomic_fetch_add(err + 2 + base + i, (unsigned long long)acc[i], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    }
};

constexpr int kUReg = 2;            // utf8 columns whose cells stay in registers across the look-back
constexpr uint32_t kSpanRing = 32;  // span ring entries (> pipeline depth)
constexpr uint32_t kLb = 128;       // look-back ring entries (>= 64 + sub-tiles in flight)

__device__ __forceinline__ DecBlock ldblk(const DecodeArgs& A, uint64_t i) {
    const CAS DecBlock* p = (const CAS DecBlock*)A.blocks + i;
    DecBlock r;
    r.data = p->data; r.row_off = p->row_off; r.n_rows = p->n_rows; r.tile_base = p->tile_base;
    r.ro32 = p->ro32;
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

// The arguments are re-read from the kernarg segment every sub-tile (s_load,
// K$ hits) through a pointer the compiler cannot see through: otherwise values
// derived from them are hoisted out of the loop into SGPRs and spill.
__device__ __forceinline__ DecodeArgs load_args() {
    const CAS DecodeArgs* ap = (const CAS DecodeArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ap));
    DecodeArgs A;
    A.blocks = ap->blocks; A.proj = ap->proj; A.outs = ap->outs; A.lookback = ap->lookback;
    A.nulls = ap->nulls; A.lens = ap->lens; A.err = ap->err;
    A.total_tiles = ap->total_tiles; A.nblocks = ap->nblocks; A.nproj = ap->nproj; A.nutf8 = ap->nutf8;
    A.bs = ap->bs; A.stage = ap->stage; A.rows_per_tile = ap->rows_per_tile; A.local = ap->local;
    A.ufix[0] = ap->ufix[0]; A.ufix[1] = ap->ufix[1];
    A.nslots = ap->nslots; A.depth = ap->depth; A.dro = ap->dro; A.dst = ap->dst; A.slot_bytes = ap->slot_bytes;
    A.lds_ro = ap->lds_ro; A.lds_stage = ap->lds_stage; A.lds_ready = ap->lds_ready; A.lds_free = ap->lds_free;
    A.lds_span = ap->lds_span; A.lds_lbf = ap->lds_lbf; A.lds_lba = ap->lds_lba; A.lds_lbi = ap->lds_lbi;
    A.lds_nulls = ap->lds_nulls; A.lds_scratch = ap->lds_scratch; A.lds_fa = ap->lds_fa; A.lds_fc = ap->lds_fc;
    A.lds_total = ap->lds_total;
    // every field above: a new DecodeArgs member must be copied here too
    static_assert(sizeof(DecodeArgs) == 176, "load_args: copy every DecodeArgs field");
    return A;
}

// ---- byte sources -----------------------------------------------------------
// Fill bytes staged in LDS (the hot path): unguarded reads; a stale or
// out-of-range LDS read is harmless (beyond the allocation it returns 0) and
// its result is masked by the caller.
struct StageSrc {
    static constexpr bool kHbm = false;
    const LAS uint8_t* s;  // 16-B aligned, >= 32 B of padding past the data
    // Aligned dword reads (ds_read2_b32) + v_alignbyte: an unaligned ds_read_b32
    // is correct on gfx950 but ~25x slower (tools/ubench/lds_unaligned.hip).
    __device__ __forceinline__ uint32_t u8(uint32_t a) const { return s[a]; }
    __device__ __forceinline__ uint32_t u32(uint32_t a) const {
        const LAS uint32_t* w = (const LAS uint32_t*)(s + (a & ~3u));
        return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
    }
    __device__ __forceinline__ uint32_t u16(uint32_t a) const { return u32(a) & 0xFFFFu; }
    __device__ __forceinline__ uint64_t u64(uint32_t a) const {
        const LAS uint32_t* w = (const LAS uint32_t*)(s + (a & ~3u));
        const uint32_t sh = a & 3u, w0 = w[0], w1 = w[1], w2 = w[2];
        return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) |
               ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    }
    // the first n <= 4 bytes at a, zero-extended (the over-read stays in the pad)
    __device__ __forceinline__ uint32_t head(uint32_t a, uint32_t n) const {
        const uint32_t v = u32(a);
        return n >= 4 ? v : v & ((1u << (8 * n)) - 1);
    }
    // bitset bytes 0..3 of a row (bs <= 4)
    __device__ __forceinline__ uint32_t bits(uint32_t ra, uint32_t bs) const { return u32(ra); }
};
// A fill whose rows outgrew the stage is decoded straight from HBM: exact-width
// loads only, never a byte past the field, and callers point unwanted reads at
// the fill's first byte.
struct HbmSrc {
    static constexpr bool kHbm = true;
    const GAS uint8_t* g;
    __device__ __forceinline__ uint32_t u8(uint32_t a) const { return g[a]; }
    __device__ __forceinline__ uint32_t u16(uint32_t a) const { return *(const GAS u16u*)(g + a); }
    __device__ __forceinline__ uint32_t u32(uint32_t a) const { return *(const GAS u32u*)(g + a); }
    __device__ __forceinline__ uint64_t u64(uint32_t a) const { return *(const GAS u64u*)(g + a); }
    __device__ __forceinline__ uint32_t head(uint32_t a, uint32_t n) const {
        uint32_t v = 0;
        for (uint32_t q = 0; q < n && q < 4; q++) v |= (uint32_t)g[a + q] << (8 * q);
        return v;
    }
    __device__ __forceinline__ uint32_t bits(uint32_t ra, uint32_t bs) const {
        uint32_t v = 0;
        for (uint32_t q = 0; q < bs; q++) v |= (uint32_t)g[ra + q] << (8 * q);
        return v;
    }
};

template <class Src>
__device__ __forceinline__ bool utf8_valid_slow(const Src& src, uint32_t at, uint32_t n) {
    Utf8Dfa dfa;
    for (uint32_t q = 0; q < n; q++) dfa.step(src.u8(at + q));
    return dfa.ok();
}

// Unwanted HBM reads are pointed at the fill's first byte; LDS reads are not
// guarded at all.
template <class Src>
__device__ __forceinline__ uint32_t at(bool ok, uint32_t a) {
    return Src::kHbm && !ok ? 0u : a;
}

// ---- the workgroup's fill sequence ---------------------------------------------
// Block-local mode: workgroup w owns blocks w, w+G, ... whole, in fill order.
// Window mode: global fills w, w+G, w+2G, ... of the concatenated blocks.
__device__ __forceinline__ uint64_t tiles_end(const DecodeArgs& A, uint32_t b) {
    return b + 1 < A.nblocks ? ldblk(A, b + 1).tile_base : A.total_tiles;
}

// Fills in this workgroup's sequence.
__device__ __forceinline__ uint32_t wg_tiles(const DecodeArgs& A) {
    const uint32_t w = blockIdx.x, G = gridDim.x;
    if (!A.local) return A.total_tiles > w ? (uint32_t)((A.total_tiles - w + G - 1) / G) : 0u;
    uint64_t n = 0;
    for (uint32_t b = w; b < A.nblocks; b += G) n += tiles_end(A, b) - ldblk(A, b).tile_base;
    return (uint32_t)n;
}

// The loader's cursor: the fill and its block's state, in registers (a scalar
// load only when the block changes).
struct LCur {
    uint64_t t, tb, te, n_rows;
    const uint8_t* data;
    const uint64_t* row_off;  // u32 offsets when ro32 (DecBlock)
    uint32_t b, ok, ro32;
};

__device__ __forceinline__ void cur_block(const DecodeArgs& A, LCur& c, uint32_t b) {
    const DecBlock blk = ldblk(A, b);
    c.b = b;
    c.tb = blk.tile_base;
    c.te = tiles_end(A, b);
    c.n_rows = blk.n_rows;
    c.data = blk.data;
    c.row_off = blk.row_off;
    c.ro32 = blk.ro32;
}

__device__ __forceinline__ LCur cur_first(const DecodeArgs& A) {
    LCur c;
    c.t = c.tb = c.te = c.n_rows = 0;
    c.data = nullptr;
    c.row_off = nullptr;
    c.ro32 = 0;
    c.b = 0;
    c.ok = 0;
    const uint32_t w = blockIdx.x, G = gridDim.x;
    if (A.local) {
        for (uint32_t b = w; b < A.nblocks; b += G) {
            cur_block(A, c, b);
            if (c.te > c.tb) { c.t = c.tb; c.ok = 1; return c; }
        }
        return c;
    }
    if (w >= A.total_tiles) return c;
    uint32_t b = 0;
    while (b + 1 < A.nblocks && ldblk(A, b + 1).tile_base <= w) b++;
    cur_block(A, c, b);
    c.t = w;
    c.ok = 1;
    return c;
}

__device__ __forceinline__ void cur_next(const DecodeArgs& A, LCur& c) {
    if (!c.ok) return;
    const uint32_t G = gridDim.x;
    if (A.local) {
        if (c.t + 1 < c.te) { c.t++; return; }
        for (uint32_t b = c.b + G; b < A.nblocks; b += G) {
            cur_block(A, c, b);
            if (c.te > c.tb) { c.t = c.tb; return; }
        }
        c.ok = 0;
        return;
    }
    c.t += G;
    if (c.t >= A.total_tiles) { c.ok = 0; return; }
    while (c.t >= c.te) cur_block(A, c, c.b + 1);
}

// A slot's descriptor, written by the loader (lane 0) before the DMA is issued.
struct SlotDesc {
    uint64_t t, r0, abase, tfirst;
    const uint8_t* data;
    const uint64_t* row_off;
    uint32_t b, nr, flags;
};
static_assert(sizeof(SlotDesc) <= 64, "slot descriptor");
enum : uint32_t { kFirst = 1, kLast = 2, kHbmTile = 4, kHuge = 8, kRo32 = 16 };

// ---- loader wave ----------------------------------------------------------------
// LDS-DMA by inline asm: hipcc then keeps these loads out of its s_waitcnt
// bookkeeping (as builtins they are pending LDS writes that it drains with
// vmcnt(0) before later ds_reads).  The loader counts them itself
// (wait_vmcnt) and issues no other vector-memory instruction.
__device__ __forceinline__ void glds16(const GAS void* src, LAS void* dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"((uint32_t)(uintptr_t)dst)
                 : "memory");
}
__device__ __forceinline__ void glds4(const GAS void* src, LAS void* dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"((uint32_t)(uintptr_t)dst)
                 : "memory");
}

// Exactly one vector-memory instruction per call: the real LDS-DMA (>= 1 lane
// active) or, for a chunk past the data, lane 0 loading 16 B of a valid
// address into the scratch slot.  The per-fill instruction count is fixed.
__device__ __forceinline__ void dma_1k(const GAS uint8_t* g, uint32_t nb, uint32_t c, LAS uint8_t* dst,
                                       LAS uint8_t* scratch, const GAS uint8_t* valid, uint32_t lane) {
    const uint32_t off = c * 1024 + lane * 16;
    if (c * 1024 < nb) {
        if (off < nb) glds16(g + off, dst + c * 1024);
    } else {
        if (lane == 0) glds16(valid, scratch);
    }
}

// Span DMA for one fill: row_off[r0] and row_off[r0 + nr] (two u64, four
// dword lanes; u32 offsets: lanes 0 and 2, the high dwords masked by the
// reader) into span ring entry e; a dummy for "no such fill".
__device__ __forceinline__ void span_dma(const DecodeArgs& A, const LCur& c, LAS uint8_t* lds, uint32_t e,
                                         uint32_t lane) {
    LAS uint8_t* dst = lds + A.lds_span + e * 16;
    if (c.ok) {
        const uint64_t r0 = (c.t - c.tb) * A.rows_per_tile;
        const uint64_t nr = min((uint64_t)A.rows_per_tile, c.n_rows - r0);
        if (c.ro32) {
            const GAS uint32_t* p = (const GAS uint32_t*)c.row_off + (lane < 2 ? r0 : r0 + nr);
            if (lane == 0 || lane == 2) glds4(p, dst);
        } else {
            const GAS uint8_t* p = (const GAS uint8_t*)(c.row_off + (lane < 2 ? r0 : r0 + nr)) + (lane & 1) * 4;
            if (lane < 4) glds4(p, dst);
        }
    } else {
        if (lane == 0) glds4((const GAS void*)A.blocks, lds + A.lds_scratch);
    }
}

// s_waitcnt vmcnt(n) for a run-time n (clamped to the 6-bit field).
__device__ __forceinline__ void wait_vmcnt(uint32_t n) {
    switch (min(n, 63u)) {
#define W(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
        W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15)
        W(16) W(17) W(18) W(19) W(20) W(21) W(22) W(23) W(24) W(25) W(26) W(27) W(28) W(29) W(30) W(31)
        W(32) W(33) W(34) W(35) W(36) W(37) W(38) W(39) W(40) W(41) W(42) W(43) W(44) W(45) W(46) W(47)
        W(48) W(49) W(50) W(51) W(52) W(53) W(54) W(55) W(56) W(57) W(58) W(59) W(60) W(61) W(62) W(63)
#undef W
    }
}

__device__ __forceinline__ uint32_t lds_load(const LAS uint32_t* f) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void set_flag(LAS uint32_t* f, uint32_t v) {
    __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void spin_report() {
    const CAS DecodeArgs* ap = (const CAS DecodeArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    report(ap->err, kStInternal);
}
// Bounded spins on LDS flags and counters: a protocol bug reports
// MURR_E_INTERNAL and lets the waves drain instead of hanging the GPU.
__device__ __forceinline__ void spin_until_eq(const LAS uint32_t* f, uint32_t v) {
    uint32_t spins = 0;
    while (lds_load(f) != v) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > kSpinLimit) { spin_report(); return; }
    }
}
__device__ __forceinline__ void spin_until_ge(const LAS uint32_t* f, uint32_t v) {
    uint32_t spins = 0;
    while (lds_load(f) < v) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > kSpinLimit) { spin_report(); return; }
    }
}

template <int NW>
__device__ __forceinline__ void loader_wave(LAS uint8_t* lds) {
    constexpr uint32_t NC = NW - 1;
    const uint32_t lane = tidx() & 63;
    const DecodeArgs A = load_args();
    const uint32_t J = wg_tiles(A), S = A.nslots, P = A.depth, F = A.rows_per_tile;
    const uint32_t E = 1 + A.dro + A.dst;  // vector-memory instructions per step
    LAS uint32_t* ready = (LAS uint32_t*)(lds + A.lds_ready);
    LAS uint32_t* freec = (LAS uint32_t*)(lds + A.lds_free);
    LAS uint8_t* scratch = lds + A.lds_scratch;
    // prologue: spans of fills 0 .. P-1
    LCur cs = cur_first(A);
    LCur ci = cs;  // the fill being issued; cs runs P fills ahead
    for (uint32_t k = 0; k < P; k++) {
        span_dma(A, cs, lds, k % kSpanRing, lane);
        cur_next(A, cs);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    Stamp st;
    st.start();
    for (uint32_t j = 0; j < J; j++) {
        const uint32_t slot = j % S;
        LAS uint8_t* sb = lds + slot * A.slot_bytes;
        st.lap(3);
        if (j >= S) spin_until_ge(freec + slot, NC * (j / S));  // every consumer of fill j-S is done
        st.lap(0);
        // this fill's span: landed (step j-P's wait, or the prologue)
        const LAS uint64_t* sp = (const LAS uint64_t*)(lds + A.lds_span + (j % kSpanRing) * 16);
        const uint64_t om = ci.ro32 ? 0xFFFFFFFFull : ~0ull;
        const uint64_t base = sgpr64(sp[0]) & om, end = sgpr64(sp[1]) & om;
        const uint64_t r0 = (ci.t - ci.tb) * F;
        const uint32_t nr = (uint32_t)min((uint64_t)F, ci.n_rows - r0);
        const uint64_t abase = base & ~15ull;
        const uint64_t span = ((end + 15) & ~15ull) - abase;
        uint32_t flags = (r0 == 0 ? kFirst : 0) | (r0 + nr == ci.n_rows ? kLast : 0) | (ci.ro32 ? kRo32 : 0);
        if (end - abase > 0xFFFFFFF0ull) flags |= kHuge;
        else if (span > A.stage) flags |= kHbmTile;
        if (lane == 0) {
            LAS SlotDesc* d = (LAS SlotDesc*)sb;
            d->t = ci.t; d->r0 = r0; d->abase = abase; d->tfirst = ci.tb;
            d->data = ci.data; d->row_off = ci.row_off;
            d->b = ci.b; d->nr = nr; d->flags = flags;
            ((LAS uint32_t*)(lds + A.lds_fc))[slot] = 0;
        }
        for (uint32_t u = lane; u < A.nutf8; u += 64) ((LAS uint64_t*)(lds + A.lds_fa))[u * S + slot] = 0;
        // fill j+P's span, then fill j's row offsets and blob bytes
        span_dma(A, cs, lds, (j + P) % kSpanRing, lane);
        cur_next(A, cs);
        const uint32_t ow = ci.ro32 ? 4 : 8;  // row offset width
        const uintptr_t rp = (uintptr_t)ci.row_off + r0 * ow;
        const uintptr_t s0 = rp & ~(uintptr_t)15;
        const uint32_t nb_ro = (uint32_t)(((rp - s0) + (uint64_t)(nr + 1) * ow + 15) & ~15ull);
        const GAS uint8_t* valid = (const GAS uint8_t*)s0;
        for (uint32_t k = 0; k < A.dro; k++)
            dma_1k((const GAS uint8_t*)s0, nb_ro, k, sb + A.lds_ro, scratch, valid, lane);
        const uint32_t nb = (flags & (kHbmTile | kHuge)) ? 0u : (uint32_t)span;
        for (uint32_t k = 0; k < A.dst; k++)
            dma_1k(gp(ci.data) + abase, nb, k, sb + A.lds_stage, scratch, valid, lane);
        st.lap(1);
        // the fill issued P-1 steps ago has landed: hand it over
        wait_vmcnt((P - 1) * E);
        st.lap(2);
        if (j + 1 >= P && lane == 0) set_flag(ready + (j + 1 - P) % S, j + 2 - P);
        cur_next(A, ci);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st.flush(A.err, 0);
    if (lane == 0)
        for (uint32_t k = J + 1 > P ? J + 1 - P : 0; k < J; k++) set_flag(ready + k % S, k + 1);
}

// ---- consumer: one sub-tile ------------------------------------------------------
struct Tile {
    uint64_t t, r0, abase, tfirst;
    const uint8_t* data;
    const uint64_t* row_off;
    uint32_t b, nr, flags;
};

__device__ __forceinline__ Tile read_desc(const LAS uint8_t* sb) {
    const LAS SlotDesc* d = (const LAS SlotDesc*)sb;
    Tile T;
    T.t = sgpr64(d->t); T.r0 = sgpr64(d->r0); T.abase = sgpr64(d->abase);
    T.tfirst = sgpr64(d->tfirst);
    T.data = (const uint8_t*)sgpr64((uint64_t)d->data);
    T.row_off = (const uint64_t*)sgpr64((uint64_t)d->row_off);
    T.b = sgpr(d->b); T.nr = sgpr(d->nr); T.flags = sgpr(d->flags);
    return T;
}

// Per-row state of one sub-tile's KC chunks, shared by every column.
// rl is normalised to 0 for a missing, malformed or out-of-tile row, so
// "present" is rl != 0 (a present row holds its bitset: rl >= bs >= 1); no
// per-row booleans stay live (lane masks would pile up in SGPRs).
template <int KC>
struct Rows {
    uint32_t ra[KC], rl[KC], bits[KC];
};

// ReadRow::is_null (read.rs:32-37) for a row that is present; a missing row
// (add_empty) is null in every column.
template <int KC, class Src>
__device__ __forceinline__ bool null_bit(const Rows<KC>& W, int k, uint32_t bit, uint32_t bs, const Src& src) {
    if (bs <= 4) return W.rl[k] == 0 || ((W.bits[k] >> bit) & 1);
    const uint32_t b = src.u8(at<Src>(W.rl[k] != 0, W.ra[k] + (bit >> 3)));
    return W.rl[k] == 0 || ((b >> (bit & 7)) & 1);
}

// Rows of chunk k in the sub-tile (wave-uniform).
__device__ __forceinline__ uint32_t chunk_rows(const Tile& T, int k) {
    const uint32_t c0 = k * 64;
    return c0 < T.nr ? min(64u, T.nr - c0) : 0u;
}

// One fixed-width or bool column over the sub-tile's KC chunks.  KIND: 1 bool,
// else the value width in bytes (0 = one byte).  Returns the nulls.
template <int KIND, int KC, class Src>
__device__ __forceinline__ uint32_t fixed_col(const Src& src, const Rows<KC>& W, const Tile& T, uint64_t word0,
                                              const DecProj& pc, const DecOut& o, uint32_t bs, uint32_t* badk) {
    constexpr uint32_t WID = KIND == 8 ? 8 : KIND == 4 ? 4 : KIND == 2 ? 2 : 1;
    const uint32_t lane = tidx() & 63;
    const uint32_t fo = bs + pc.offset, bit = pc.bit;
    uint32_t nn = 0;
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const uint32_t nk = chunk_rows(T, k);  // wave-uniform
        const bool isnull = null_bit(W, k, bit, bs, src);
        const bool have = !isnull && fo + WID <= W.rl[k];
        *badk |= (uint32_t)(!isnull && !have) << k;
        const uint32_t a = at<Src>(have, W.ra[k] + fo);
        const uint64_t vm = __ballot(!isnull);  // out-of-tile lanes are null
        nn += nk - (uint32_t)__popcll(vm);
        if (nk && lane == 0) gp((uint64_t*)o.validity)[word0 + k] = vm;
        const uint32_t i = k * 64 + lane;
        const bool act = lane < nk && !(MURR_ABLATE & 2);
        if constexpr (KIND == 1) {
            const uint32_t v = src.u8(a);
            const uint64_t m = __ballot(have && v != 0);
            if (nk && lane == 0) gp((uint64_t*)o.values)[word0 + k] = m;
        } else if constexpr (KIND == 8) {
            const uint64_t v = src.u64(a);
            if (act) (gp((uint64_t*)o.values) + T.r0)[i] = have ? v : 0;
        } else if constexpr (KIND == 4) {
            const uint32_t v = src.u32(a);
            if (act) (gp((uint32_t*)o.values) + T.r0)[i] = have ? v : 0;
        } else if constexpr (KIND == 2) {
            const uint32_t v = src.u16(a);
            if (act) (gp((uint16_t*)o.values) + T.r0)[i] = have ? (uint16_t)v : 0;
        } else {
            const uint32_t v = src.u8(a);
            if (act) (gp(o.values) + T.r0)[i] = have ? (uint8_t)v : 0;
        }
    }
    return nn;
}

// read_dynamic (read.rs:45-55) for one chunk of one utf8 column: payload
// address and string length per lane (0 for null / missing / malformed),
// sets *bad for a non-null cell the reference would panic on.
template <int KC, class Src>
__device__ __forceinline__ uint32_t utf8_cell(const Src& src, const Rows<KC>& W, int k, uint32_t fo, uint32_t bs,
                                              bool isnull, uint32_t* pay, bool* bad) {
    const bool s_ok = !isnull && fo + 4 <= W.rl[k];
    const uint32_t slot = src.u32(at<Src>(s_ok, W.ra[k] + fo));
    const uint32_t vlen = W.rl[k] - bs;  // >= 4 when s_ok (fo >= bs)
    const bool p_ok = s_ok && slot <= vlen - 4;
    const uint32_t len = src.u32(at<Src>(p_ok, W.ra[k] + bs + slot));
    const bool good = p_ok && len <= vlen - 4 - slot;
    *bad = !isnull && !good;
    *pay = W.ra[k] + bs + slot + 4;
    return good ? len : 0;
}

// Pass A of one utf8 column: cells, per-chunk inclusive scans, validity words,
// the sub-tile's string bytes (*tot).  Returns the nulls.
template <int KC, class Src>
__device__ __forceinline__ uint32_t utf8_col(const Src& src, const Rows<KC>& W, const Tile& T, uint64_t word0,
                                             const DecProj& pc, const DecOut& o, uint32_t bs, uint32_t* badk,
                                             uint32_t (&pay)[KC], uint32_t (&len)[KC], uint32_t (&inc)[KC],
                                             uint32_t* tot) {
    const uint32_t lane = tidx() & 63;
    const uint32_t fo = bs + pc.offset;
    uint32_t nn = 0, wt = 0;
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const uint32_t nk = chunk_rows(T, k);
        const bool isnull = null_bit(W, k, pc.bit, bs, src);
        bool bad;
        len[k] = utf8_cell(src, W, k, fo, bs, isnull, &pay[k], &bad);
        *badk |= (uint32_t)bad << k;
        inc[k] = wave_scan_u32(len[k]);  // < fill span < 4 GiB
        wt += __builtin_amdgcn_readlane(inc[k], 63);
        const uint64_t vm = __ballot(!isnull);
        nn += nk - (uint32_t)__popcll(vm);
        if (nk && lane == 0) gp((uint64_t*)o.validity)[word0 + k] = vm;
    }
    *tot = wt;
    return nn;
}

// Copy one string (stage or HBM) to vb[d .. d+slen) with unaligned dword
// stores and a 0-3 byte tail; returns the OR of its bytes (UTF-8 pre-check).
template <class Src>
__device__ __forceinline__ uint32_t copy_str(const Src& src, GAS uint8_t* vb, uint32_t d, uint32_t pay,
                                             uint32_t slen) {
    uint32_t hib = 0, q = 0;
#pragma unroll 1
    for (; q + 4 <= slen; q += 4) {
        const uint32_t v = src.u32(pay + q);
        *(GAS u32u*)(vb + (d + q)) = v;
        hib |= v;
    }
    const uint32_t n = slen - q;
    if (n) {
        const uint32_t v = src.head(pay + q, n);
        hib |= v;
        if (n & 2) *(GAS u16u*)(vb + (d + q)) = (uint16_t)v;
        if (n & 1) vb[d + q + (n & 2)] = (uint8_t)(v >> (8 * (n & 2)));
    }
    return hib;
}

// Pass B of one utf8 column (projection index p) with the sub-tile's prefix:
// offsets, string bytes, UTF-8 validation.  REG: the cells come from pass A's
// registers; otherwise they are re-parsed from the source.
template <int KC, bool REG, class Src>
__device__ __forceinline__ void utf8_emit(const DecodeArgs& A, const Src& src, const Rows<KC>& W, const Tile& T,
                                          uint32_t p, uint64_t prefix, uint32_t ttot,
                                          const uint32_t (&rpay)[KC], const uint32_t (&rlen)[KC],
                                          const uint32_t (&rinc)[KC]) {
    const uint32_t lane = tidx() & 63;
    const uint32_t bs = A.bs;
    const DecProj pc = ldproj(A, p);
    const DecOut o = ldout(A, (uint64_t)T.b * A.nproj + p);
    if (lane == 0) {
        if (T.flags & kFirst) gp(o.offsets)[0] = 0;
        if (T.flags & kLast) gp(A.lens)[(uint64_t)T.b * A.nproj + p] = prefix + ttot;
    }
    uint64_t base = prefix;
    GAS int32_t* ob = gp(o.offsets) + T.r0 + 1;
    const uint32_t fo = bs + pc.offset;
#pragma unroll
    for (int k = 0; k < KC; k++) {
        uint32_t slen, pay, inc;
        if constexpr (REG) {
            slen = rlen[k]; pay = rpay[k]; inc = rinc[k];
        } else {
            bool bad;
            slen = utf8_cell(src, W, k, fo, bs, null_bit(W, k, pc.bit, bs, src), &pay, &bad);
            inc = wave_scan_u32(slen);
        }
        const uint32_t tot = __builtin_amdgcn_readlane(inc, 63);
        const uint32_t i = k * 64 + lane;
        const bool act = lane < chunk_rows(T, k);
        const uint64_t end = base + tot;
        uint32_t hib = 0;
        if (end <= 0x7FFFFFFFull && end <= o.values_cap) {  // wave-uniform fast path
            if (act) ob[i] = (int32_t)(base + inc);
            GAS uint8_t* vb = gp(o.values) + base;
            if (slen && !(MURR_ABLATE & 1)) hib = copy_str(src, vb, inc - slen, pay, slen);
        } else {
            const uint64_t e = base + inc;
            if (act) {
                if (e > 0x7FFFFFFFull) report(A.err, err_key(T.b, T.r0 + i, p, kStOverflow));
                else ob[i] = (int32_t)e;
                if (slen && e > o.values_cap) report(A.err, err_key(T.b, T.r0 + i, p, kStCapacity));
            }
#pragma unroll 1
            for (uint32_t q = 0; q < slen; q += 4) hib |= src.head(pay + q, min(4u, slen - q));
        }
        if ((hib & 0x80808080u) && !utf8_valid_slow(src, pay, slen))
            report(A.err, err_key(T.b, T.r0 + i, p, kStUtf8));
        base = end;
    }
}

// One-hop window sum of other workgroups' fill aggregates over [lo, t): the
// whole wave loads the granules (agent-scope relaxed loads = sc1, bypassing
// this CU's L1), every load in flight before the first check.  Only fills
// that are resident or done are ever waited on; spins are bounded.
__device__ __forceinline__ uint64_t window_sum(const uint64_t* st, uint64_t lo, uint64_t t,
                                               unsigned long long* err, uint64_t ekey) {
    constexpr int K = 4;
    const uint32_t lane = tidx() & 63;
    uint64_t sum = 0;
    for (uint64_t j0 = lo; j0 < t; j0 += 64 * K) {
        uint64_t v[K];
#pragma unroll
        for (int i = 0; i < K; i++) {
            const uint64_t j = j0 + i * 64 + lane;
            v[i] = j < t ? __hip_atomic_load(gp(st) + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1;
        }
#pragma unroll
        for (int i = 0; i < K; i++) {
            const uint64_t j = j0 + i * 64 + lane;
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
    return wave_sum64(sum);
}

// LDS look-back ring over the workgroup's sub-tile sequence: flag of entry
// s % kLb = (s + 1) << 2 | state (1: aggregates published, 2: inclusive).
struct LookBack {
    LAS uint32_t* f;
    LAS uint64_t* agg;  // [nutf8][kLb]
    LAS uint64_t* inc;  // [nutf8][kLb]
};

__device__ __forceinline__ LookBack lookback_of(const DecodeArgs& A, LAS uint8_t* lds) {
    return LookBack{(LAS uint32_t*)(lds + A.lds_lbf), (LAS uint64_t*)(lds + A.lds_lba),
                    (LAS uint64_t*)(lds + A.lds_lbi)};
}

__device__ __forceinline__ void lb_publish(const LookBack& L, uint32_t s, uint32_t state) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // values before the flag
    if ((tidx() & 63) == 0) set_flag(L.f + s % kLb, ((s + 1) << 2) | state);
}

// Decoupled look-back: the number d of predecessors s-1 .. s-d that are
// aggregate-only before the first inclusive one (s-1-d).  Lane l watches s-1-l.
__device__ __forceinline__ uint32_t lb_depth(const LookBack& L, uint32_t s) {
    const uint32_t lane = tidx() & 63;
    const uint32_t want = s - lane;  // sequence tag of sub-tile s-1-lane
    uint32_t spins = 0;
    for (;;) {
        const uint32_t f = lane < s ? lds_load(L.f + (s - 1 - lane) % kLb) : 0u;
        const bool mine = (f >> 2) == want;
        const uint64_t incl = __ballot(mine && (f & 2));
        const uint64_t pub = __ballot(mine && (f & 3));
        if (incl) {
            const uint32_t d = (uint32_t)__builtin_ctzll(incl);
            const uint64_t need = d == 63 ? ~0ull : ((2ull << d) - 1);
            if ((pub & need) == need) return d;
        }
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSpinLimit) { spin_report(); return 0; }
    }
}

// inc[u][s-1-d] + the aggregates agg[u][s-1-l], l < d.
__device__ __forceinline__ uint64_t lb_sum(const LookBack& L, uint32_t u, uint32_t s, uint32_t d) {
    uint64_t v = sgpr64(L.inc[u * kLb + (s - 1 - d) % kLb]);
    for (uint32_t l = 0; l < d; l++) v += sgpr64(L.agg[u * kLb + (s - 1 - l) % kLb]);
    return v;
}

// The prefix of sub-tile s (w-th of its fill) for every utf8 column, with the
// aggregates of pass A already in L.agg: publishes the inclusive prefixes
// and returns those of the first kUReg columns in pre[].
__device__ __forceinline__ void prefixes(const DecodeArgs& A, const Tile& T, LAS uint8_t* lds, uint32_t s,
                                         uint32_t w, uint32_t slot, uint32_t NC, uint64_t (&pre)[kUReg]) {
    const uint32_t lane = tidx() & 63, nutf8 = A.nutf8;
    const LookBack L = lookback_of(A, lds);
    const uint32_t e = s % kLb;
    if (!A.local) {
        // the fill's aggregate, for other workgroups: the last sub-tile to add
        // its own publishes the sum (LDS operations of a wave are in order)
        LAS unsigned long long* fa = (LAS unsigned long long*)(lds + A.lds_fa);
        LAS uint32_t* fc = (LAS uint32_t*)(lds + A.lds_fc);
        for (uint32_t u = lane; u < nutf8; u += 64)
            __hip_atomic_fetch_add(fa + u * A.nslots + slot, (unsigned long long)L.agg[u * kLb + e], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        uint32_t c = 0;
        if (lane == 0) c = __hip_atomic_fetch_add(fc + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        c = __builtin_amdgcn_readlane(c, 0);
        if (c == NC - 1)
            for (uint32_t u = lane; u < nutf8; u += 64)
                __hip_atomic_store(gp(A.lookback) + (uint64_t)u * A.total_tiles + T.t,
                                   (uint64_t)__hip_atomic_load(fa + u * A.nslots + slot, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP) + 1,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // Local mode: a block's first sub-tile starts at 0; every other one looks
    // back.  Window mode: a fill's first sub-tile takes this workgroup's
    // previous sub-tile (same block) plus the window of other workgroups'
    // fills between; the others look back to it (it never publishes an
    // aggregate-only state, so no look-back can skip the window term).
    const bool direct = A.local ? (T.flags & kFirst) != 0 : w == 0;
    bool have_prev = false;
    uint32_t d = 0;
    uint64_t lo = T.tfirst;
    if (!direct) {
        lb_publish(L, s, 1);
        d = lb_depth(L, s);
        have_prev = true;
    } else if (!A.local) {
        const uint64_t G = gridDim.x;
        if (T.t >= T.tfirst + G) {
            have_prev = true;
            lo = T.t - G + 1;
            spin_until_eq(L.f + (s - 1) % kLb, (s << 2) | 2);  // sub-tile s-1's inclusive prefix
        }
    }
    const bool window = direct && !A.local;
#pragma unroll
    for (int u = 0; u < kUReg; u++) {
        pre[u] = 0;
        if ((uint32_t)u >= nutf8) continue;
        if (have_prev) pre[u] = lb_sum(L, u, s, d);
        if (window)
            pre[u] += sgpr64(window_sum(A.lookback + (uint64_t)u * A.total_tiles, lo, T.t, A.err,
                                        err_key(T.b, T.r0, A.ufix[u], 0)));
        if (lane == 0) L.inc[u * kLb + e] = pre[u] + L.agg[u * kLb + e];
    }
#pragma unroll 1
    for (uint32_t u = kUReg; u < nutf8; u++) {
        uint64_t pr = have_prev ? lb_sum(L, u, s, d) : 0;
        if (window)
            pr += sgpr64(window_sum(A.lookback + (uint64_t)u * A.total_tiles, lo, T.t, A.err, err_key(T.b, T.r0, 0, 0)));
        if (lane == 0) L.inc[u * kLb + e] = pr + L.agg[u * kLb + e];
    }
    lb_publish(L, s, 2);
}

template <int KC, class Src>
__device__ __forceinline__ void decode_tile(const DecodeArgs& A, const Src& src, const Tile& T,
                                            const LAS uint32_t* ro, uint32_t rs, LAS uint8_t* lds, uint32_t s, uint32_t w,
                                            uint32_t slot, uint32_t NC, LAS uint32_t* wnull, Stamp& st) {
    const uint32_t lane = tidx() & 63;
    const uint32_t bs = A.bs, nproj = A.nproj, nutf8 = A.nutf8;
    const uint32_t abase = (uint32_t)T.abase;
    const uint64_t word0 = T.r0 >> 6;  // validity / bool word of chunk 0
    const LookBack L = lookback_of(A, lds);
    const uint32_t e = s % kLb;

    Rows<KC> W;
    uint32_t badk = 0;
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const uint32_t i = k * 64 + lane;
        const uint32_t a0 = ro[rs * i], a1 = ro[rs * (i + 1)];
        const uint32_t rl = i < T.nr ? a1 - a0 : 0;
        W.ra[k] = a0 - abase;
        badk |= (uint32_t)(rl != 0 && rl < bs) << k;
        W.rl[k] = rl >= bs ? rl : 0;
        W.bits[k] = bs <= 4 ? src.bits(at<Src>(W.rl[k] != 0, W.ra[k]), bs) : 0;
    }

    // ---- pass A: fixed-width and bool columns (dispatch once per column) ----
#pragma unroll 1
    for (uint32_t p = 0; p < nproj; p++) {
        const DecProj pc = ldproj(A, p);
        if (pc.is_utf8) continue;
        const DecOut o = ldout(A, (uint64_t)T.b * nproj + p);
        uint32_t nn;
        if (pc.dtype == kBool) nn = fixed_col<1, KC>(src, W, T, word0, pc, o, bs, &badk);
        else if (pc.width == 4) nn = fixed_col<4, KC>(src, W, T, word0, pc, o, bs, &badk);
        else if (pc.width == 8) nn = fixed_col<8, KC>(src, W, T, word0, pc, o, bs, &badk);
        else if (pc.width == 2) nn = fixed_col<2, KC>(src, W, T, word0, pc, o, bs, &badk);
        else nn = fixed_col<0, KC>(src, W, T, word0, pc, o, bs, &badk);
        if (lane == 0 && nn) wnull[p] += nn;
    }
    // ---- pass A: utf8 columns (cells of the first kUReg kept in registers) ----
    uint32_t upay[kUReg][KC], ulen[kUReg][KC], uinc[kUReg][KC], utot[kUReg];
#pragma unroll
    for (int u = 0; u < kUReg; u++) {
        utot[u] = 0;
        if ((uint32_t)u >= nutf8) continue;  // uniform
        const uint32_t p = A.ufix[u];
        const DecProj pc = ldproj(A, p);
        const DecOut o = ldout(A, (uint64_t)T.b * nproj + p);
        const uint32_t nn = utf8_col(src, W, T, word0, pc, o, bs, &badk, upay[u], ulen[u], uinc[u], &utot[u]);
        if (lane == 0) {
            L.agg[u * kLb + e] = utot[u];
            if (nn) wnull[p] += nn;
        }
    }
    if (nutf8 > kUReg) {
#pragma unroll 1
        for (uint32_t p = 0; p < nproj; p++) {
            const DecProj pc = ldproj(A, p);
            if (!pc.is_utf8 || pc.uslot < kUReg) continue;
            const DecOut o = ldout(A, (uint64_t)T.b * nproj + p);
            uint32_t xp[KC], xl[KC], xi[KC], wt;
            const uint32_t nn = utf8_col(src, W, T, word0, pc, o, bs, &badk, xp, xl, xi, &wt);
            if (lane == 0) {
                L.agg[pc.uslot * kLb + e] = wt;
                if (nn) wnull[p] += nn;
            }
        }
    }

    // Exact error reports, in the reference's order (projection order inside a
    // row; the packed key orders rows).  Cold: only rows the fast pass flagged.
    if (__ballot(badk != 0)) {
#pragma unroll
        for (int k = 0; k < KC; k++) {
            if (!((badk >> k) & 1)) continue;
            const uint32_t i = k * 64 + lane;
            const uint64_t row = T.r0 + i;
            const uint32_t ra = W.ra[k], rl = ro[rs * (i + 1)] - ro[rs * i];
            if (rl < bs) { report(A.err, err_key(T.b, row, 0, kStMalformed)); continue; }
            for (uint32_t p = 0; p < nproj; p++) {
                const DecProj pc = ldproj(A, p);
                if ((src.u8(ra + (pc.bit >> 3)) >> (pc.bit & 7)) & 1) continue;
                const uint32_t fo = bs + pc.offset;
                bool bad;
                if (pc.is_utf8) {
                    bad = fo + 4 > rl;
                    if (!bad) {
                        const uint32_t slot_v = src.u32(ra + fo);
                        bad = slot_v > rl - bs - 4;
                        if (!bad) bad = src.u32(ra + bs + slot_v) > rl - bs - 4 - slot_v;
                    }
                } else {
                    bad = fo + pc.width > rl;
                }
                if (bad) { report(A.err, err_key(T.b, row, p, kStMalformed)); break; }
            }
        }
    }
    st.lap(1);
    if (!nutf8) return;

    uint64_t pre[kUReg];
    prefixes(A, T, lds, s, w, slot, NC, pre);
    st.lap(2);
    if (MURR_ABLATE & 4) return;

    // ---- pass B: utf8 offsets and string bytes --------------------------------
#pragma unroll
    for (int u = 0; u < kUReg; u++) {
        if ((uint32_t)u >= nutf8) break;
        utf8_emit<KC, true>(A, src, W, T, A.ufix[u], pre[u], utot[u], upay[u], ulen[u], uinc[u]);
    }
    if (nutf8 > kUReg) {
#pragma unroll 1
        for (uint32_t p = 0; p < nproj; p++) {
            const DecProj pc = ldproj(A, p);
            if (!pc.is_utf8 || pc.uslot < kUReg) continue;
            const uint32_t x = pc.uslot * kLb + e;
            const uint64_t tot = sgpr64(L.agg[x]);
            utf8_emit<KC, false>(A, src, W, T, p, sgpr64(L.inc[x]) - tot, (uint32_t)tot, upay[0], ulen[0], uinc[0]);
        }
    }
}

__device__ __forceinline__ void flush_nulls(const DecodeArgs& A, LAS uint32_t* wnull, uint32_t b) {
    for (uint32_t p = tidx() & 63; p < A.nproj; p += 64) {
        const uint32_t v = wnull[p];
        if (v) {
            __hip_atomic_fetch_add(gp(A.nulls) + (uint64_t)b * A.nproj + p, (unsigned long long)v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            wnull[p] = 0;
        }
    }
}

template <int NW, int KC>
__device__ __forceinline__ void consumer_wave(LAS uint8_t* lds, uint32_t w) {
    constexpr uint32_t NC = NW - 1, SUB = 64 * KC;
    const uint32_t lane = tidx() & 63;
    uint32_t J, S;
    {
        const DecodeArgs A = load_args();
        J = wg_tiles(A);
        S = A.nslots;
    }
    uint32_t cur_b = ~0u;
    Stamp st;
    st.start();
    for (uint32_t j = 0; j < J; j++) {
        const DecodeArgs A = load_args();
        const uint32_t slot = j % S;
        LAS uint8_t* sb = lds + slot * A.slot_bytes;
        LAS uint32_t* wnull = (LAS uint32_t*)(lds + A.lds_nulls) + w * A.nproj;
        st.lap(3);
        spin_until_eq((const LAS uint32_t*)(lds + A.lds_ready) + slot, j + 1);
        st.lap(0);
        const Tile D = read_desc(sb);
        // this wave's sub-tile of the fill
        const uint32_t s0 = w * SUB;
        Tile T = D;
        T.r0 = D.r0 + s0;
        T.nr = D.nr > s0 ? min(SUB, D.nr - s0) : 0u;
        T.flags = (D.flags & (kHbmTile | kHuge)) | ((D.flags & kFirst) && w == 0 ? kFirst : 0u) |
                  ((D.flags & kLast) && T.nr && s0 + T.nr == D.nr ? kLast : 0u);
        const uint32_t rs = (D.flags & kRo32) ? 1u : 2u;  // dwords per row offset
        const LAS uint32_t* ro =
            (const LAS uint32_t*)(sb + A.lds_ro + (((uintptr_t)D.row_off + D.r0 * rs * 4) & 15)) + rs * s0;
        if (T.b != cur_b) {  // this wave's null counters belong to one block
            if (cur_b != ~0u) flush_nulls(A, wnull, cur_b);
            cur_b = T.b;
        }
        const uint32_t s = j * NC + w;
        if (T.flags & kHuge) {  // a fill over 4 GiB (unsupported): report, prefixes of 0
            if (lane == 0 && w == 0) report(A.err, err_key(T.b, D.r0, 0, kStMalformed));
            if (A.nutf8) {
                const LookBack L = lookback_of(A, lds);
                for (uint32_t u = lane; u < A.nutf8; u += 64) L.agg[u * kLb + s % kLb] = 0;
                uint64_t pre[kUReg];
                prefixes(A, T, lds, s, w, slot, NC, pre);
            }
        } else if (T.flags & kHbmTile) {
            decode_tile<KC>(A, HbmSrc{gp(T.data) + T.abase}, T, ro, rs, lds, s, w, slot, NC, wnull, st);
        } else {
            decode_tile<KC>(A, StageSrc{sb + A.lds_stage}, T, ro, rs, lds, s, w, slot, NC, wnull, st);
        }
        st.lap(3);
        // every LDS read of the slot has returned: count this wave off the fill
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0)
            __hip_atomic_fetch_add((LAS uint32_t*)(lds + A.lds_free) + slot, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (cur_b != ~0u) {
        const DecodeArgs A = load_args();
        flush_nulls(A, (LAS uint32_t*)(lds + A.lds_nulls) + w * A.nproj, cur_b);
    }
    st.flush(load_args().err, 4);
}

// NW waves: waves 0 .. NW-2 consume, wave NW-1 loads.  At least 4 waves per
// SIMD (<= 128 VGPRs) so two 8-wave workgroups can share a CU.
template <int NW, int KC>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4, 8))) decode_kernel(DecodeArgs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_[];
    LAS uint8_t* lds = (LAS uint8_t*)lds_;
    const uint32_t tid = tidx();
    {
        const DecodeArgs A = load_args();
        // flags, counters and per-wave null counters start at 0
        for (uint32_t i = tid; i < A.nslots; i += 64 * NW) {
            ((LAS uint32_t*)(lds + A.lds_ready))[i] = 0;
            ((LAS uint32_t*)(lds + A.lds_free))[i] = 0;
        }
        for (uint32_t i = tid; i < kLb; i += 64 * NW) ((LAS uint32_t*)(lds + A.lds_lbf))[i] = 0;
        for (uint32_t i = tid; i < (NW - 1) * A.nproj; i += 64 * NW) ((LAS uint32_t*)(lds + A.lds_nulls))[i] = 0;
    }
    __syncthreads();
    const uint32_t wave = sgpr(tid >> 6);
    if (wave == NW - 1) loader_wave<NW>(lds);
    else consumer_wave<NW, KC>(lds, wave);
}

}  // namespace

// The LDS plan of a launch (DecodeArgs): S slots [descriptor | row-offset
// slice | blob stage], then ready flags, free counters, the span ring, the
// look-back ring, per-wave null counters, a DMA scratch and the per-slot fill
// aggregates (window mode).
void decode_lds_plan(DecodeArgs& a, uint32_t nw, uint32_t kc, uint32_t slots, uint32_t depth) {
    const uint32_t F = 64 * kc * (nw - 1);
    auto r16 = [](uint32_t x) { return (x + 15) & ~15u; };
    a.rows_per_tile = F;
    const uint32_t ro_bytes = r16(8 * (F + 1) + 16);
    a.dro = (ro_bytes + 1023) / 1024;
    a.stage = (a.stage + 1023) & ~1023u;
    a.dst = a.stage / 1024;
    a.lds_ro = 64;
    a.lds_stage = 64 + ro_bytes;
    a.slot_bytes = r16(a.lds_stage + a.stage + 32);
    a.nslots = slots;
    a.depth = depth;
    uint32_t o = a.nslots * a.slot_bytes;
    a.lds_ready = o; o += r16(4 * slots);
    a.lds_free = o; o += r16(4 * slots);
    a.lds_span = o; o += kSpanRing * 16;
    a.lds_lbf = o; o += 4 * kLb;
    a.lds_lba = o; o += 8 * kLb * a.nutf8;
    a.lds_lbi = o; o += 8 * kLb * a.nutf8;
    a.lds_nulls = o; o += r16(4 * (nw - 1) * a.nproj);
    a.lds_scratch = o; o += 64;
    a.lds_fa = o; o += 8 * slots * a.nutf8;
    a.lds_fc = o; o += r16(4 * slots);
    a.lds_total = o;
}

#define MURR_DECODE_SHAPES(X) X(4, 1) X(4, 2) X(4, 4) X(8, 1) X(8, 2) X(8, 4)

bool decode_shape_ok(uint32_t nw, uint32_t kc) {
#define X(W, K) if (nw == W && kc == K) return true;
    MURR_DECODE_SHAPES(X)
#undef X
    return false;
}

hipError_t launch_decode(const DecodeArgs& a, uint32_t nw, uint32_t kc, uint32_t grid, hipStream_t s) {
#define X(W, K)                                                                              \
    if (nw == W && kc == K) {                                                                \
        hipLaunchKernelGGL((decode_kernel<W, K>), dim3(grid), dim3(64 * W), a.lds_total, s, a); \
        return hipGetLastError();                                                            \
    }
    MURR_DECODE_SHAPES(X)
#undef X
    return hipErrorInvalidValue;
}

int decode_blocks_per_cu(uint32_t nw, uint32_t kc, uint32_t lds) {
    int n = 0;
    hipError_t e = hipErrorInvalidValue;
#define X(W, K) \
    if (nw == W && kc == K) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_kernel<W, K>, 64 * W, lds);
    MURR_DECODE_SHAPES(X)
#undef X
    return e == hipSuccess ? n : 1;
}

}  // namespace murr
