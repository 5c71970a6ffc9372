// murr_jit_encode.hip — schema-specialised encode kernel (Arrow buffers -> row
// blobs), compiled at run time per segment layout like the decode kernel
// (murr_jit.cpp).  The host prepends a prelude fixing the bitset size, the
// static capacity and, per column in segment order, its kind and offset.
//
// Replaces Table::write's row loop: WriteRow::new (0xFF bitset), then every
// column's ColumnDecoder::write_to_row (src/io/table/mod.rs:97-109,
// src/io/row/write.rs:19-52, primitive.rs:85-95, bool_.rs:111-117,
// utf8.rs:113-119).  Same contract and arguments as encode_kernel
// (murr_kernels.hip).
//
// One thread builds one row of a 256-row tile.  The row's fixed part (bitset
// + static region) is assembled in registers with compile-time byte
// placement, shifted to its byte position and merged into an LDS stage of the
// tile (zeroed first; ds_or on the two edge dwords, plain stores between);
// utf8 payloads are merged the same way.  The stage then goes out with
// aligned 16-B stores.  Without utf8 columns every row has the same size and
// row i starts at i * (bs + cap); with them, murr_jit_encode_sizes sums each
// tile's row sizes (validity and utf8 offsets only), murr_jit_encode_scan
// turns the sums into tile starts, and the encode scans its rows inside the
// tile.

#ifdef __HIPCC_RTC__
typedef unsigned char uint8_t;
typedef unsigned short uint16_t;
typedef unsigned int uint32_t;
typedef unsigned long long uint64_t;
typedef int int32_t;
typedef long long int64_t;
typedef unsigned long long uintptr_t;
#else  // offline syntax/ISA check build
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#define GAS __attribute__((address_space(1)))
#define LAS __attribute__((address_space(3)))
#define CAS __attribute__((address_space(4)))
#define DEV __device__ __forceinline__

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace mje {

struct Col {  // = murr::EncCol
    const uint8_t* values;
    const uint8_t* validity;
    const int32_t* offsets;
    uint64_t offset;
    uint32_t dtype, index, soff, width;
};
struct Args {  // = murr::EncodeArgs
    const Col* cols;
    uint8_t* out;
    uint64_t* row_off;       // n_rows + 1
    uint64_t* lookback;      // [total_tiles]
    unsigned long long* err;
    uint64_t n_rows, out_cap, total_tiles;
    uint32_t ncols, nutf8, bs, cap;
    uint64_t row_base;       // row_off values are row_base + offset in out
};

#ifndef MJE_TILE
#define MJE_TILE 256
#endif
constexpr uint32_t TILE = MJE_TILE, NWAVE = MJE_TILE / 64, BS = MJE_BS, CAP = MJE_CAP, NCOLS = MJE_NCOLS, NUTF8 = MJE_NUTF8,
                   STAGE = MJE_STAGE;
constexpr uint32_t FIXED = BS + CAP;
constexpr uint32_t NR = (FIXED + 3) / 4;  // dwords of the fixed part
// kStRecount: a tile's exact size differs from its estimate (never returned:
// the host recounts with the sizes pass, murr_encode_batch_at)
enum : uint32_t { kStCapacity = 6, kStInternal = 10, kStRecount = 12 };
constexpr uint32_t kSpinLimit = 1u << 22;

DEV uint64_t err_key(uint64_t block, uint64_t row, uint32_t col, uint32_t status) {
    if (row > 0xFFFFFFFFull) row = 0xFFFFFFFFull;
    if (block > 0x3FFFFull) block = 0x3FFFFull;
    return (block << 46) | (row << 14) | ((uint64_t)(col & 0x3FF) << 4) | (status & 0xF);
}
DEV void report(unsigned long long* err, uint64_t key) {
    __hip_atomic_fetch_max((GAS unsigned long long*)err, (unsigned long long)~key, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
DEV uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
DEV uint64_t sgpr64(uint64_t v) {
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) | __builtin_amdgcn_readfirstlane((uint32_t)v);
}
template <class T> DEV GAS T* gp(T* p) { return (GAS T*)p; }
template <class T> DEV const GAS T* gp(const T* p) { return (const GAS T*)p; }

DEV const CAS Args* args() {
    const CAS Args* ap = (const CAS Args*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ap));
    return ap;
}
DEV Col ldcol(uint32_t c) {
    const CAS Col* p = (const CAS Col*)args()->cols + c;
    Col r;
    r.values = p->values; r.validity = p->validity; r.offsets = p->offsets; r.offset = p->offset;
    return r;
}

// The columns' descriptors in a lane table: field f (values, validity,
// offsets, offset) of column c is the u64 in lane (f * NCOLS + c) % 64 of VGPR
// pair (f * NCOLS + c) / 64 -- one pair for up to 16 columns -- loaded once per
// workgroup by one vector load per pair; a use is two v_readlane per field
// with a compile-time lane, instead of a chain of scalar loads (the
// kernel-argument pointer, then the descriptor) and its wait: about 140 scalar
// loads per wave on config C's column set.  Past 64 columns: scalar loads.
// On for eight columns or more: config E's ten 0.308 -> 0.299 ms, C's sixteen
// neutral, B's two 0.210 -> 0.227 (the table's load opens every one-tile
// workgroup; profiles/r04/probes/ab29.txt).
#ifndef MJE_TAB
#define MJE_TAB (NCOLS >= 8)
#endif
constexpr uint32_t TABP = MJE_TAB && NCOLS <= 64 ? (4 * NCOLS + 63) / 64 : 0;  // VGPR pairs (0: scalar loads)
struct ColTab {
    uint32_t lo[TABP ? TABP : 1], hi[TABP ? TABP : 1];
};
DEV ColTab load_tab(uint32_t lane) {
    ColTab t;
#pragma unroll
    for (uint32_t j = 0; j < TABP; j++) {
        const uint32_t L = 64 * j + lane, f = L / NCOLS, c = L % NCOLS;
        uint64_t v = 0;
        if (f < 4) v = *((const GAS uint64_t*)((const GAS Col*)args()->cols + c) + f);
        t.lo[j] = (uint32_t)v;
        t.hi[j] = (uint32_t)(v >> 32);
    }
    return t;
}
template <uint32_t C> DEV Col tcol(const ColTab& t) {
    if constexpr (TABP == 0) {
        return ldcol(C);
    } else {
        auto rl64 = [&](uint32_t f) {
            const uint32_t L = f * NCOLS + C;
            return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(t.hi[L / 64], L % 64) << 32) |
                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane(t.lo[L / 64], L % 64);
        };
        Col r;
        r.values = (const uint8_t*)rl64(0);
        r.validity = (const uint8_t*)rl64(1);
        r.offsets = (const int32_t*)rl64(2);
        r.offset = rl64(3);
        return r;
    }
}

// Arrow validity (null buffer absent = all valid).
DEV bool valid(const Col& c, uint64_t e) {
    if (!c.validity) return true;
    return (gp(c.validity)[e >> 3] >> (e & 7)) & 1;
}
// Bit (ew + lane) of an Arrow bitmap for the 64 rows of a wave (ew uniform):
// three scalar dwords cover the wave's 64 bits, so the texture data path --
// the encode's bound -- sees no load; a window that would
// reach past the bitmap's bytes (nbytes = ceil((offset + n) / 8)) takes the
// per-lane byte load.
DEV bool bit_of_wave(const uint8_t* bm, uint64_t ew, uint32_t lane, uint64_t nbytes) {
    // a bitmap that does not start on a dword: its bits counted from the dword below
    const uint32_t mis = (uint32_t)((uintptr_t)bm & 3u);
    bm -= mis;
    ew += 8 * mis;
    nbytes += mis;
    const uint64_t d = ew >> 5;
    if ((d + 3) * 4 <= nbytes) {
        const CAS uint32_t* p = (const CAS uint32_t*)bm + d;
        const uint32_t x0 = p[0], x1 = p[1], x2 = p[2];
        const uint32_t sh = (uint32_t)ew & 31u;
        const uint64_t lo = ((uint64_t)x1 << 32) | x0;
        const uint64_t w = sh ? (lo >> sh) | ((uint64_t)x2 << (64 - sh)) : lo;
        return (w >> lane) & 1;
    }
    const uint64_t e = ew + lane;
    return (gp(bm)[e >> 3] >> (e & 7)) & 1;
}
DEV bool valid_wave(const Col& c, uint64_t ew, uint32_t lane, uint64_t nbytes) {
    if (!c.validity) return true;
    return bit_of_wave(c.validity, ew, lane, nbytes);
}

// Column kinds at compile time (0 utf8, 9 bool, else width) and each bool
// column's ordinal among the bool columns.
constexpr uint32_t kKind[NCOLS ? NCOLS : 1] = {
#define MJE_K(C, KIND, SOFF, U) KIND,
    MJE_COLS(MJE_K)
#undef MJE_K
};
constexpr uint32_t bool_ord(uint32_t c) {
    uint32_t n = 0;
    for (uint32_t j = 0; j < c; j++) n += kKind[j] == 9;
    return n;
}
constexpr uint32_t NBOOL = bool_ord(NCOLS);

// Every bitmap word a wave needs, in one vector load.  Lane j < NCOLS takes
// column j's validity bitmap, lane NCOLS + k the k-th bool column's values;
// each loads the three dwords covering the wave's 64 bits and realigns them
// to a 64-bit window (wlo, whi), and column C's window is then two
// v_readlane's.  This replaced three scalar loads per bitmap whose uses sat
// in separate branches, so a wave waited for each column's bitmaps in turn
// (validity reads were a third of config C's encode).  A lane
// whose window would pass the bitmap's bytes (the batch's last rows) marks
// its bitmap for the per-lane byte path (`slow`).
#ifndef MJE_VBITS
#define MJE_VBITS 1
#endif
constexpr bool VBITS = MJE_VBITS && NCOLS + NBOOL <= 64;
struct Bits {
    uint32_t wlo, whi;  // lane j: the window of bitmap j
    uint64_t slow;      // bitmaps read per lane instead
};

// The fixed part of one row as dwords, byte placement at compile time.
struct Row {
    uint32_t w[NR + 1];
};
template <uint32_t OFF> DEV void put8(Row& r, uint32_t v) { r.w[OFF / 4] |= (v & 0xFFu) << (8 * (OFF % 4)); }
template <uint32_t OFF> DEV void put16(Row& r, uint32_t v) {
    v &= 0xFFFFu;
    r.w[OFF / 4] |= v << (8 * (OFF % 4));
    if constexpr (OFF % 4 == 3) r.w[OFF / 4 + 1] |= v >> 8;
}
template <uint32_t OFF> DEV void put32(Row& r, uint32_t v) {
    r.w[OFF / 4] |= v << (8 * (OFF % 4));
    if constexpr (OFF % 4 != 0) r.w[OFF / 4 + 1] |= v >> (32 - 8 * (OFF % 4));
}

// Wave64 inclusive scan (u32) on DPP; block scan across the 4 waves.
DEV uint32_t wave_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);
    return v;
}

// Merge `v` (4 stream bytes starting at stage byte b) into the zeroed stage.
DEV void or_bytes(LAS uint32_t* stw, uint32_t b, uint32_t v, uint32_t nbytes) {
    if (nbytes < 4) v &= (1u << (8 * nbytes)) - 1u;
    const uint32_t d = b >> 2, sh = b & 3u;
    __hip_atomic_fetch_or(stw + d, v << (8 * sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (sh && (v >> (32 - 8 * sh)))
        __hip_atomic_fetch_or(stw + d + 1, v >> (32 - 8 * sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Copy stage[0, span) to out[g0, g0 + span): aligned 16-B stores in the middle,
// byte stores for the unaligned head and tail (other tiles own their
// neighbours).
// The blob stream's whole 16-B pieces: non-temporal stores (written once,
// read by the caller's own later work): config B's column set 0.219 -> 0.212
// ms, C 1.037 -> 1.018, E 0.320 -> 0.310 (profiles/r04/probes/ab27.txt).
#ifndef MJE_OUT_NT
#define MJE_OUT_NT 1
#endif
DEV void write_out(const LAS uint8_t* buf, GAS uint8_t* out, uint64_t g0, uint64_t span, uint32_t tid) {
    const uint64_t g1 = g0 + span;
    const uint64_t a0 = (g0 + 15) & ~15ull, a1 = g1 & ~15ull;
    if (a0 >= a1) {
        for (uint64_t k = tid; k < span; k += TILE) out[g0 + k] = buf[k];
        return;
    }
    if (tid < a0 - g0) out[g0 + tid] = buf[tid];
    if (tid < g1 - a1) out[a1 + tid] = buf[a1 - g0 + tid];
    const uint32_t lb0 = (uint32_t)(a0 - g0), sh = lb0 & 3u;
    const LAS uint32_t* w = (const LAS uint32_t*)buf;
    const uint64_t nch = (a1 - a0) >> 4;
    GAS u32x4* o = (GAS u32x4*)(out + a0);
    for (uint64_t c = tid; c < nch; c += TILE) {
        const uint32_t q = (lb0 >> 2) + 4 * (uint32_t)c;
        const uint32_t d0 = w[q], d1 = w[q + 1], d2 = w[q + 2], d3 = w[q + 3], d4 = w[q + 4];
        u32x4 v;
        v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
        v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
        v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
        v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
#if MJE_OUT_NT
        __builtin_nontemporal_store(v, o + c);
#else
        o[c] = v;
#endif
    }
}

// One row's fixed part and payload sizes.  `pos` = payload append position
// (write.rs:44-52), starting at bs + cap.
// Strings of up to 4 * MJE_PF - 4 bytes are loaded whole with the row, among
// the other columns' loads: 9 dwords for wide rows (a fixed part of 32 bytes
// or more) with one or two utf8 columns (config C 1.04-1.08 -> 1.01-1.04 ms,
// E unchanged), else 5 (config B's 9-byte rows 0.212 -> 0.222 ms at 9; past
// two utf8 columns 4 more dwords each would cost occupancy);
// profiles/r03/probes/enc_pf_ab.txt.
#ifndef MJE_PF
#define MJE_PF (MJE_BS + MJE_CAP >= 32 && MJE_NUTF8 <= 2 ? 9 : 5)
#endif
constexpr uint32_t PF = MJE_PF;  // aligned dwords of each string loaded with the row (the rest later)
// String staging (MJE_SBW bytes of LDS per wave, 0 = off).  The strings of a
// wave's 64 rows in one utf8 column are one contiguous range of the Arrow
// values buffer: the wave copies each column's range into its part of LDS by
// LDS-DMA (16-B pieces, 1 KiB per wave-instruction) and every lane reads its
// string from there -- instead of PF scattered dword loads per lane and
// column, which made the texture data path the encode's bound (DESIGN.md
// §3.2).  A wave whose ranges do not fit takes the per-lane loads.
#ifndef MJE_SBW
#define MJE_SBW 0
#endif
#ifndef MJE_STREAM
#define MJE_STREAM 1
#endif
constexpr uint32_t SBW = NUTF8 && MJE_STREAM ? MJE_SBW : 0;
DEV void glds16(const GAS void* src, LAS void* dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst))
                 : "memory");
}
// Where a wave's staged strings are: per utf8 column, the LDS byte offset of
// its range (in the wave's part) and the 16-B aligned global address it starts at.
struct StrStage {
    uint32_t base[NUTF8 ? NUTF8 : 1];
    uint64_t g0[NUTF8 ? NUTF8 : 1];
    bool on;
};
struct RowBuild {
    ColTab t;  // the columns' descriptors (load_tab)
    Row r;
    uint32_t vmask[(NCOLS + 31) / 32 ? (NCOLS + 31) / 32 : 1];  // valid bits, segment order
    uint32_t pos;
    uint32_t ulen[NUTF8 ? NUTF8 : 1];
    uint64_t ustart[NUTF8 ? NUTF8 : 1];  // Arrow data offset of the string
    uint32_t pre[NUTF8 ? NUTF8 : 1][PF];  // its first PF aligned dwords (without string staging)
    int32_t s0[NUTF8 ? NUTF8 : 1], s1[NUTF8 ? NUTF8 : 1];  // its Arrow offsets
    uint32_t x[NCOLS ? NCOLS : 1], xh[NCOLS ? NCOLS : 1];  // fixed-width values as loaded (xh: high dword of 8-byte ones)
};

DEV Bits load_bits(uint64_t rw, uint32_t lane, const ColTab& tab) {
    Bits b{0u, 0u, 0ull};
    if constexpr (VBITS) {
        // lane j's bitmap and element offset, picked from the columns'
        // descriptors (scalar loads, cached) -- no vector load before the
        // bitmap load, and nothing at all when no column has a bitmap
        const uint8_t* bm = nullptr;
        uint64_t eoff = 0;
        bool any = false;
#define MJE_BM(C, KIND, SOFF, U)                                                          \
        {                                                                                 \
            const Col c = tcol<C>(tab);                                                   \
            any = any || c.validity || KIND == 9;                                         \
            if (lane == C) { bm = c.validity; eoff = c.offset; }                          \
            if (KIND == 9 && lane == NCOLS + bool_ord(C)) { bm = c.values; eoff = c.offset; } \
        }
        MJE_COLS(MJE_BM)
#undef MJE_BM
        if (!any) return b;
        const uint32_t mis = (uint32_t)((uintptr_t)bm & 3u);
        const uint64_t ew = eoff + rw + 8 * mis;
        const uint64_t nbytes = (eoff + args()->n_rows + 7) / 8 + mis;
        const uint64_t d = ew >> 5;
        const bool fast = bm && (d + 3) * 4 <= nbytes;
        uint32_t x0 = 0, x1 = 0, x2 = 0;
        if (fast) {
            const GAS uint32_t* p = (const GAS uint32_t*)(bm - mis) + d;
            x0 = p[0];
            x1 = p[1];
            x2 = p[2];
        }
        const uint32_t sh = (uint32_t)ew & 31u;
        const uint64_t lo = ((uint64_t)x1 << 32) | x0;
        const uint64_t w = sh ? (lo >> sh) | ((uint64_t)x2 << (64 - sh)) : lo;
        b.wlo = (uint32_t)w;
        b.whi = (uint32_t)(w >> 32);
        b.slow = __ballot(bm && !fast);
    }
    return b;
}
// Bit `lane` of bitmap j's window (j compile-time).
template <uint32_t J> DEV bool bits_at(const Bits& b, uint32_t lane) {
    const uint64_t w = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(b.whi, J) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane(b.wlo, J);
    return (w >> lane) & 1;
}

// One row is built in four phases, each over every column, so that a wave's
// loads are all in flight before it waits for any of them: the utf8 offsets;
// the bitmap windows (load_bits); every fixed-width value; then, once the
// offsets and the bitmaps are in, each string's first dwords; and last the row
// assembly.  Every load is unconditional (in bounds for any row < n_rows)
// and masked by the validity bit afterwards: a load guarded by the bit would
// wait for the validity load, one more round trip per column.

// The validity of column C's cell in this lane's row.
template <uint32_t C>
DEV bool valid_of(const Col& c, uint64_t rw, uint32_t lane, const Bits& bits) {
    if (!c.validity) return true;
    if constexpr (VBITS) {
        if (!((bits.slow >> C) & 1)) return bits_at<C>(bits, lane);
    }
    return bit_of_wave(c.validity, sgpr64(c.offset + rw), lane, (c.offset + args()->n_rows + 7) >> 3);
}

template <uint32_t C, uint32_t KIND, uint32_t SOFF, uint32_t U> DEV void ld_offs(RowBuild& B, uint64_t row) {
    if constexpr (KIND == 0) {
        const Col c = tcol<C>(B.t);
        const uint64_t e = c.offset + row;
        B.s0[U] = gp(c.offsets)[e];
        B.s1[U] = gp(c.offsets)[e + 1];
    }
}

template <uint32_t C, uint32_t KIND, uint32_t SOFF, uint32_t U> DEV void ld_fixed(RowBuild& B, uint64_t row) {
    if constexpr (KIND != 0 && KIND != 9) {
        const Col c = tcol<C>(B.t);
        const uint64_t e = c.offset + row;
        if constexpr (KIND == 8) {
            const GAS uint32_t* p = (const GAS uint32_t*)(gp(c.values) + e * 8);
            B.x[C] = p[0];
            B.xh[C] = p[1];
        } else if constexpr (KIND == 4) {
            B.x[C] = ((const GAS uint32_t*)gp(c.values))[e];
        } else if constexpr (KIND == 2) {
            B.x[C] = ((const GAS uint16_t*)gp(c.values))[e];
        } else {
            B.x[C] = gp(c.values)[e];
        }
    }
}

// A string's first aligned dwords, so their latency overlaps the row assembly
// and the tile scan (an aligned dword never crosses a page: bytes around the
// string are safe to load and masked later).
template <uint32_t C, uint32_t KIND, uint32_t SOFF, uint32_t U>
DEV void ld_str(RowBuild& B, uint64_t rw, uint32_t lane, const Bits& bits, bool staged) {
    if constexpr (KIND == 0) {
        const Col c = tcol<C>(B.t);
        const bool v = valid_of<C>(c, rw, lane, bits);
        const uint32_t len = v ? (uint32_t)(B.s1[U] - B.s0[U]) : 0u;
        const uint64_t a = v ? (uint64_t)(int64_t)B.s0[U] : 0u;
        B.ulen[U] = len;
        B.ustart[U] = a;
        if constexpr (SBW > 0) return;  // (read at emit time: from the wave's LDS copy, or from HBM when it did not fit)
        const uintptr_t sp = (uintptr_t)(gp(c.values) + a);
        const GAS uint32_t* w = (const GAS uint32_t*)(sp & ~(uintptr_t)3);
        const uint32_t nd = v ? (len + (uint32_t)(sp & 3) + 3) / 4 : 0u;
#pragma unroll
        for (uint32_t i = 0; i < PF; i++) B.pre[U][i] = i < nd ? w[i] : 0u;
    }
}

// The wave's string range of utf8 column C (rows rw .. rw + nact - 1, their
// Arrow offsets already in B.s0 / B.s1) into its LDS part at S.base[U], by
// LDS-DMA.  `at`: bytes of the part used so far; S.on drops to false when a
// range does not fit (then no DMA is issued for it or any later column).
template <uint32_t C, uint32_t KIND, uint32_t SOFF, uint32_t U>
DEV void stage_col(const RowBuild& B, LAS uint8_t* part, uint32_t nact, uint32_t lane, uint32_t& at, StrStage& S) {
    if constexpr (KIND == 0 && SBW > 0) {
        if (!S.on) return;
        const Col c = tcol<C>(B.t);
        const int32_t first = __builtin_amdgcn_readfirstlane(B.s0[U]);
        const int32_t last = __builtin_amdgcn_readlane(B.s1[U], nact - 1);
        const uint64_t g0 = ((uint64_t)(uintptr_t)gp(c.values) + (uint64_t)(int64_t)first) & ~15ull;
        const uint64_t g1 = ((uint64_t)(uintptr_t)gp(c.values) + (uint64_t)(int64_t)last + 15) & ~15ull;
        const uint64_t sz = last >= first ? g1 - g0 : ~0ull;
        if (sz > SBW - at) {
            S.on = false;
            return;
        }
        S.base[U] = at;
        S.g0[U] = g0;
        for (uint32_t q = 0; q * 1024 < sz; q++)
            if (q * 1024 + lane * 16 < sz)
                glds16((const GAS uint8_t*)(uintptr_t)g0 + q * 1024 + lane * 16, part + at + q * 1024);
        at += (uint32_t)sz;
    }
}

// rw: the wave's first row (uniform)
template <uint32_t C, uint32_t KIND, uint32_t SOFF, uint32_t U>
DEV void put_col(RowBuild& B, uint64_t rw, uint32_t lane, const Bits& bits) {
    const Col c = tcol<C>(B.t);
    const bool v = valid_of<C>(c, rw, lane, bits);
    B.vmask[C / 32] |= (uint32_t)v << (C % 32);
    constexpr uint32_t OFF = BS + SOFF;
    if constexpr (KIND == 0) {  // utf8: slot = payload offset relative to the static region
        put32<OFF>(B.r, v ? B.pos - BS : 0u);
        if (v) B.pos += 4 + B.ulen[U];
    } else if constexpr (KIND == 9) {  // bool: b as u8 (bool_.rs:111-117)
        uint32_t b = 0;
        if constexpr (VBITS) {
            constexpr uint32_t J = NCOLS + bool_ord(C);
            b = (bits.slow >> J) & 1 ? bit_of_wave(c.values, sgpr64(c.offset + rw), lane, (c.offset + args()->n_rows + 7) >> 3)
                                    : bits_at<J>(bits, lane);
        } else {
            b = bit_of_wave(c.values, sgpr64(c.offset + rw), lane, (c.offset + args()->n_rows + 7) >> 3);
        }
        put8<OFF>(B.r, v ? b : 0u);
    } else if constexpr (KIND == 8) {
        put32<OFF>(B.r, v ? B.x[C] : 0u);
        put32<OFF + 4>(B.r, v ? B.xh[C] : 0u);
    } else if constexpr (KIND == 4) {
        put32<OFF>(B.r, v ? B.x[C] : 0u);
    } else if constexpr (KIND == 2) {
        put16<OFF>(B.r, v ? B.x[C] : 0u);
    } else {
        put8<OFF>(B.r, v ? B.x[C] : 0u);
    }
}

// The bitset (WriteRow::new fills 0xFF; set_non_null clears a column's bit).
DEV void put_bitset(RowBuild& B) {
#pragma unroll
    for (uint32_t k = 0; k < (BS + 3) / 4; k++) {
        uint32_t w = ~0u;
        if (k * 32 < NCOLS) w &= ~B.vmask[k];  // bits of valid columns cleared
        const uint32_t nb = BS - 4 * k < 4 ? BS - 4 * k : 4;
        if (nb < 4) w &= (1u << (8 * nb)) - 1u;
        B.r.w[k] |= w;
    }
}

// Utf8 payloads of one row into the stage: u32 len, then the bytes, read as
// the aligned dwords that cover them (an aligned dword never crosses a page,
// so the bytes around the string are safe to load and are masked off).
template <uint32_t C, uint32_t U>
DEV void put_payload(const RowBuild& B, LAS uint32_t* stw, uint32_t rb, uint32_t& p) {
    const uint32_t n = B.ulen[U];
    if (!((B.vmask[C / 32] >> (C % 32)) & 1)) return;
    or_bytes(stw, rb + p, n, 4);
    p += 4;
    const Col c = tcol<C>(B.t);
    const uintptr_t sa_ptr = (uintptr_t)(gp(c.values) + B.ustart[U]);
    const uint32_t sa = (uint32_t)(sa_ptr & 3);
    const GAS uint32_t* w = (const GAS uint32_t*)(sa_ptr - sa);
    const uint32_t d0 = rb + p - sa;  // stage byte of w[0]'s first byte
    auto merge = [&](uint32_t v, uint32_t i) {
        // keep the bytes b with 0 <= 4i + b - sa < n
        const int32_t lo = (int32_t)sa - 4 * (int32_t)i, hi = (int32_t)(n + sa) - 4 * (int32_t)i;
        if (lo > 0) v &= ~0u << (8 * lo);
        if (hi < 4) v &= (1u << (8 * hi)) - 1u;
        const uint32_t x = d0 + 4 * i, dw = x >> 2, sh = x & 3u;
        if (v << (8 * sh))
            __hip_atomic_fetch_or(stw + dw, v << (8 * sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (sh && (v >> (32 - 8 * sh)))
            __hip_atomic_fetch_or(stw + dw + 1, v >> (32 - 8 * sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
#pragma unroll
    for (uint32_t i = 0; i < PF; i++)
        if (4 * i < n + sa) merge(B.pre[U][i], i);  // loaded with the row
    // the rest in batches of four loads issued together (one round trip per
    // 16 bytes instead of one per dword)
    for (uint32_t i = PF; 4 * i < n + sa; i += 4) {
        uint32_t x[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) x[q] = 4 * (i + q) < n + sa ? w[i + q] : 0u;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++)
            if (4 * (i + q) < n + sa) merge(x[q], i + q);
    }
    p += n;
}

// The bytes of one row written to the stage in order, as whole dwords: the
// dwords wholly inside the row are plain LDS stores; the first (when the row
// starts mid-dword) and the last partial one are shared with the neighbouring
// rows and are OR-merged into the zeroed stage.
#ifndef MJE_STREAM
#define MJE_STREAM 1
#endif
// Bytes [lo, hi) of dword v to stage bytes a + lo .. a + hi (a dword-aligned):
// the partial dwords a row shares with its neighbours are written bytewise,
// so the stage needs no zeroing pass before the rows are merged into it.
// Short rows (a fixed part under 32 bytes, e.g. config B's 9) zero the
// stage and OR-merge the shared edge dwords instead: with two edges per ~18
// bytes the byte writes cost more than the zeroing pass (B 0.212 vs 0.226 ms;
// C 1.07 vs 1.11 and E 0.353 vs 0.359 ms the other way round).
#ifndef MJE_ZERO
#define MJE_ZERO (MJE_BS + MJE_CAP < 32)
#endif
DEV void put_bytes(LAS uint32_t* stw, uint32_t d, uint32_t v, uint32_t lo, uint32_t hi) {
    if (MJE_ZERO) {
        const uint32_t m = (hi >= 4 ? ~0u : (1u << (8 * hi)) - 1u) & (~0u << (8 * lo));
        __hip_atomic_fetch_or(stw + d, v & m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
    }
    if (lo == 0 && hi >= 4) {
        stw[d] = v;
        return;
    }
    LAS uint8_t* b = (LAS uint8_t*)(stw + d);
#pragma unroll
    for (uint32_t j = 0; j < 4; j++)
        if (j >= lo && j < hi) b[j] = (uint8_t)(v >> (8 * j));
}

struct Emit {
    LAS uint32_t* stw;
    uint32_t d, d0, sh;  // next stage dword, the row's first dword, its byte offset in it
    uint64_t acc;        // pending bytes, lowest first
    uint32_t nb;         // how many (< 4 between puts)
    DEV void start(LAS uint32_t* s, uint32_t rb) {
        stw = s;
        d = d0 = rb >> 2;
        sh = rb & 3u;
        acc = 0;
        nb = sh;  // the first dword's leading bytes are the previous row's (zero here)
    }
    DEV void emit(uint32_t w) {
        if (d == d0 && sh) put_bytes(stw, d, w, sh, 4);  // the first dword's leading bytes are the previous row's
        else stw[d] = w;
        d++;
    }
    DEV void put(uint32_t v, uint32_t m) {  // the low m (1..4) bytes of v
        if (m < 4) v &= (1u << (8 * m)) - 1u;
        acc |= (uint64_t)v << (8 * nb);
        nb += m;
        if (nb >= 4) {
            emit((uint32_t)acc);
            acc >>= 32;
            nb -= 4;
        }
    }
    DEV void finish() {
        if (nb) put_bytes(stw, d, (uint32_t)acc, d == d0 ? sh : 0u, nb);
    }
};

// Utf8 payload of column C into the emitter: u32 len, then the string in
// 4-byte chunks realigned from the aligned dwords that cover it (dwords past
// the string are never loaded; they read as 0).
#ifndef MJE_ABL_NOSTR  // ablation (tuning): string bytes not copied
#define MJE_ABL_NOSTR 0
#endif
#ifndef MJE_ABL_NOOUT  // ablation (tuning): the stage is not written out
#define MJE_ABL_NOOUT 0
#endif
// String bytes [0, n) into the emitter from the aligned dwords w[0..] that
// cover them (sa = the string's offset in w[0]); dwords past the string are
// never read (they count as 0).
template <class W> DEV void emit_str(Emit& E, W* w, uint32_t n, uint32_t sa) {
    uint32_t cur = n ? w[0] : 0u;
#pragma unroll 1
    for (uint32_t q = 0; 4 * q < n; q += 4) {
        uint32_t x[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) x[k] = 4 * (q + 1 + k) < n + sa ? w[q + 1 + k] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
            if (4 * (q + k) < n) E.put(__builtin_amdgcn_alignbyte(x[k], k ? x[k - 1] : cur, sa), umin(4u, n - 4 * (q + k)));
        cur = x[3];
    }
}

template <uint32_t C, uint32_t U>
DEV void emit_payload(const RowBuild& B, Emit& E, const StrStage& S, const LAS uint8_t* part) {
    if (!((B.vmask[C / 32] >> (C % 32)) & 1)) return;
    const uint32_t n = B.ulen[U];
    E.put(n, 4);
    if (MJE_ABL_NOSTR) return;
    const Col c = tcol<C>(B.t);
    const uintptr_t sa_ptr = (uintptr_t)(gp(c.values) + B.ustart[U]);
    const uint32_t sa = (uint32_t)(sa_ptr & 3);
    if constexpr (SBW > 0) {
        // the string's aligned dwords from the wave's LDS copy of its range,
        // or (a wave whose ranges did not fit) from HBM
        if (S.on) {
            emit_str(E, (const LAS uint32_t*)(part + S.base[U] + (uint32_t)((uint64_t)(sa_ptr - sa) - S.g0[U])), n, sa);
        } else {
            emit_str(E, (const GAS uint32_t*)(sa_ptr - sa), n, sa);
        }
        return;
    }
    const GAS uint32_t* w = (const GAS uint32_t*)(sa_ptr - sa);
    // chunk q = string bytes [4q, 4q + 4) = alignbyte(w[q + 1], w[q], sa)
#pragma unroll
    for (uint32_t q = 0; q + 1 < PF; q++)
        if (4 * q < n) E.put(__builtin_amdgcn_alignbyte(B.pre[U][q + 1], B.pre[U][q], sa), umin(4u, n - 4 * q));
    uint32_t cur = B.pre[U][PF - 1];
    for (uint32_t q = PF - 1; 4 * q < n; q += 4) {
        uint32_t x[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) x[k] = 4 * (q + 1 + k) < n + sa ? w[q + 1 + k] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
            if (4 * (q + k) < n) E.put(__builtin_amdgcn_alignbyte(x[k], k ? x[k - 1] : cur, sa), umin(4u, n - 4 * (q + k)));
        cur = x[3];
    }
}

}  // namespace mje

// MJE_WPE (tuning): a register budget admitting that many waves per SIMD.
#if defined(MJE_WPE) && MJE_WPE
#define MJE_WPE_ATTR __attribute__((amdgpu_waves_per_eu(MJE_WPE)))
#else
#define MJE_WPE_ATTR
#endif
// A workgroup per tile: workgroup g runs on XCD (g + c) % 8 for a launch-wide
// c, so tiles dealt in index order put neighbouring tiles -- whose output
// spans share a partial line at each end -- on different XCDs.  Runs of
// MJE_XRUN consecutive tiles can go to workgroups of one XCD instead (a
// bijection on the first multiple of 8 * MJE_XRUN tiles; the rest as is).
// Tuning only: neutral on the config B and C column sets, config E 0.335 vs
// 0.323 ms at runs of 8 (profiles/r04/probes/ab23.txt), so off.
#ifndef MJE_XRUN
#define MJE_XRUN 1
#endif
#ifndef MJE_CHECK
#define MJE_CHECK 0
#endif
namespace mje {
DEV bool sizes_inline() {
    bool ok = true;
#define MJE_NOVAL(C, KIND, SOFF, U) if (KIND == 0) ok = ok && ((const CAS Col*)args()->cols + C)->validity == nullptr;
    MJE_COLS(MJE_NOVAL)
#undef MJE_NOVAL
    return ok;
}
}  // namespace mje
namespace mje {
DEV uint64_t tile_of(uint64_t g, uint64_t total) {
    if (MJE_XRUN <= 1 || gridDim.x != total) return g;
    constexpr uint64_t R = MJE_XRUN, P = 8 * R;
    if (g >= total / P * P) return g;
    const uint64_t x = g % 8, r = g / 8;  // XCD slot, rank on that XCD
    return (r / R) * P + x * R + (r % R);
}
}  // namespace mje

extern "C" __global__ void __launch_bounds__(MJE_TILE) MJE_WPE_ATTR murr_jit_encode(mje::Args) {
    using namespace mje;
    __shared__ __attribute__((aligned(16))) uint32_t stage[STAGE / 4 + 8];
    __shared__ __attribute__((aligned(16))) uint8_t sstr[SBW ? NWAVE * SBW : 16];
    __shared__ uint64_t s_w[8];
    LAS uint32_t* stw = (LAS uint32_t*)stage;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const CAS Args* A = args();
    const uint64_t n_rows = A->n_rows, total_tiles = A->total_tiles, out_cap = A->out_cap;

    const ColTab tab = load_tab(lane);
    // estimated tile sizes to check: only with a utf8 validity buffer (the
    // prelude's MJE_CHECK; code in the loop costs layouts without one ~10 %,
    // profiles/r04/probes/ab46.txt)
    constexpr bool chk = MJE_CHECK != 0 && NUTF8 > 0;
    for (uint64_t t0 = blockIdx.x; t0 < total_tiles; t0 += gridDim.x) {
        const uint64_t t = tile_of(t0, total_tiles);
        const uint64_t r0 = t * TILE;
        const uint32_t nr = (uint32_t)min((uint64_t)TILE, n_rows - r0);
        const bool active = tid < nr;
        const uint64_t row = r0 + (active ? tid : 0u);
        // the tile's start (murr_jit_encode_sizes + murr_jit_encode_scan left the
        // exclusive prefix of the tile totals in lookback[t]), loaded up front
        // (checked layouts load it and the next tile's start -- where this one
        // must end, see tile_bytes_inline -- by scalar loads: written by the
        // scan's launch before this one.  Measured per layout: config C 0.933
        // vs 0.970 ms scalar, config B, unchecked, 0.232 vs 0.212 ms vector;
        // profiles/r04/probes/ab47.txt, ab48.txt)
        const uint64_t t_pre = NUTF8 == 0 ? 0
                               : chk      ? ((const CAS uint64_t*)A->lookback)[t]
                                          : ((const GAS uint64_t*)A->lookback)[t];
        const uint64_t t_nxt = chk && t + 1 < total_tiles ? ((const CAS uint64_t*)A->lookback)[t + 1] : 0;

        RowBuild B;
        B.t = tab;
#pragma unroll
        for (uint32_t k = 0; k <= NR; k++) B.r.w[k] = 0;
#pragma unroll
        for (uint32_t k = 0; k < sizeof(B.vmask) / 4; k++) B.vmask[k] = 0;
        B.pos = FIXED;
        const uint64_t rw = r0 + 64 * wave;
#define MJE_DO_OFFS(C, KIND, SOFF, U) ld_offs<C, KIND, SOFF, U>(B, row);
        MJE_COLS(MJE_DO_OFFS)
#undef MJE_DO_OFFS
        const Bits bits = load_bits(rw, lane, tab);
        // the wave's string ranges into LDS (issued before the fixed-width
        // loads, so the compiler's counted waits for those cover them too)
        StrStage S;
        LAS uint8_t* part = (LAS uint8_t*)sstr + (SBW ? wave * SBW : 0u);
        S.on = SBW > 0 && rw < n_rows;
        if (SBW > 0 && S.on) {
            const uint32_t nact = (uint32_t)min((uint64_t)64, n_rows - rw);
            uint32_t at = 0;
#define MJE_DO_STAGE(C, KIND, SOFF, U) stage_col<C, KIND, SOFF, U>(B, part, nact, lane, at, S);
            MJE_COLS(MJE_DO_STAGE)
#undef MJE_DO_STAGE
        }
#define MJE_DO_FIXED(C, KIND, SOFF, U) ld_fixed<C, KIND, SOFF, U>(B, row);
        MJE_COLS(MJE_DO_FIXED)
#undef MJE_DO_FIXED
#define MJE_DO_STR(C, KIND, SOFF, U) ld_str<C, KIND, SOFF, U>(B, rw, lane, bits, S.on);
        MJE_COLS(MJE_DO_STR)
#undef MJE_DO_STR
#define MJE_DO_PUT(C, KIND, SOFF, U) put_col<C, KIND, SOFF, U>(B, rw, lane, bits);
        MJE_COLS(MJE_DO_PUT)
#undef MJE_DO_PUT
        put_bitset(B);
        const uint32_t size = active ? B.pos : 0u;

        uint64_t start, tstart, span;
        if (NUTF8 == 0) {
            start = (r0 + tid) * (uint64_t)FIXED;
            tstart = r0 * (uint64_t)FIXED;
            span = (uint64_t)nr * FIXED;
        } else {
            // block scan of the row sizes, then the window prefix
            const uint32_t inc = wave_scan(size);
            if (lane == 63) s_w[wave] = inc;
            __syncthreads();
            uint64_t before = 0, agg = 0;
#pragma unroll
            for (uint32_t w = 0; w < NWAVE; w++) {
                const uint64_t v = s_w[w];
                before += w < wave ? v : 0u;
                agg += v;
            }
            __syncthreads();
            tstart = t_pre;
            start = tstart + before + inc - size;
            span = agg;
            if (chk && t + 1 < total_tiles && tstart + span != t_nxt) {
                if (tid == 0) report(A->err, err_key(0, r0, 0, kStRecount));
            }
        }
        if (active) {
            gp(A->row_off)[row] = A->row_base + start;
            if (row + 1 == n_rows) gp(A->row_off)[row + 1] = A->row_base + start + size;
        }
        if (tstart + span > out_cap) {
            if (tid == 0) report(A->err, err_key(0, r0, 0, kStCapacity));
            continue;  // uniform
        }
        if (span <= STAGE) {
            // merge the rows (every byte of the span is some row's: no zeroing
            // in stream mode), write it out
            if (!MJE_STREAM || MJE_ZERO) {  // (tuning: the OR-merge path)
                for (uint32_t k = tid; k < (uint32_t)((span + 7) >> 2) + 1; k += TILE) stw[k] = 0;
                __syncthreads();
            }
#if MJE_STREAM
            if (SBW > 0 && S.on) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wave's string DMA landed
            if (active && NUTF8) {
                Emit E;
                E.start(stw, (uint32_t)(start - tstart));
#pragma unroll
                for (uint32_t k = 0; k < NR; k++) E.put(B.r.w[k], k + 1 < NR ? 4u : FIXED - 4 * (NR - 1));
#define MJE_DO_EMIT(C, KIND, SOFF, U) if (KIND == 0) emit_payload<C, U>(B, E, S, part);
                MJE_COLS(MJE_DO_EMIT)
#undef MJE_DO_EMIT
                E.finish();
            } else
#endif
            if (active) {
                const uint32_t rb = (uint32_t)(start - tstart), sh = rb & 3u, d0 = rb >> 2;
#pragma unroll
                for (uint32_t k = 0; k <= NR; k++) {
                    const uint32_t cur = B.r.w[k], prev = k ? B.r.w[k - 1] : 0u;
                    const uint32_t v = sh ? __builtin_amdgcn_alignbyte(cur, prev, 4 - sh) : cur;
                    // dwords wholly inside the fixed part are this row's alone
                    if (k >= 1 && 4 * k + 4 <= FIXED + sh) stw[d0 + k] = v;
                    else if (MJE_STREAM && !NUTF8) {  // an edge shared with a neighbour: this row's bytes only
                        if (FIXED + sh > 4 * k) put_bytes(stw, d0 + k, v, k ? 0u : sh, FIXED + sh - 4 * k);
                    } else if (v) {
                        __hip_atomic_fetch_or(stw + d0 + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if (NUTF8) {
                    uint32_t p = FIXED;
#define MJE_DO_PAY(C, KIND, SOFF, U) if (KIND == 0) put_payload<C, U>(B, stw, rb, p);
                    MJE_COLS(MJE_DO_PAY)
#undef MJE_DO_PAY
                }
            }
            __syncthreads();
            if (!MJE_ABL_NOOUT) write_out((const LAS uint8_t*)stage, gp(A->out), tstart, span, tid);
            __syncthreads();
        } else if (active) {
            // a tile over the stage: bytes straight to HBM (cold)
            GAS uint8_t* o = gp(A->out) + start;
            for (uint32_t b = 0; b < FIXED; b++) o[b] = (uint8_t)(B.r.w[b >> 2] >> (8 * (b & 3)));
            if (NUTF8) {
                uint32_t p = FIXED;
#define MJE_DO_PAYG(C, KIND, SOFF, U)                                                   \
    if (KIND == 0 && ((B.vmask[C / 32] >> (C % 32)) & 1)) {                             \
        const uint32_t n = B.ulen[U];                                                   \
        for (uint32_t b = 0; b < 4; b++) o[p + b] = (uint8_t)(n >> (8 * b));            \
        const GAS uint8_t* s = gp(tcol<C>(B.t).values) + B.ustart[U];                       \
        for (uint32_t b = 0; b < n; b++) o[p + 4 + b] = s[b];                           \
        p += 4 + n;                                                                     \
    }
                MJE_COLS(MJE_DO_PAYG)
#undef MJE_DO_PAYG
            }
        }
    }
}

// Row sizes of each tile: bs + cap + sum over non-null utf8 of (4 + len),
// summed into lookback[t] (the Arrow validity and offsets only).
extern "C" __global__ void __launch_bounds__(MJE_TILE) murr_jit_encode_sizes(mje::Args) {
    using namespace mje;
    __shared__ uint64_t s_w[NWAVE];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const CAS Args* A = args();
    const uint64_t n_rows = A->n_rows, total_tiles = A->total_tiles;
    for (uint64_t t = blockIdx.x; t < total_tiles; t += gridDim.x) {
        const uint64_t row = t * TILE + tid;
        uint64_t size = 0;
        if (row < n_rows) {
            size = FIXED;
#define MJE_DO_SIZE(C, KIND, SOFF, U)                                                        \
            if (KIND == 0) {                                                                 \
                const Col c = ldcol(C);                                                      \
                const uint64_t e = c.offset + row;                                           \
                const uint32_t l = (uint32_t)(gp(c.offsets)[e + 1] - gp(c.offsets)[e]);      \
                const uint64_t ew = c.offset + t * TILE + 64 * wave;                         \
                if (valid_wave(c, ew, lane, (c.offset + n_rows + 7) >> 3)) size += 4 + l;    \
            }
            MJE_COLS(MJE_DO_SIZE)
#undef MJE_DO_SIZE
        }
        for (int m = 32; m >= 1; m >>= 1) size += (uint64_t)__shfl_xor((unsigned long long)size, m, 64);
        if (lane == 0) s_w[wave] = size;
        __syncthreads();
        if (tid == 0) {
            uint64_t tot = 0;
#pragma unroll
            for (uint32_t w = 0; w < NWAVE; w++) tot += s_w[w];
            gp(A->lookback)[t] = tot;
        }
        __syncthreads();
    }
}

// Tile totals without the sizes pass.  When no utf8 column has a validity
// buffer every row carries every payload, so a tile of nr rows holds
// nr (FIXED + 4 NUTF8) bytes plus its string bytes: two offsets per column
// (the host skips murr_jit_encode_sizes on the same condition).  With
// validity buffers (`spec`), a tile holds nr FIXED bytes plus, per utf8
// column, 4 bytes per valid row and the offsets' span -- exact when every
// null string is empty, as Arrow writers leave them; the encode kernel checks
// each tile's exact size against this estimate (kStRecount) and the host
// recounts with the sizes pass when any differs.
namespace mje {
// Set bits of bitmap bm in [b0, b0 + n): dword loads from bm's aligned
// base, never past the byte holding bit b0 + n - 1.
DEV uint32_t popc_bits(const uint8_t* bm, uint64_t b0, uint32_t n) {
    const uint32_t mis = (uint32_t)((uintptr_t)bm & 3u);
    const GAS uint32_t* p = (const GAS uint32_t*)(bm - mis);
    const uint64_t s = b0 + 8 * mis, e = s + n, lim = (b0 + n + 7) / 8 + mis;  // bytes readable from p
    uint32_t cnt = 0;
    for (uint64_t w = s >> 5; w < (e + 31) >> 5; w++) {
        uint32_t v = 0;
        if (4 * w + 4 <= lim) {
            v = p[w];
        } else {
            for (uint32_t k = 0; k < 4; k++)
                if (4 * w + k < lim) v |= (uint32_t)((const GAS uint8_t*)p)[4 * w + k] << (8 * k);
        }
        uint32_t m = ~0u;
        if (w == (s >> 5)) m &= ~0u << (s & 31);
        if (w == ((e - 1) >> 5) && (e & 31)) m &= ~0u >> (32 - (e & 31));
        cnt += __popc(v & m);
    }
    return cnt;
}
// Totals of the N consecutive tiles t0 .. t0 + N - 1 (those below hi); each
// column's descriptor is read once, every offset load issued together.
template <uint32_t N> DEV void tile_bytes_inline(uint64_t t0, uint64_t hi, uint64_t (&x)[N]) {
    const uint64_t n_rows = args()->n_rows;
    uint64_t nr[N];
#pragma unroll
    for (uint32_t q = 0; q < N; q++) {
        const uint64_t r0 = (t0 + q) * TILE;
        nr[q] = t0 + q < hi ? min((uint64_t)TILE, n_rows - r0) : 0;
        x[q] = nr[q] * FIXED;
    }
#define MJE_TB(C, KIND, SOFF, U)                                                            \
    if (KIND == 0) {                                                                        \
        const Col c = ldcol(C);                                                             \
        _Pragma("unroll") for (uint32_t q = 0; q < N; q++) {                                \
            const uint64_t e = c.offset + (t0 + q) * TILE;                                  \
            if (nr[q]) {                                                                    \
                const uint32_t nv = c.validity ? popc_bits(c.validity, e, (uint32_t)nr[q]) : (uint32_t)nr[q]; \
                x[q] += 4ull * nv + (uint64_t)(int64_t)(gp(c.offsets)[e + nr[q]] - gp(c.offsets)[e]); \
            }                                                                               \
        }                                                                                   \
    }
    MJE_COLS(MJE_TB)
#undef MJE_TB
}
}  // namespace mje

// Exclusive prefix of the tile totals in place, in two launches of this
// kernel over contiguous ranges of SCAN_PER tiles per workgroup: pass 0 (or
// 3) sums each range into lookback[T + 1 + g]; pass 4 adds up the sums of the
// ranges before its own (a few hundred at most) and rewrites its range as
// its exclusive prefix.  (Passes 2 + 1: the same with a one-workgroup scan of
// the sums in between, a third launch; tuning MURR_ENC_SCAN3.)
#ifndef MJE_SCAN_PER
#define MJE_SCAN_PER 1024
#endif
constexpr uint32_t SCAN_PER = MJE_SCAN_PER;
static_assert(SCAN_PER % 1024 == 0, "whole threads per tile group");
DEV uint64_t block_excl(uint64_t x, LAS uint64_t* s_t, uint64_t* total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t inc = x;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t y = (uint64_t)__shfl_up((unsigned long long)inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) s_t[wave] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
    for (uint32_t w = 0; w < 16; w++) {
        const uint64_t v = s_t[w];
        before += w < wave ? v : 0u;
        all += v;
    }
    __syncthreads();
    *total = all;
    return before + inc - x;
}
extern "C" __global__ void __launch_bounds__(1024) murr_jit_encode_scan(mje::Args, uint32_t pass) {
    using namespace mje;
    __shared__ uint64_t s_t[16];
    const uint32_t tid = threadIdx.x;
    const CAS Args* A = args();
    GAS uint64_t* v = gp(A->lookback);
    const uint64_t T = A->total_tiles;
    GAS uint64_t* sums = v + T + 1;
    const uint64_t ngroups = (T + SCAN_PER - 1) / SCAN_PER;
    if (pass == 2) {  // one workgroup: exclusive scan of the group sums, 1024 at a time
        uint64_t carry = 0;
        for (uint64_t g0 = 0; g0 < ngroups; g0 += 1024) {
            const uint64_t g = g0 + tid;
            const uint64_t x = g < ngroups ? sums[g] : 0;
            uint64_t tot;
            const uint64_t ex = block_excl(x, (LAS uint64_t*)s_t, &tot);
            if (g < ngroups) sums[g] = carry + ex;
            carry += tot;
        }
        return;
    }
    const uint64_t g = blockIdx.x, lo = g * SCAN_PER, hi = min(T, lo + SCAN_PER);
    constexpr uint32_t PER = SCAN_PER / 1024;  // 4 per thread, contiguous
    uint64_t x[PER], s = 0;
    if (pass == 3 || (pass == 0 && sizes_inline())) {
        // tile totals from the offsets (no sizes pass; pass 3: estimates,
        // checked by the encode kernel), kept for pass 1
        tile_bytes_inline<PER>(lo + tid * PER, hi, x);
#pragma unroll
        for (uint32_t q = 0; q < PER; q++)
            if (lo + tid * PER + q < hi) v[lo + tid * PER + q] = x[q];
    } else {
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint64_t j = lo + tid * PER + q;
            x[q] = j < hi ? v[j] : 0;
        }
    }
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) s += x[q];
    uint64_t tot;
    const uint64_t ex = block_excl(s, (LAS uint64_t*)s_t, &tot);
    if (pass == 0 || pass == 3) {
        if (tid == 0) sums[g] = tot;
        return;
    }
    uint64_t run = ex;
    if (pass == 1) {
        run += sums[g];
    } else {  // pass 4: the ranges before this one
        for (uint64_t k0 = 0; k0 < g; k0 += 1024) {
            uint64_t t2;
            (void)block_excl(k0 + tid < g ? sums[k0 + tid] : 0, (LAS uint64_t*)s_t, &t2);
            run += t2;
        }
    }
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) {
        const uint64_t j = lo + tid * PER + q;
        if (j < hi) v[j] = run;
        run += x[q];
    }
}
