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
constexpr uint32_t kWaveBuf = 2048;  // bytes of strings one wave assembles per 64-row chunk
constexpr uint32_t kSpinLimit = 1u << 22;
enum : uint32_t { kStUtf8 = 1, kStOverflow = 4, kStMalformed = 5, kStCapacity = 6, kStInternal = 10 };

__device__ __forceinline__ void report(unsigned long long* err, uint64_t key) {
    __hip_atomic_fetch_max(gp(err), (unsigned long long)~key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- byte sources: LDS stage (aligned dword reads, padded) or HBM ---------
struct LdsSrc {
    const uint8_t* s;  // LDS, 16-B aligned, >= 16 B of padding past the data
    __device__ __forceinline__ uint32_t u32(uint32_t a) const {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (a & ~3u));
        return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
    }
    __device__ __forceinline__ uint64_t u64(uint32_t a) const {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (a & ~3u));
        uint32_t sh = a & 3u, w0 = w[0], w1 = w[1], w2 = w[2];
        return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) |
               ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    }
    __device__ __forceinline__ uint32_t u8(uint32_t a) const { return s[a]; }
};

struct GlbSrc {
    const GAS uint8_t* g;  // HBM (16-B aligned); never reads a dword holding no requested byte
    __device__ __forceinline__ uint32_t u32(uint32_t a) const {
        const GAS uint32_t* w = reinterpret_cast<const GAS uint32_t*>(g + (a & ~3u));
        const uint32_t sh = a & 3u;
        return sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
    }
    __device__ __forceinline__ uint64_t u64(uint32_t a) const {
        return (uint64_t)u32(a) | ((uint64_t)u32(a + 4) << 32);
    }
    __device__ __forceinline__ uint32_t u8(uint32_t a) const { return g[a]; }
};

// Read W (1,2,4,8) little-endian bytes at a.
template <class Src, class Addr>
__device__ __forceinline__ uint64_t read_w(const Src& s, Addr a, uint32_t w) {
    if (w == 8) return s.u64(a);
    if (w == 4) return s.u32(a);
    if (w == 2) return s.u8(a) | (s.u8(a + 1) << 8);
    return s.u8(a);
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
// Diagnostic phase stamps (MURR_DEBUG_DECODE & 8): thread 0 of each workgroup
// adds s_memtime deltas into s_st[j]; s_st[7] holds the last stamp.
__device__ __forceinline__ void dstamp(const DecodeArgs& A, uint64_t* s_st, int j) {
    if ((A.debug & 8) && threadIdx.x == 0) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        s_st[j] += t - s_st[7];
        s_st[7] = t;
    }
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
__device__ uint64_t window_prefix(const uint64_t* st, uint64_t lo, uint64_t t, uint64_t base,
                                  uint64_t* s_w, unsigned long long* err, uint64_t ekey) {
    constexpr int K = 4;  // granules per thread per pass: 1024 predecessors
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t sum = 0;
    for (uint64_t j0 = lo; j0 < t; j0 += 256 * K) {
        uint64_t v[K];
#pragma unroll
        for (int i = 0; i < K; i++) {  // every load in flight before the first check
            const uint64_t j = j0 + i * 256 + tid;
            v[i] = j < t ? __hip_atomic_load(gp(st) + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1;
        }
#pragma unroll
        for (int i = 0; i < K; i++) {
            const uint64_t j = j0 + i * 256 + tid;
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
    const uint64_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
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
__device__ __forceinline__ void write_out(const uint8_t* buf, GAS uint8_t* out, uint64_t g0,
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
    const uint32_t* w = reinterpret_cast<const uint32_t*>(buf);
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
// bytes, global_load_lds_dwordx4, 1 KiB per wave-instruction), and tile i+2's
// blob span is loaded, so HBM stays busy while tile i is decoded from LDS:
//   A: utf8 lengths per 64-row chunk -> chunk prefixes; tile aggregate published
//   F: validity of every column (__ballot words), fixed-width and bool values
//   B: per utf8 column: cross-tile prefix (window_prefix), i32 offsets, string
//      bytes assembled per wave in LDS and stored 16 B wide, UTF-8 validated.
// Row state (offsets) is re-read from the staged slice, so the row loops stay
// rolled and the register budget small.
// Descriptor tables are wave-uniform: read them through the constant address
// space so they become s_load (lgkmcnt) instead of vector loads whose vmcnt
// waits would drain the LDS-DMA in flight (vmcnt retires in order).
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
    L.pre = 0;
    L.rowoff = ((8 * nutf8 * (R / 64 + 1) + 15) & ~15u);
    L.stage = L.rowoff + ((8 * (R + 1) + 16 + 15) & ~15u);
    L.bytes = L.stage + stage + 32;
    return L;
}

// read_dynamic (read.rs:45-55) for one non-null cell: string length and
// payload address; a slice the reference would panic on -> *bad.
template <class Src>
__device__ __forceinline__ uint32_t utf8_cell(const Src& src, uint32_t ra, uint32_t rl, uint32_t bs,
                                              uint32_t fo, uint32_t* pay, bool* bad) {
    *bad = false;
    *pay = 0;
    if (fo + 4 > rl) { *bad = true; return 0; }
    const uint32_t vlen = rl - bs;  // static + payload region
    const uint32_t prel = src.u32(ra + fo);
    if ((uint64_t)prel + 4 > vlen) { *bad = true; return 0; }
    const uint32_t l = src.u32(ra + bs + prel);
    if ((uint64_t)prel + 4 + l > vlen) { *bad = true; return 0; }
    *pay = ra + bs + prel + 4;
    return l;
}

// Tile t's rows and blob span (b: this workgroup's current block, monotone).
__device__ __forceinline__ DecTile tile_info(const DecodeArgs& A, uint64_t t, uint32_t* b) {
    DecTile T;
    T.t = t;
    T.ok = 0;
    if (t >= A.total_tiles) return T;
    while (*b + 1 < A.nblocks && ldblk(A, *b + 1).tile_base <= t) (*b)++;
    const DecBlock blk = ldblk(A, *b);
    T.b = *b;
    T.tfirst = blk.tile_base;
    T.r0 = (t - blk.tile_base) * A.rows_per_tile;
    T.nr = (uint32_t)min((uint64_t)A.rows_per_tile, blk.n_rows - T.r0);
    T.last = T.r0 + T.nr == blk.n_rows;
    // Scalar loads (constant address space -> s_load, counted by lgkmcnt): they
    // must not queue behind the LDS-DMA on vmcnt, which is in order.
    const CAS uint64_t* ro = (const CAS uint64_t*)(blk.row_off + T.r0);
    T.base = ro[0];
    T.end = ro[T.nr];
    T.abase = T.base & ~15ull;
    T.ok = 1;
    return T;
}

// Issue tile T's LDS-DMA: row-offset slice [r0, r0+nr] and, when it fits the
// stage, the blob span rounded out to 16-B granules (never past the granule
// holding the last byte, so never past the allocation).  No waits here.
__device__ __forceinline__ void issue_stage(const DecodeArgs& A, const DecTile& T, uint8_t* buf,
                                            const DecLayout& L) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const GAS uint64_t* ro = gp(ldblk(A, T.b).row_off) + T.r0;
    const uintptr_t s0 = (uintptr_t)ro & ~(uintptr_t)15;
    const uint32_t nb_off = (uint32_t)((((uintptr_t)ro - s0) + (uint64_t)(T.nr + 1) * 8 + 15) & ~15ull);
    const GAS uint8_t* go = (const GAS uint8_t*)s0;
    for (uint32_t c = wave; c * 1024 < nb_off; c += 4) {
        const uint32_t off = c * 1024 + lane * 16;
        if (off < nb_off)
            __builtin_amdgcn_global_load_lds((const GAS void*)(go + off), (LAS void*)(buf + L.rowoff + c * 1024),
                                             16, 0, 0);
    }
    const uint64_t span = ((T.end + 15) & ~15ull) - T.abase;
    if (span <= A.stage) {
        const GAS uint8_t* g = gp(ldblk(A, T.b).data) + T.abase;
        const uint32_t nb = (uint32_t)span;
        for (uint32_t c = wave; c * 1024 < nb; c += 4) {
            const uint32_t off = c * 1024 + lane * 16;
            if (off < nb)
                __builtin_amdgcn_global_load_lds((const GAS void*)(g + off), (LAS void*)(buf + L.stage + c * 1024),
                                                 16, 0, 0);
        }
    }
}

// Tile bytes live in LDS (staged) or, for a tile larger than the stage, in
// HBM.  One decoder serves both through a wave-uniform branch per access, so
// the kernel carries one copy of the tile code (code size is what bounds it:
// two inlined copies of this decoder did not fit the instruction cache).
struct TileSrc {
    const uint8_t* l;      // LDS stage
    const GAS uint8_t* g;  // HBM, 16-B aligned tile start
    bool lds;
    __device__ __forceinline__ uint32_t u8(uint32_t a) const { return lds ? (uint32_t)l[a] : (uint32_t)g[a]; }
    __device__ __forceinline__ uint32_t u32(uint32_t a) const {
        return lds ? LdsSrc{l}.u32(a) : GlbSrc{g}.u32(a);
    }
    __device__ __forceinline__ uint64_t u64(uint32_t a) const {
        return lds ? LdsSrc{l}.u64(a) : GlbSrc{g}.u64(a);
    }
};

// UTF-8 validation of one string, out of line (rarely the hot path: the
// caller skips strings whose bytes are all ASCII).
__device__ __attribute__((noinline)) bool utf8_valid_slow(TileSrc src, uint32_t at, uint32_t n) {
    Utf8Dfa dfa;
    for (uint32_t q = 0; q < n; q++) dfa.step(src.u8(at + q));
    return dfa.ok();
}

// read_dynamic (read.rs:45-55) for one cell: string length (0 for NULL /
// absent rows) and payload address; *bad = a slice the reference would panic on.
__device__ __forceinline__ uint32_t utf8_cell_ts(const TileSrc& src, uint32_t ra, uint32_t rl, uint32_t bs,
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

__device__ __attribute__((noinline)) uint64_t window_prefix_ni(const uint64_t* st, uint64_t lo, uint64_t t,
                                                              uint64_t base, uint64_t* s_w,
                                                              unsigned long long* err, uint64_t ekey) {
    return window_prefix(st, lo, t, base, s_w, err, ekey);
}

__device__ __forceinline__ void decode_tile(const DecodeArgs& A, const TileSrc& src, const DecTile& T,
                                            uint8_t* buf, const DecLayout& L, uint32_t* s_nulls,
                                            uint64_t* s_w, uint8_t* s_wbuf, const DecProj* s_proj,
                                            const DecOut* s_out, uint64_t* s_mine, uint64_t* s_st) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t bs = A.bs, R = A.rows_per_tile;
    const uint64_t* rowoff = reinterpret_cast<const uint64_t*>(
        buf + L.rowoff + (((uintptr_t)(ldblk(A, T.b).row_off + T.r0)) & 15));
    uint64_t* pre = reinterpret_cast<uint64_t*>(buf + L.pre);
    const uint32_t nchunk = (T.nr + 63) / 64;
    const uint32_t nk = (T.nr + 255) / 256;

    // row i of the tile: blob offset (relative to abase), length (0 = absent),
    // null bitset (cached when bs <= 4; ~0 when the row is absent / too short)
    auto row_at = [&](uint32_t i, uint32_t* ra, uint32_t* rl, uint32_t* bits) {
        const uint32_t ic = i < T.nr ? i : T.nr - 1;
        const uint64_t a = rowoff[ic], z = rowoff[ic + 1];
        *ra = (uint32_t)(a - T.abase);
        *rl = i < T.nr ? (uint32_t)(z - a) : 0;
        const bool ok = *rl >= bs && *rl > 0;
        uint32_t bv = ~0u;
        if (ok && bs <= 4) {
            bv = 0;
            for (uint32_t q = 0; q < bs; q++) bv |= src.u8(*ra + q) << (8 * q);
        }
        *bits = bv;
    };
    auto null_of = [&](uint32_t ra, uint32_t rl, uint32_t bits, uint32_t bit) -> bool {
        if (bs <= 4) return (bits >> bit) & 1;
        return !(rl >= bs && rl > 0) || ((src.u8(ra + (bit >> 3)) >> (bit & 7)) & 1);
    };

    // ---- phase A: utf8 chunk totals -> chunk prefixes, aggregate published ----
    if (A.nutf8) {
#pragma unroll 1
        for (uint32_t k = 0; k < nk; k++) {
            uint32_t ra, rl, bits;
            row_at(k * 256 + tid, &ra, &rl, &bits);
            const uint32_t c = k * 4 + wave;
            for (uint32_t p = 0; p < A.nproj; p++) {
                const DecProj pc = s_proj[p];
                if (!pc.is_utf8) continue;
                uint32_t pay;
                bool bad;
                const uint32_t slen = utf8_cell_ts(src, ra, rl, bs, bs + pc.offset, !null_of(ra, rl, bits, pc.bit),
                                                   &pay, &bad);
                const uint32_t tot = wave_total_u32(slen);  // < tile span < 4 GiB
                if (lane == 0 && c < nchunk) pre[pc.uslot * (R / 64 + 1) + c] = tot;
            }
        }
        lds_barrier();
        if (tid < A.nutf8) {  // chunk totals -> exclusive prefixes (+ aggregate at [nchunk])
            uint64_t* pu = pre + tid * (R / 64 + 1);
            uint64_t run = 0;
            for (uint32_t c = 0; c < nchunk; c++) {
                const uint64_t v = pu[c];
                pu[c] = run;
                run += v;
            }
            pu[nchunk] = run;
            publish(A.lookback + (uint64_t)tid * A.total_tiles + T.t, run + 1);
        }
    }
    dstamp(A, s_st, 2);

    // ---- phase F: validity of every column, fixed-width and bool values -----
#pragma unroll 1
    for (uint32_t k = 0; k < nk; k++) {
        const uint32_t i = k * 256 + tid;
        const bool act = i < T.nr;
        uint32_t ra, rl, bits;
        row_at(i, &ra, &rl, &bits);
        const uint64_t row = T.r0 + i;
        if (rl && rl < bs) report(A.err, err_key(T.b, row, 0, kStMalformed));  // split_at panics
        const bool live = k * 256 + wave * 64 < T.nr;
        const uint64_t word = ((T.r0 + k * 256) >> 6) + wave;
        for (uint32_t p = 0; p < A.nproj; p++) {
            const DecProj pc = s_proj[p];
            const DecOut o = s_out[p];
            const bool isnull = null_of(ra, rl, bits, pc.bit);
            const uint64_t vm = __ballot(act && !isnull);
            const uint32_t nnull = __popcll(__ballot(act && isnull));
            if (lane == 0 && nnull) atomicAdd(&s_nulls[p], nnull);  // LDS
            if (lane == 0 && live) reinterpret_cast<GAS uint64_t*>(gp(o.validity))[word] = vm;
            if (pc.is_utf8) continue;
            const uint32_t fo = bs + pc.offset;
            bool fnull = isnull;
            if (!fnull && fo + pc.width > rl) {
                report(A.err, err_key(T.b, row, p, kStMalformed));
                fnull = true;
            }
            if (pc.dtype == kBool) {
                const bool v = !fnull && src.u8(ra + fo) != 0;
                const uint64_t m = __ballot(act && v);
                if (lane == 0 && live) reinterpret_cast<GAS uint64_t*>(gp(o.values))[word] = m;
            } else if (act) {
                const uint64_t v = fnull ? 0 : read_w(src, ra + fo, pc.width);
                GAS uint8_t* dst = gp(o.values) + row * pc.width;
                switch (pc.width) {
                case 8: *reinterpret_cast<GAS uint64_t*>(dst) = v; break;
                case 4: *reinterpret_cast<GAS uint32_t*>(dst) = (uint32_t)v; break;
                case 2: *reinterpret_cast<GAS uint16_t*>(dst) = (uint16_t)v; break;
                default: *dst = (uint8_t)v; break;
                }
            }
        }
    }
    dstamp(A, s_st, 3);
    if (!A.nutf8) return;

    // ---- phase B: cross-tile prefix, offsets, string bytes -------------------
    uint8_t* wb = s_wbuf + wave * (kWaveBuf + 32);
    for (uint32_t p = 0; p < A.nproj; p++) {
        const DecProj pc = s_proj[p];
        if (!pc.is_utf8) continue;
        const DecOut o = s_out[p];
        const uint64_t* pu = pre + pc.uslot * (R / 64 + 1);
        const uint64_t agg = pu[nchunk];
        // this workgroup's own inclusive prefix of tile t - G (same block) or 0
        uint64_t* mine = s_mine + pc.uslot;
        const uint64_t G = gridDim.x;
        const bool have_prev = T.t >= T.tfirst + G;
        const uint64_t lo = have_prev ? T.t - G + 1 : T.tfirst;
        const uint64_t* st = A.lookback + (uint64_t)pc.uslot * A.total_tiles;
        const uint64_t prefix = (A.debug & 2) ? 0 : window_prefix_ni(st, lo, T.t, have_prev ? *mine : 0, s_w, A.err,
                                                                  err_key(T.b, T.r0, p, 0));
        if (tid == 0) {
            *mine = prefix + agg;
            if (T.t == T.tfirst) gp(o.offsets)[0] = 0;
            if (T.last) gp(A.lens)[(uint64_t)T.b * A.nproj + p] = prefix + agg;
        }
        const uint32_t fo = bs + pc.offset;
#pragma unroll 1
        for (uint32_t k = 0; k < nk; k++) {
            const uint32_t i = k * 256 + tid;
            const bool act = i < T.nr;
            uint32_t ra, rl, bits, pay;
            bool bad;
            row_at(i, &ra, &rl, &bits);
            const uint32_t slen = utf8_cell_ts(src, ra, rl, bs, fo, !null_of(ra, rl, bits, pc.bit), &pay, &bad);
            const uint64_t row = T.r0 + i;
            if (bad) report(A.err, err_key(T.b, row, p, kStMalformed));
            const uint64_t inc = wave_scan_u32(slen);  // < tile span < 4 GiB
            const uint32_t c = k * 4 + wave;
            const bool live = c < nchunk;
            const uint64_t ws = prefix + (live ? pu[c] : 0);      // this wave chunk's output start
            const uint64_t wn = live ? pu[c + 1] - pu[c] : 0;      // and its byte count
            const uint64_t end = ws + inc, d0 = end - slen;
            if (act) {
                if (end > 0x7FFFFFFFull) report(A.err, err_key(T.b, row, p, kStOverflow));
                else gp(o.offsets)[row + 1] = (int32_t)end;
                if (slen && end > o.values_cap) report(A.err, err_key(T.b, row, p, kStCapacity));
            }
            // The wave's 64 consecutive rows own one contiguous output range
            // [ws, ws+wn): assemble it in LDS (kWaveBuf bytes at a time), note any
            // non-ASCII byte on the way, and store it with aligned 16-B stores.
            bool ascii = true;
            const bool emit = wn && !(A.debug & 1) && ws + wn <= o.values_cap && ws + wn <= 0x7FFFFFFFull;
            if (emit) {
#pragma unroll 1
                for (uint64_t w0 = ws; w0 < ws + wn; w0 += kWaveBuf) {
                    const uint64_t w1 = min(w0 + kWaveBuf, ws + wn);
                    const uint64_t lo_b = max(d0, w0), hi_b = min(end, w1);
#pragma unroll 1
                    for (uint64_t q = lo_b; q < hi_b; q++) {
                        const uint32_t ch = src.u8(pay + (uint32_t)(q - d0));
                        ascii &= ch < 0x80;
                        wb[q - w0] = (uint8_t)ch;
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes landed
                    write_out(wb, gp(o.values), w0, w1 - w0, lane, 64);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before reuse
                }
            } else if (slen) {
#pragma unroll 1
                for (uint32_t q = 0; q < slen; q++) ascii &= src.u8(pay + q) < 0x80;
            }
            if (!ascii && !utf8_valid_slow(src, pay, slen)) report(A.err, err_key(T.b, row, p, kStUtf8));
        }
    }
    dstamp(A, s_st, 4);
}

// LDS (dynamic): [buffer 0][buffer 1][s_nulls: nproj u32][s_w: 4 u64]
//                [wave string buffers: 4 x (kWaveBuf + 32) when utf8 is projected]
//                [s_proj: nproj DecProj][s_out: nproj DecOut (current tile's block)][s_mine: nutf8 u64]
__global__ void __launch_bounds__(256) decode_kernel(DecodeArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const DecLayout L = dec_layout(A.rows_per_tile, A.nutf8, A.stage);
    uint8_t* bufs[2] = {lds, lds + L.bytes};
    const uint32_t np16 = (4 * A.nproj + 15) & ~15u;
    uint32_t* s_nulls = reinterpret_cast<uint32_t*>(lds + 2 * L.bytes);
    uint64_t* s_w = reinterpret_cast<uint64_t*>(lds + 2 * L.bytes + np16);
    uint8_t* s_wbuf = lds + 2 * L.bytes + np16 + 32;
    DecProj* s_proj = reinterpret_cast<DecProj*>(s_wbuf + (A.nutf8 ? 4 * (kWaveBuf + 32) : 0));
    DecOut* s_out = reinterpret_cast<DecOut*>(s_proj + A.nproj);
    uint64_t* s_mine = reinterpret_cast<uint64_t*>(s_out + A.nproj);
    uint64_t* s_st = s_mine + A.nutf8;  // 8 diagnostic stamp slots
    if (threadIdx.x < 8) s_st[threadIdx.x] = threadIdx.x == 7 ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // output descriptors of block b into LDS: uniform index -> s_load (no vmcnt)
    auto fill_out = [&](uint32_t blk) {
        if (wave == 0)
            for (uint32_t p = 0; p < A.nproj; p++) {
                const DecOut o = ldout(A, (uint64_t)blk * A.nproj + p);
                if (lane == 0) s_out[p] = o;
            }
    };
    const uint32_t tid = threadIdx.x;
    const uint64_t G = gridDim.x;
    for (uint32_t p = tid; p < A.nproj; p += 256) {
        s_nulls[p] = 0;
        s_proj[p] = ldproj(A, p);
    }
    uint32_t b = 0;
    DecTile cur = tile_info(A, blockIdx.x, &b);
    if (!cur.ok) return;  // uniform
    fill_out(cur.b);
    uint32_t out_b = cur.b;
    issue_stage(A, cur, bufs[0], L);
    DecTile nxt = tile_info(A, blockIdx.x + G, &b);
    for (uint64_t i = 0; cur.ok; i++) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA for `cur` landed
        __syncthreads();                                  // ... and every other wave's
        dstamp(A, s_st, 0);
        if (nxt.ok) issue_stage(A, nxt, bufs[(i + 1) & 1], L);
        const DecTile nn = tile_info(A, cur.t + 2 * G, &b);
        dstamp(A, s_st, 1);
        uint8_t* buf = bufs[i & 1];
        const bool span_ok = cur.end - cur.abase <= 0xFFFFFFF0ull;  // > 4 GiB tile: unsupported
        if (!span_ok) {
            if (tid == 0) {
                report(A.err, err_key(cur.b, cur.r0, 0, kStMalformed));
                for (uint32_t u = 0; u < A.nutf8; u++) publish(A.lookback + (uint64_t)u * A.total_tiles + cur.t, 1);
            }
        } else if (A.debug & 4) {
            // ablation: staging only
        } else {
            const TileSrc src{buf + L.stage, gp(ldblk(A, cur.b).data) + cur.abase,
                              ((cur.end + 15) & ~15ull) - cur.abase <= A.stage};
            decode_tile(A, src, cur, buf, L, s_nulls, s_w, s_wbuf, s_proj, s_out, s_mine, s_st);
        }
        lds_barrier();
        for (uint32_t p = tid; p < A.nproj; p += 256) {
            const uint32_t v = s_nulls[p];
            if (v) {
                __hip_atomic_fetch_add(gp(A.nulls) + (uint64_t)cur.b * A.nproj + p, (unsigned long long)v,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_nulls[p] = 0;
            }
        }
        cur = nxt;
        nxt = nn;
        if (cur.ok && cur.b != out_b) {  // next tile's block outputs (read after the loop-top barrier)
            fill_out(cur.b);
            out_b = cur.b;
        }
        dstamp(A, s_st, 5);
    }
    if ((A.debug & 8) && threadIdx.x == 0)
        for (int j = 0; j < 7; j++) __hip_atomic_fetch_add(gp(A.stamps) + j, (unsigned long long)s_st[j],
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
            tstart = window_prefix(A.lookback, have_prev ? t - G + 1 : 0, t, have_prev ? prev_incl : 0,
                                   s_w, A.err, err_key(0, r0, 0, 0));
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
            write_out(stage, gp(A.out), tstart, span, tid, 256);
            __syncthreads();
        } else if (active) {
            encode_row(A, row, A.out + start);
        }
    }
}

}  // namespace

uint32_t decode_lds_bytes(uint32_t stage, uint32_t nproj, uint32_t nutf8, uint32_t rows_per_tile) {
    const DecLayout L = dec_layout(rows_per_tile, nutf8, stage);
    return 2 * L.bytes + ((4 * nproj + 15) & ~15u) + 32 + (nutf8 ? 4 * (kWaveBuf + 32) : 0) +
           nproj * (uint32_t)(sizeof(DecProj) + sizeof(DecOut)) + 8 * nutf8 + 64;
}

hipError_t launch_decode(const DecodeArgs& a, uint32_t grid, hipStream_t s) {
    const uint32_t lds = decode_lds_bytes(a.stage, a.nproj, a.nutf8, a.rows_per_tile);
    hipLaunchKernelGGL(decode_kernel, dim3(grid), dim3(kTile), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_encode(const EncodeArgs& a, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(encode_kernel, dim3(grid), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

int decode_blocks_per_cu(uint32_t lds, uint32_t rows_per_tile) {
    int n = 0;
    hipError_t e;
    (void)rows_per_tile;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_kernel, kTile, lds);
    return e == hipSuccess ? n : 1;
}

int encode_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, encode_kernel, kTile, 0) != hipSuccess) return 1;
    return n;
}

}  // namespace murr
