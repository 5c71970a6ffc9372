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

constexpr uint32_t kUtf8 = 0, kBool = 1;
constexpr uint32_t kSpinLimit = 1u << 22;
enum : uint32_t { kStUtf8 = 1, kStOverflow = 4, kStMalformed = 5, kStCapacity = 6, kStInternal = 10 };

__device__ __forceinline__ void report(unsigned long long* err, uint64_t key) {
    atomicMax(err, (unsigned long long)~key);
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
    const uint8_t* g;  // HBM (16-B aligned); never reads a dword holding no requested byte
    __device__ __forceinline__ uint32_t u32(uint32_t a) const {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(g + (a & ~3u));
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
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t sum = 0;
    for (uint64_t j = lo + tid; j < t; j += 256) {
        uint64_t v = __hip_atomic_load(st + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t spins = 0;
        while (v == 0) {
            __builtin_amdgcn_s_sleep(2);
            v = __hip_atomic_load(st + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (++spins > kSpinLimit) {
                report(err, ekey | kStInternal);
                v = 1;
                break;
            }
        }
        sum += v - 1;
    }
    sum = wave_sum(sum);
    if (lane == 0) s_w[wave] = sum;
    __syncthreads();
    const uint64_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    return base + tot;
}

__device__ __forceinline__ void publish(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// ---- decode -------------------------------------------------------------------
// A tile is R = 256*RPT rows; thread tid owns rows r0 + k*256 + tid (k < RPT),
// so every (k, wave) pair covers 64 consecutive rows: coalesced row_off loads
// and value stores, and one ballot = one 64-bit bitmap word.  Row addresses are
// u32 offsets from the tile's 16-B aligned blob start, in LDS or in HBM.
struct DecTile {
    uint32_t b;         // block
    uint64_t t, tfirst; // global tile, first tile of the block
    uint64_t r0;        // first row of the tile inside the block
    uint32_t nr;        // rows in the tile
    bool last;          // last tile of the block
};

template <int RPT, class Src>
__device__ __forceinline__ void decode_tile(const DecodeArgs& A, const Src& src, const DecTile& T,
                                            const uint32_t (&ra)[RPT], const uint32_t (&rl)[RPT],
                                            uint32_t* s_nulls, uint64_t* s_tot, uint64_t* s_w) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t bs = A.bs;
    const uint64_t nproj = A.nproj;
    // Null bitsets of my rows (bit = 1 -> NULL), cached when bs <= 4.
    uint32_t bits[RPT];
    uint32_t okm = 0, actm = 0;  // bit k: row k present & well formed / row k in tile
#pragma unroll
    for (int k = 0; k < RPT; k++) {
        const bool act = k * 256 + tid < T.nr;
        const bool present = act && rl[k] > 0;
        const bool short_row = present && rl[k] < bs;  // ReadRow::new split_at panics
        if (short_row) report(A.err, err_key(T.b, T.r0 + k * 256 + tid, 0, kStMalformed));
        actm |= (uint32_t)act << k;
        okm |= (uint32_t)(present && !short_row) << k;
        bits[k] = ~0u;
        if (present && !short_row && bs <= 4) {
            bits[k] = 0;
            for (uint32_t j = 0; j < bs; j++) bits[k] |= src.u8(ra[k] + j) << (8 * j);
        }
    }

    for (uint32_t p = 0; p < A.nproj; p++) {
        const DecProj pc = A.proj[p];
        const DecOut o = A.outs[(uint64_t)T.b * nproj + p];
        const uint32_t fo = bs + pc.offset;
        uint32_t nullm = 0, nnull = 0;
#pragma unroll
        for (int k = 0; k < RPT; k++) {
            bool isnull = true;
            if ((okm >> k) & 1) {
                const uint32_t byte = pc.bit >> 3;
                const uint32_t bv = (bs <= 4) ? (bits[k] >> (8 * byte)) : src.u8(ra[k] + byte);
                isnull = (bv >> (pc.bit & 7)) & 1;
            }
            const bool act = (actm >> k) & 1;
            nullm |= (uint32_t)isnull << k;
            const uint64_t vm = __ballot(act && !isnull);
            nnull += __popcll(__ballot(act && isnull));
            if (lane == 0 && k * 256 + wave * 64 < T.nr)
                reinterpret_cast<uint64_t*>(o.validity)[((T.r0 + k * 256) >> 6) + wave] = vm;
        }
        if (lane == 0 && nnull) atomicAdd(&s_nulls[p], nnull);

        if (!pc.is_utf8) {
#pragma unroll
            for (int k = 0; k < RPT; k++) {
                const uint64_t row = T.r0 + k * 256 + tid;
                const bool act = (actm >> k) & 1;
                bool fnull = (nullm >> k) & 1;
                if (!fnull && fo + pc.width > rl[k]) {
                    report(A.err, err_key(T.b, row, p, kStMalformed));
                    fnull = true;
                }
                if (pc.dtype == kBool) {
                    const bool v = !fnull && src.u8(ra[k] + fo) != 0;
                    const uint64_t m = __ballot(act && v);
                    if (lane == 0 && k * 256 + wave * 64 < T.nr)
                        reinterpret_cast<uint64_t*>(o.values)[((T.r0 + k * 256) >> 6) + wave] = m;
                } else if (act) {
                    const uint64_t v = fnull ? 0 : read_w(src, ra[k] + fo, pc.width);
                    uint8_t* dst = o.values + row * pc.width;
                    switch (pc.width) {
                    case 8: *reinterpret_cast<uint64_t*>(dst) = v; break;
                    case 4: *reinterpret_cast<uint32_t*>(dst) = (uint32_t)v; break;
                    case 2: *reinterpret_cast<uint16_t*>(dst) = (uint16_t)v; break;
                    default: *dst = (uint8_t)v; break;
                    }
                }
            }
            continue;
        }

        // ---- utf8: read_dynamic (read.rs:45-55) -> lengths, tile scan, window
        //      prefix across tiles, offsets, copy + validate (utf8.rs:86-96)
        uint32_t slen[RPT], pay[RPT];
#pragma unroll
        for (int k = 0; k < RPT; k++) {
            slen[k] = 0;
            pay[k] = 0;
            if (!((nullm >> k) & 1)) {
                const uint64_t row = T.r0 + k * 256 + tid;
                const uint32_t vlen = rl[k] - bs;  // static + payload region
                if (fo + 4 > rl[k]) {
                    report(A.err, err_key(T.b, row, p, kStMalformed));
                } else {
                    const uint32_t prel = src.u32(ra[k] + fo);
                    if ((uint64_t)prel + 4 > vlen) {
                        report(A.err, err_key(T.b, row, p, kStMalformed));
                    } else {
                        const uint32_t l = src.u32(ra[k] + bs + prel);
                        if ((uint64_t)prel + 4 + l > vlen) report(A.err, err_key(T.b, row, p, kStMalformed));
                        else { slen[k] = l; pay[k] = ra[k] + bs + prel + 4; }
                    }
                }
            }
            const uint64_t inc = wave_incl_scan(slen[k], lane);
            if (lane == 63) s_tot[k * 4 + wave] = inc;
        }
        __syncthreads();
        // exclusive prefix of each (k, wave) total, k-major (read after the
        // barriers inside window_prefix)
        uint64_t* s_pre = s_tot + 4 * RPT;
        if (tid < 4 * RPT) {
            uint64_t run = 0;
            for (uint32_t j = 0; j < tid; j++) run += s_tot[j];
            s_pre[tid] = run;
        }
        uint64_t agg = 0;
#pragma unroll
        for (int j = 0; j < 4 * RPT; j++) agg += s_tot[j];
        uint64_t* st = A.lookback + (uint64_t)pc.uslot * A.total_tiles;
        if (tid == 0) publish(st + T.t, agg + 1);
        // this workgroup's own inclusive prefix of tile t - G (same block) or 0
        uint64_t* mine = A.prev + (uint64_t)blockIdx.x * A.nutf8 + pc.uslot;
        const uint64_t G = gridDim.x;
        const bool have_prev = T.t >= T.tfirst + G;
        const uint64_t lo = have_prev ? T.t - G + 1 : T.tfirst;
        const uint64_t prefix = window_prefix(st, lo, T.t, have_prev ? *mine : 0, s_w, A.err,
                                              err_key(T.b, T.r0, p, 0));
        if (tid == 0) {
            *mine = prefix + agg;
            if (T.t == T.tfirst) o.offsets[0] = 0;
            if (T.last) A.lens[(uint64_t)T.b * nproj + p] = prefix + agg;
        }
#pragma unroll
        for (int k = 0; k < RPT; k++) {
            const uint64_t inc = wave_incl_scan(slen[k], lane);
            if (!((actm >> k) & 1)) continue;
            const uint64_t row = T.r0 + k * 256 + tid;
            const uint64_t end = prefix + s_pre[k * 4 + wave] + inc;
            if (end > 0x7FFFFFFFull) {
                report(A.err, err_key(T.b, row, p, kStOverflow));
                continue;
            }
            o.offsets[row + 1] = (int32_t)end;
            if (slen[k] == 0) continue;
            if (end > o.values_cap) {
                report(A.err, err_key(T.b, row, p, kStCapacity));
                continue;
            }
            uint8_t* dst = o.values + (end - slen[k]);
            Utf8Dfa dfa;
            for (uint32_t j = 0; j < slen[k]; j++) {
                const uint32_t c = src.u8(pay[k] + j);
                dst[j] = (uint8_t)c;
                dfa.step(c);
            }
            if (!dfa.ok()) report(A.err, err_key(T.b, row, p, kStUtf8));
        }
        __syncthreads();  // s_tot / s_pre reused by the next utf8 column
    }
}

// LDS layout (dynamic): [stage: A.stage + 32][s_nulls: nproj u32][s_tot, s_pre: 4*RPT u64 each][s_w: 4 u64]
template <int RPT>
__global__ void __launch_bounds__(256) decode_kernel(DecodeArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* stage = lds;
    uint32_t* s_nulls = reinterpret_cast<uint32_t*>(lds + A.stage + 32);
    uint64_t* s_tot = reinterpret_cast<uint64_t*>(lds + A.stage + 32 + ((4 * A.nproj + 15) & ~15u));
    uint64_t* s_w = s_tot + 8 * RPT;
    constexpr uint32_t R = 256 * RPT;
    const uint32_t tid = threadIdx.x;
    uint32_t b = 0;  // this workgroup visits tiles in increasing order

    for (uint64_t t = blockIdx.x; t < A.total_tiles; t += gridDim.x) {
        while (b + 1 < A.nblocks && A.blocks[b + 1].tile_base <= t) b++;
        const DecBlock blk = A.blocks[b];
        DecTile T;
        T.b = b;
        T.t = t;
        T.tfirst = blk.tile_base;
        T.r0 = (t - blk.tile_base) * R;
        T.nr = (uint32_t)min((uint64_t)R, blk.n_rows - T.r0);
        T.last = T.r0 + T.nr == blk.n_rows;
        for (uint32_t p = tid; p < A.nproj; p += 256) s_nulls[p] = 0;

        const uint64_t base = blk.row_off[T.r0], end = blk.row_off[T.r0 + T.nr];
        const uint64_t abase = base & ~15ull;
        uint32_t ra[RPT], rl[RPT];
#pragma unroll
        for (int k = 0; k < RPT; k++) {
            ra[k] = rl[k] = 0;
            if (k * 256 + tid < T.nr) {
                const uint64_t* ro = blk.row_off + T.r0 + k * 256 + tid;
                const uint64_t a = ro[0], z = ro[1];
                ra[k] = (uint32_t)(a - abase);
                rl[k] = (uint32_t)(z - a);
            }
        }
        const bool in_lds = end - abase <= A.stage;
        if (end - abase > 0xFFFFFFF0ull) {  // one tile spanning > 4 GiB of blobs: unsupported
            if (tid == 0) report(A.err, err_key(b, T.r0, 0, kStMalformed));
            continue;
        }
        if (in_lds) {
            // Coalesced 16-B loads of the tile's contiguous blob bytes into LDS.
            const uint64_t efull = end & ~15ull;
            const uint64_t nfull = (efull - abase) >> 4;
            const uint4* g = reinterpret_cast<const uint4*>(blk.data + abase);
            uint4* l = reinterpret_cast<uint4*>(stage);
            for (uint64_t k = tid; k < nfull; k += 256) l[k] = g[k];
            if (tid < end - efull) stage[efull - abase + tid] = blk.data[efull + tid];
        }
        __syncthreads();
        if (in_lds) decode_tile<RPT>(A, LdsSrc{stage}, T, ra, rl, s_nulls, s_tot, s_w);
        else decode_tile<RPT>(A, GlbSrc{blk.data + abase}, T, ra, rl, s_nulls, s_tot, s_w);
        __syncthreads();
        for (uint32_t p = tid; p < A.nproj; p += 256)
            if (s_nulls[p]) atomicAdd(&A.nulls[(uint64_t)b * A.nproj + p], (unsigned long long)s_nulls[p]);
        __syncthreads();
    }
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

// Copy stage[0..span) (LDS) to out[g0..g0+span) with aligned 16-B stores.
__device__ __forceinline__ void write_out(const uint8_t* stage, uint8_t* out, uint64_t g0,
                                          uint64_t span) {
    const uint32_t tid = threadIdx.x;
    const uint64_t g1 = g0 + span;
    const uint64_t a0 = (g0 + 15) & ~15ull, a1 = g1 & ~15ull;
    if (a0 >= a1) {
        for (uint64_t k = tid; k < span; k += 256) out[g0 + k] = stage[k];
        return;
    }
    if (tid < a0 - g0) out[g0 + tid] = stage[tid];
    if (tid < g1 - a1) out[a1 + tid] = stage[a1 - g0 + tid];
    const uint32_t lb0 = (uint32_t)(a0 - g0);
    const uint32_t sh = lb0 & 3u;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(stage);
    const uint64_t nch = (a1 - a0) >> 4;
    uint4* o = reinterpret_cast<uint4*>(out + a0);
    for (uint64_t c = tid; c < nch; c += 256) {
        const uint32_t q = (lb0 >> 2) + 4 * (uint32_t)c;
        uint32_t d0 = w[q], d1 = w[q + 1], d2 = w[q + 2], d3 = w[q + 3], d4 = w[q + 4];
        uint4 v;
        v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
        v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
        v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
        v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
        o[c] = v;
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
            write_out(stage, A.out, tstart, span);
            __syncthreads();
        } else if (active) {
            encode_row(A, row, A.out + start);
        }
    }
}

}  // namespace

uint32_t decode_lds_bytes(uint32_t stage, uint32_t nproj, int rpt) {
    return stage + 32 + ((4 * nproj + 15) & ~15u) + 8 * (8 * rpt + 4);
}

hipError_t launch_decode(const DecodeArgs& a, int rpt, uint32_t grid, hipStream_t s) {
    const uint32_t lds = decode_lds_bytes(a.stage, a.nproj, rpt);
    switch (rpt) {
    case 1: hipLaunchKernelGGL(decode_kernel<1>, dim3(grid), dim3(kTile), lds, s, a); break;
    case 2: hipLaunchKernelGGL(decode_kernel<2>, dim3(grid), dim3(kTile), lds, s, a); break;
    case 4: hipLaunchKernelGGL(decode_kernel<4>, dim3(grid), dim3(kTile), lds, s, a); break;
    default: hipLaunchKernelGGL(decode_kernel<8>, dim3(grid), dim3(kTile), lds, s, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_encode(const EncodeArgs& a, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(encode_kernel, dim3(grid), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

int decode_blocks_per_cu(int rpt, uint32_t lds) {
    int n = 0;
    hipError_t e;
    switch (rpt) {
    case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_kernel<1>, kTile, lds); break;
    case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_kernel<2>, kTile, lds); break;
    case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_kernel<4>, kTile, lds); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_kernel<8>, kTile, lds); break;
    }
    return e == hipSuccess ? n : 1;
}

int encode_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, encode_kernel, kTile, 0) != hipSuccess) return 1;
    return n;
}

}  // namespace murr
