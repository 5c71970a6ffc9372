// murr_sst.hip — RocksDB data blocks -> (user key, value) entries on the
// device: the bulk read of an SST's data blocks a
// warm-up or rehydration does, ending in the row-blob decode block the decode
// kernel takes and the key column the device index takes.
//
// Formats (restated in oracle/murr_sst.c, which the tests check against):
// the reference's store (src/io/store/rocksdb/block.rs:97-121) writes
// block-based SSTs with 512-byte blocks, restart interval 8, a BinaryAndHash
// data-block index and the default compression (Snappy).  A block's contents
// are plain, raw Snappy, or RocksDB's LZ4 (varint32 length + LZ4 block);
// uncompressed they are entries
// [varint32 shared][varint32 non_shared][varint32 value_len][key delta][value]
// then u32 restart offsets, for BinaryAndHash the hash buckets (u8) and
// their count (u16), and a u32 footer num_restarts | index_type << 31.  Keys
// are internal keys: user key + 8-byte LE trailer (sequence << 8 | type).
//
// A lane group per block.  The stored block is staged into
// the group's LDS slot, inflated there (tags parsed wave-uniformly from 8-byte LDS
// windows, every literal and match copied by the group's lanes at once; a match
// longer than its offset repeats its pattern by i % offset), and the entries
// are walked from LDS: headers uniformly, key deltas and values copied by the
// lanes, the internal key rebuilt in place in an LDS key buffer as the block
// format defines it.  sst_count inflates from the stored bytes and keeps each inflated tier-0 block in a fixed 1 KiB HBM slot
// for sst_decode, which stages it back instead of inflating again.  Slots come
// in two tiers:
// blocks up to 1 KiB uncompressed (16 lanes each, 8 per workgroup: the
// reference's 512-byte blocks) and up to 4 KiB (a wave each); a block larger
// than that, or with an internal key > kKeyCap, is tier 2: one thread
// inflates it into a raw buffer and walks it serially (sst_big_count,
// sst_big_decode).
#include <cstdlib>

#include "murr_device.h"

namespace murr {

namespace {

using namespace dev;

constexpr uint32_t kSstCorrupt = 5;  // err_key status: MURR_E_MALFORMED_ROW (row = block index)
constexpr uint32_t kThreads = 128;   // threads per workgroup (kThreads / G blocks)
constexpr uint32_t kKeyCap = 256;    // internal key bytes
constexpr uint32_t kPad = 32;        // the 16-B staging shift + window reads 11 bytes past a position

// A block slot in LDS for blocks of up to RAW uncompressed bytes (stored bytes
// up to Snappy's bound for RAW).  Tier 0: RAW 1024 (the reference's 512-byte
// blocks plus their last entry), 16 lanes per block; tier 1: RAW 4096, a
// wave per block; larger blocks (tier 2) go thread-serial through HBM.
template <uint32_t RAW, bool COMP = true>  // COMP false: no stored-block region (tier-0 decode)
struct alignas(16) BlockLds {
    static constexpr uint32_t kRaw = RAW;
    static constexpr uint32_t kComp = (RAW + RAW / 6 + 32 + 15) & ~15u;
    uint8_t raw[RAW + kPad];
    uint8_t comp[COMP ? kComp + kPad : 16];
    uint8_t key[kKeyCap + kPad];
};
static_assert(sizeof(BlockLds<1024>) % 16 == 0 && sizeof(BlockLds<4096>) % 16 == 0, "LDS slots stay aligned");
constexpr uint32_t kTier0Raw = 1024, kTier1Raw = 4096;

// unaligned little-endian u32 (byte loads: blocks are byte-packed)
__device__ __forceinline__ uint32_t ld_u32u(const uint8_t* p) {
    return (uint32_t)gp(p)[0] | ((uint32_t)gp(p)[1] << 8) | ((uint32_t)gp(p)[2] << 16) | ((uint32_t)gp(p)[3] << 24);
}

__device__ __forceinline__ void sst_report(unsigned long long* err, uint64_t block) {
    __hip_atomic_fetch_max((GAS unsigned long long*)err, (unsigned long long)~err_key(0, block, 0, kSstCorrupt),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ SstBlock ldblock(const SstBlock* b) {
    const GAS SstBlock* q = gp(b);
    SstBlock r;
    r.data = q->data; r.size = q->size; r.compression = q->compression; r.pad = 0;
    return r;
}

// Lanes of one wave exchange bytes through LDS: order this wave's LDS
// accesses (the LDS serves a wave's instructions in issue order; this keeps
// the compiler from moving them across).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- thread-serial path (big blocks) -------------------------------------------

// varint32 at p (bounded by end); false when malformed.
__device__ __forceinline__ bool varint32(const uint8_t*& p, const uint8_t* end, uint32_t& v) {
    uint32_t r = 0;
    for (int shift = 0; shift <= 28; shift += 7) {
        if (p >= end) return false;
        const uint32_t b = *gp(p);
        p++;
        r |= (b & 0x7Fu) << shift;
        if (!(b & 0x80u)) {
            v = r;
            return true;
        }
    }
    return false;
}

// Raw Snappy into dst[0, ulen); false when malformed.
__device__ bool inflate_snappy(const uint8_t* p, const uint8_t* end, GAS uint8_t* dst, uint64_t ulen) {
    uint32_t skip;
    if (!varint32(p, end, skip)) return false;
    uint64_t o = 0;
    while (p < end) {
        const uint32_t tag = *gp(p);
        p++;
        uint32_t len, off;
        const uint32_t kind = tag & 3u;
        if (kind == 0) {  // literal
            len = tag >> 2;
            if (len >= 60) {
                const uint32_t nb = len - 59;
                if ((uint64_t)(end - p) < nb) return false;
                len = 0;
                for (uint32_t i = 0; i < nb; i++) len |= (uint32_t)gp(p)[i] << (8 * i);
                p += nb;
            }
            len += 1;
            if ((uint64_t)(end - p) < len || o + len > ulen) return false;
            for (uint32_t i = 0; i < len; i++) dst[o + i] = gp(p)[i];
            p += len;
            o += len;
            continue;
        }
        if (kind == 1) {
            if (p >= end) return false;
            len = 4 + ((tag >> 2) & 7u);
            off = ((tag >> 5) << 8) | *gp(p);
            p += 1;
        } else if (kind == 2) {
            if (end - p < 2) return false;
            len = 1 + (tag >> 2);
            off = (uint32_t)gp(p)[0] | ((uint32_t)gp(p)[1] << 8);
            p += 2;
        } else {
            if (end - p < 4) return false;
            len = 1 + (tag >> 2);
            off = ld_u32u(p);
            p += 4;
        }
        if (off == 0 || off > o || o + len > ulen) return false;
        for (uint32_t i = 0; i < len; i++, o++) dst[o] = dst[o - off];  // in order: an overlap repeats
    }
    return o == ulen;
}

// LZ4 length extension: 15 means more bytes follow, each added until one < 255.
__device__ __forceinline__ bool lz4_ext(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
    uint32_t b;
    do {
        if (p >= end) return false;
        b = *gp(p);
        p++;
        v += b;
    } while (b == 255);
    return true;
}

// varint32 length + one LZ4 block into dst[0, ulen); false when malformed.
__device__ bool inflate_lz4(const uint8_t* p, const uint8_t* end, GAS uint8_t* dst, uint64_t ulen) {
    uint32_t skip;
    if (!varint32(p, end, skip)) return false;
    uint64_t o = 0;
    for (;;) {
        if (p >= end) return false;  // the last sequence (literals only) ends the block
        const uint32_t tok = *gp(p);
        p++;
        uint64_t lit = tok >> 4;
        if (lit == 15 && !lz4_ext(p, end, lit)) return false;
        if ((uint64_t)(end - p) < lit || o + lit > ulen) return false;
        for (uint64_t i = 0; i < lit; i++) dst[o + i] = gp(p)[i];
        p += lit;
        o += lit;
        if (p == end) break;
        if (end - p < 2) return false;
        const uint32_t off = (uint32_t)gp(p)[0] | ((uint32_t)gp(p)[1] << 8);
        p += 2;
        uint64_t ml = tok & 15u;
        if (ml == 15 && !lz4_ext(p, end, ml)) return false;
        ml += 4;
        if (off == 0 || off > o || o + ml > ulen) return false;
        for (uint64_t i = 0; i < ml; i++, o++) dst[o] = dst[o - off];
    }
    return o == ulen;
}

// The entry region [0, limit) of an uncompressed block from its footer.
__device__ __forceinline__ bool block_layout(const uint8_t* blk, uint64_t n, uint64_t& limit) {
    if (n < 4) return false;
    const uint32_t footer = ld_u32u(blk + n - 4);
    const uint32_t nr = footer & 0x7FFFFFFFu;
    uint64_t tail = 4;
    if (footer >> 31) {  // BinaryAndHash: [buckets u8 x nb][nb u16] before the footer
        if (n < 6) return false;
        tail += 2 + (uint64_t)(ld_u32u(blk + n - 6) & 0xFFFFu);
    }
    tail += 4ull * nr;
    if (nr == 0 || tail > n) return false;
    limit = n - tail;
    return true;
}

// Walk big block b's entries from raw; count (EMIT false) or write them.
template <bool EMIT>
__device__ void big_walk(const SstArgs& A, uint64_t b) {
    const uint8_t* blk = A.raw + gp(A.uoff)[b];
    const uint64_t n = gp(A.ulen)[b];
    uint64_t limit = 0;
    if (!block_layout(blk, n, limit)) {
        if (!EMIT) sst_report(A.err, b);
        return;
    }
    const uint8_t* p = blk;
    const uint8_t* end = blk + limit;
    uint64_t cnt = 0, kbytes = 0, vbytes = 0;
    uint64_t e0 = 0, k0 = 0, v0 = 0;
    if (EMIT) {
        e0 = gp(A.eoff)[b];
        k0 = gp(A.koff)[b];
        v0 = gp(A.voff)[b];
    }
    uint64_t pstart = 0;  // previous user key: output position and length
    uint32_t plen = 0, pilen = 0;
    uint64_t ptrailer = 0;  // previous trailer
    bool bad = false;
    while (p < end) {
        uint32_t shared, nonshared, vlen;
        if (!varint32(p, end, shared) || !varint32(p, end, nonshared) || !varint32(p, end, vlen)) { bad = true; break; }
        const uint64_t ilen = (uint64_t)shared + nonshared;
        if (shared > pilen || ilen < 8 || ilen > 0x7FFFFFFFull || (uint64_t)(end - p) < (uint64_t)nonshared + vlen) {
            bad = true;
            break;
        }
        const uint32_t ulen = (uint32_t)ilen - 8;
        if (EMIT) {
            GAS uint8_t* ko = gp(A.keys) + k0 + kbytes;
            uint64_t trailer = 0;
            for (uint32_t q = 0; q < (uint32_t)ilen; q++) {
                uint32_t byte;
                if (q < shared)
                    byte = q < plen ? (uint32_t)gp(A.keys)[pstart + q] : (uint32_t)(ptrailer >> (8 * (q - plen))) & 0xFFu;
                else
                    byte = gp(p)[q - shared];
                if (q < ulen) ko[q] = (uint8_t)byte;
                else trailer |= (uint64_t)byte << (8 * (q - ulen));
            }
            const uint64_t e = e0 + cnt;
            gp(A.key_off)[e + 1] = (int32_t)(k0 + kbytes + ulen);
            gp(A.seqs)[e] = trailer >> 8;
            gp(A.types)[e] = (uint8_t)(trailer & 0xFFu);
            const uint8_t* vp = p + nonshared;
            GAS uint8_t* vo = gp(A.vals) + v0 + vbytes;
            for (uint32_t q = 0; q < vlen; q++) vo[q] = gp(vp)[q];
            gp(A.val_off)[e + 1] = v0 + vbytes + vlen;
            pstart = k0 + kbytes;
            ptrailer = trailer;
        }
        p += (uint64_t)nonshared + vlen;
        plen = ulen;
        pilen = (uint32_t)ilen;
        kbytes += ulen;
        vbytes += vlen;
        cnt++;
    }
    if (!EMIT) {
        if (bad) sst_report(A.err, b);
        gp(A.ne)[b] = cnt;
        gp(A.kb)[b] = kbytes;
        gp(A.vb)[b] = vbytes;
    }
}

// Big blocks: inflate (or copy) into raw + uoff[b], then count.
__global__ void __launch_bounds__(256) sst_big_count(SstArgs A) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= A.nblocks || gp(A.tier)[b] != 2) return;
    const SstBlock blk = ldblock(A.blocks + b);
    GAS uint8_t* dst = gp(A.raw) + gp(A.uoff)[b];
    const uint64_t ulen = gp(A.ulen)[b];
    bool ok = true;
    if (blk.compression == 0)
        for (uint64_t i = 0; i < ulen; i++) dst[i] = gp(blk.data)[i];
    else if (blk.compression == 1)
        ok = inflate_snappy(blk.data, blk.data + blk.size, dst, ulen);
    else
        ok = inflate_lz4(blk.data, blk.data + blk.size, dst, ulen);
    if (!ok) {
        sst_report(A.err, b);
        return;
    }
    big_walk<false>(A, b);
}

__global__ void __launch_bounds__(256) sst_big_decode(SstArgs A) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b < A.nblocks && gp(A.tier)[b] == 2) big_walk<true>(A, b);
}

// ---- wave-per-block path -------------------------------------------------------

// 8 bytes of an LDS region from byte p (any alignment; reads to p + 11).
__device__ __forceinline__ uint64_t win8(const uint8_t* s, uint32_t p) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (p & ~3u));
    const uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    const uint32_t sh = (p & 3u) * 8;
    return sh ? (lo >> sh) | ((uint64_t)w[2] << (64 - sh)) : lo;
}

// varint32 at s[p] (p < end) from one window: its length, 0 = malformed.
__device__ __forceinline__ uint32_t wvarint(const uint8_t* s, uint32_t p, uint32_t end, uint32_t& v) {
    const uint64_t w = win8(s, p);
    uint32_t r = 0;
    for (uint32_t i = 0; i < 5; i++) {
        if (p + i >= end) return 0;
        const uint32_t b = (uint32_t)(w >> (8 * i)) & 0xFFu;
        r |= (b & 0x7Fu) << (7 * i);
        if (!(b & 0x80u)) {
            v = r;
            return i + 1;
        }
    }
    return 0;
}

// An entry header (three varint32s, at most 15 bytes) from one 16-byte
// window at s[p] (p < end): bytes consumed, 0 = malformed.
__device__ __forceinline__ uint32_t hdr3(const uint8_t* s, uint32_t p, uint32_t end, uint32_t& a, uint32_t& b,
                                         uint32_t& c) {
    const uint64_t w0 = win8(s, p), w1 = win8(s, p + 8);
    uint32_t v[3], i = 0;
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
        uint32_t r = 0;
        bool done = false;
#pragma unroll
        for (uint32_t j = 0; j < 5; j++) {
            if (!done) {
                if (p + i >= end) return 0;
                const uint32_t byte = (uint32_t)(i < 8 ? w0 >> (8 * i) : w1 >> (8 * (i - 8))) & 0xFFu;
                r |= (byte & 0x7Fu) << (7 * j);
                done = !(byte & 0x80u);
                i++;
            }
        }
        if (!done) return 0;
        v[k] = r;
    }
    a = v[0];
    b = v[1];
    c = v[2];
    return i;
}

// Stage n bytes from src into LDS with 16-byte loads from src's 16-B aligned
// base, four per lane in flight: the block lands at dst + the returned shift.
template <uint32_t G>
__device__ __forceinline__ uint32_t stage(uint8_t* dst, const uint8_t* src, uint32_t n, uint32_t lane) {
    const uint64_t a = reinterpret_cast<uint64_t>(src);
    const uint32_t shift = (uint32_t)(a & 15u);
    const GAS u32x4* s16 = reinterpret_cast<const GAS u32x4*>(a - shift);
    u32x4* d16 = reinterpret_cast<u32x4*>(dst);
    const uint32_t chunks = (shift + n + 15) >> 4;
    for (uint32_t c = lane; c < chunks; c += 4 * G) {
        u32x4 v[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++)
            if (c + u * G < chunks) v[u] = s16[c + u * G];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++)
            if (c + u * G < chunks) d16[c + u * G] = v[u];
    }
    return shift;
}

// Lane-group copies inside the group's LDS.
template <uint32_t G>
__device__ __forceinline__ void wcopy(uint8_t* dst, const uint8_t* src, uint32_t n, uint32_t lane) {
    for (uint32_t i = lane; i < n; i += G) dst[i] = src[i];
}
// out[o, o + len) = out[o - off + (i % off)]: a match repeats its last `off` bytes
template <uint32_t G>
__device__ __forceinline__ void wmatch(uint8_t* out, uint32_t o, uint32_t off, uint32_t len, uint32_t lane) {
    if (off >= len) {
        for (uint32_t i = lane; i < len; i += G) out[o + i] = out[o - off + i];
    } else {
        for (uint32_t i = lane; i < len; i += G) out[o + i] = out[o - off + i % off];
    }
}

// Snappy from c[p, n) into r[0, ulen) (wave-uniform parse); false when malformed.
template <uint32_t G>
__device__ __forceinline__ bool winflate_snappy(const uint8_t* c, uint32_t p, uint32_t n, uint8_t* r, uint32_t ulen,
                                                uint32_t lane) {
    uint32_t o = 0;
    while (p < n) {
        const uint64_t w = win8(c, p);
        const uint32_t tag = (uint32_t)w & 0xFFu;
        p++;
        uint32_t len, off;
        const uint32_t kind = tag & 3u;
        if (kind == 0) {
            len = tag >> 2;
            if (len >= 60) {
                const uint32_t nb = len - 59;
                if (n - p < nb) return false;
                len = (uint32_t)(w >> 8) & (nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1));
                p += nb;
            }
            len += 1;
            if (n - p < len || o + len > ulen) return false;
            wcopy<G>(r + o, c + p, len, lane);
            p += len;
            o += len;
            wave_sync();
            continue;
        }
        if (kind == 1) {
            if (p >= n) return false;
            len = 4 + ((tag >> 2) & 7u);
            off = ((tag >> 5) << 8) | ((uint32_t)(w >> 8) & 0xFFu);
            p += 1;
        } else if (kind == 2) {
            if (n - p < 2) return false;
            len = 1 + (tag >> 2);
            off = (uint32_t)(w >> 8) & 0xFFFFu;
            p += 2;
        } else {
            if (n - p < 4) return false;
            len = 1 + (tag >> 2);
            off = (uint32_t)(w >> 8);
            p += 4;
        }
        if (off == 0 || off > o || o + len > ulen) return false;
        wmatch<G>(r, o, off, len, lane);
        o += len;
        wave_sync();
    }
    return o == ulen;
}

// LZ4 length extension from LDS.
__device__ __forceinline__ bool wlz4_ext(const uint8_t* c, uint32_t& p, uint32_t n, uint32_t& v) {
    uint32_t b;
    do {
        if (p >= n) return false;
        b = c[p++];
        v += b;
    } while (b == 255);
    return true;
}

// LZ4 block from c[p, n) into r[0, ulen) (wave-uniform parse).
template <uint32_t G>
__device__ __forceinline__ bool winflate_lz4(const uint8_t* c, uint32_t p, uint32_t n, uint8_t* r, uint32_t ulen,
                                             uint32_t lane) {
    uint32_t o = 0;
    for (;;) {
        if (p >= n) return false;
        const uint32_t tok = c[p++];
        uint32_t lit = tok >> 4;
        if (lit == 15 && !wlz4_ext(c, p, n, lit)) return false;
        if (n - p < lit || o + lit > ulen) return false;
        wcopy<G>(r + o, c + p, lit, lane);
        p += lit;
        o += lit;
        wave_sync();
        if (p == n) break;
        if (n - p < 2) return false;
        const uint32_t off = (uint32_t)win8(c, p) & 0xFFFFu;
        p += 2;
        uint32_t ml = tok & 15u;
        if (ml == 15 && !wlz4_ext(c, p, n, ml)) return false;
        ml += 4;
        if (off == 0 || off > o || o + ml > ulen) return false;
        wmatch<G>(r, o, off, ml, lane);
        o += ml;
        wave_sync();
    }
    return o == ulen;
}

// A claimed uncompressed length no stream of n bytes can reach is malformed
// before anything is sized from it: LZ4 expands at most 255 x (one length
// byte per 255 bytes of match), Snappy about 21 x (a 3-byte copy of 64).
__device__ __forceinline__ bool expansion_ok(uint64_t ulen, uint64_t n) { return ulen <= 256 * n + 64; }

// Stage + inflate a block into L.raw: 1 ok, 0 malformed, 2 larger than the
// slot (big_len = its uncompressed size).  The block is L.raw[r0, r0 + ulen).
template <uint32_t G, class Lds>
__device__ __forceinline__ int wave_inflate(const SstBlock& blk, Lds& L, uint32_t& r0, uint32_t& ulen,
                                            uint64_t& big_len, uint32_t lane) {
    if (blk.compression == 0) {
        big_len = blk.size;
        if (blk.size > Lds::kRaw) return 2;
        ulen = (uint32_t)blk.size;
        r0 = stage<G>(L.raw, blk.data, ulen, lane);
        wave_sync();
        return 1;
    }
    if (blk.size > Lds::kComp) {  // sized from the length prefix, read from HBM
        const uint8_t* p = blk.data;
        uint32_t v = 0;
        if (!varint32(p, blk.data + blk.size, v) || !expansion_ok(v, blk.size)) return 0;
        big_len = v;
        return 2;
    }
    const uint32_t n = (uint32_t)blk.size;
    const uint32_t c0 = stage<G>(L.comp, blk.data, n, lane);
    wave_sync();
    // the varint32 length prefix (Snappy's own, RocksDB's for LZ4)
    uint32_t v = 0;
    const uint32_t hl = n ? wvarint(L.comp, c0, c0 + n, v) : 0;
    if (!hl || !expansion_ok(v, n)) return 0;
    big_len = v;
    if (v > Lds::kRaw) return 2;
    ulen = v;
    r0 = 0;
    const bool ok = blk.compression == 1 ? winflate_snappy<G>(L.comp, c0 + hl, c0 + n, L.raw, ulen, lane)
                                         : winflate_lz4<G>(L.comp, c0 + hl, c0 + n, L.raw, ulen, lane);
    return ok ? 1 : 0;
}

// dst[0, n) = lds[x, x + n) (lds 4-byte aligned, readable to x + n + 11) by
// the group's lanes: unaligned 8-byte stores (the last one overlapping its
// neighbour with the same bytes), byte stores under 8 bytes -- a 42-byte row
// blob is one store instruction instead of six byte stores.
template <uint32_t G>
__device__ __forceinline__ void wstore8(GAS uint8_t* dst, const uint8_t* lds, uint32_t x, uint32_t n, uint32_t lane) {
    if (n >= 8) {
        for (uint32_t q = 8 * lane; q + 8 <= n; q += 8 * G) *(GAS u64u*)(dst + q) = win8(lds, x + q);
        if ((n & 7u) && lane == 0) *(GAS u64u*)(dst + n - 8) = win8(lds, x + n - 8);
    } else {
        for (uint32_t q = lane; q < n; q += G) dst[q] = lds[x + q];
    }
}

// Walk the entries of the block in L.raw[0, n); EMIT writes them at (e0, k0,
// v0).  1 ok, 0 malformed, 3 an internal key longer than the key buffer.
template <uint32_t G, bool EMIT, class Lds>
__device__ __forceinline__ int wave_walk(const SstArgs& A, Lds& L, uint32_t r0, uint32_t n, uint32_t lane,
                                         uint64_t& cnt, uint64_t& kbytes, uint64_t& vbytes, uint64_t e0, uint64_t k0,
                                         uint64_t v0) {
    cnt = kbytes = vbytes = 0;
    if (n < 4) return 0;
    const uint32_t footer = (uint32_t)win8(L.raw, r0 + n - 4);
    const uint32_t nr = footer & 0x7FFFFFFFu;
    uint64_t tail = 4;
    if (footer >> 31) {
        if (n < 6) return 0;
        tail += 2 + ((uint32_t)win8(L.raw, r0 + n - 6) & 0xFFFFu);
    }
    tail += 4ull * nr;
    if (nr == 0 || tail > n) return 0;
    const uint32_t end = r0 + n - (uint32_t)tail;
    uint32_t p = r0, pilen = 0;
    while (p < end) {
        uint32_t shared = 0, nonshared = 0, vlen = 0;
        const uint32_t k = hdr3(L.raw, p, end, shared, nonshared, vlen);
        if (!k) return 0;
        p += k;
        const uint64_t ilen = (uint64_t)shared + nonshared;
        if (shared > pilen || ilen < 8 || (uint64_t)(end - p) < (uint64_t)nonshared + vlen) return 0;
        if (ilen > kKeyCap) return 3;
        const uint32_t ul = (uint32_t)ilen - 8;
        if (EMIT) {
            wcopy<G>(L.key + shared, L.raw + p, nonshared, lane);  // the internal key, rebuilt in place
            wave_sync();
            const uint64_t e = e0 + cnt;
            wstore8<G>(gp(A.keys) + k0 + kbytes, L.key, 0, ul, lane);
            wstore8<G>(gp(A.vals) + v0 + vbytes, L.raw, p + nonshared, vlen, lane);
            if (lane == 0) {
                const uint64_t trailer = win8(L.key, ul);
                gp(A.key_off)[e + 1] = (int32_t)(k0 + kbytes + ul);
                gp(A.seqs)[e] = trailer >> 8;
                gp(A.types)[e] = (uint8_t)(trailer & 0xFFu);
                gp(A.val_off)[e + 1] = v0 + vbytes + vlen;
            }
            wave_sync();
        }
        p += nonshared + vlen;
        pilen = (uint32_t)ilen;
        kbytes += ul;
        vbytes += vlen;
        cnt++;
    }
    return 1;
}

// Tier-0 blocks inflated by sst_count wait for sst_decode in a fixed HBM slot
// (kTier0Raw bytes each, 16-byte stores), so the decode does not inflate again.
template <uint32_t G>
__device__ __forceinline__ void store_slot(GAS uint8_t* dst, const uint8_t* src, uint32_t n, uint32_t lane) {
    GAS u32x4* d16 = reinterpret_cast<GAS u32x4*>(dst);
    const u32x4* s16 = reinterpret_cast<const u32x4*>(src);
    for (uint32_t c = lane; c < (n + 15) / 16; c += G) d16[c] = s16[c];
}

// Count the blocks of tier TIER (tier 0: every block; tier 1: those on the
// tier-1 list) with G lanes per block in RAW-byte LDS slots.  A block larger
// than the slot moves to tier 1 if it fits there, else to tier 2 (as does
// one with a key past the key buffer).
template <uint32_t G, uint32_t RAW, uint32_t TIER>
__device__ __forceinline__ void count_block(const SstArgs& A, BlockLds<RAW>& L, uint64_t b, uint32_t lane) {
    const SstBlock blk = ldblock(A.blocks + b);
    uint64_t cnt = 0, kbytes = 0, vbytes = 0, big_len = 0;
    uint32_t ulen = 0, r0 = 0;
    int st = 0;  // unknown compression types, and (device tables) no data, are malformed
    if ((blk.size == 0 || blk.data) &&
        (blk.compression == 0 || blk.compression == 1 || blk.compression == 4 || blk.compression == 5)) {
        st = wave_inflate<G>(blk, L, r0, ulen, big_len, lane);
        if (st == 1) st = wave_walk<G, false>(A, L, r0, ulen, lane, cnt, kbytes, vbytes, 0, 0, 0);
    }
    if (TIER == 0 && st == 1 && blk.compression != 0)
        store_slot<G>(gp(A.slots) + b * kSstSlot, L.raw, ulen, lane);
    if (lane == 0) {
        if (st == 0) sst_report(A.err, b);
        uint32_t tier = TIER;
        if (st == 3) tier = 2;
        if (st == 2)
            tier = (TIER == 0 && big_len <= kTier1Raw && blk.size <= BlockLds<kTier1Raw>::kComp) ? 1 : 2;
        if (TIER == 0 && tier == 1)
            gp(A.list)[__hip_atomic_fetch_add(gp(A.nlist), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)] =
                (uint32_t)b;
        gp(A.tier)[b] = tier;
        gp(A.rlen)[b] = st == 1 ? ulen : 0;
        gp(A.ulen)[b] = tier == 2 ? (big_len ? big_len : 1) : 0;  // a tier-2 block owns >= 1 raw byte
        gp(A.ne)[b] = st == 1 ? cnt : 0;
        gp(A.kb)[b] = st == 1 ? kbytes : 0;
        gp(A.vb)[b] = st == 1 ? vbytes : 0;
    }
}

// ---- thread-per-block tier-0 count (sst_count_t) ------------------------------
// One thread per block, every block of the call in flight at once: the block
// is inflated straight into its HBM slot and its entries are counted from
// there.  The lane-group kernel (sst_count0) spends its time in the serial tag
// chain -- a dependent LDS round trip and a group-wide copy per tag, four
// groups diverging in one wave (PMC, round 5: ~9 k instructions per wave, 47 %
// issue-active) -- with at most ~56 blocks per CU in flight; here the chain
// is one thread's, 16-byte steps copy literals and matches (a match closer
// than 16 bytes stores its repeating 16-byte pattern, overrunning its end by
// < 16 bytes into the slot's pad, which the next tag overwrites), and the
// memory latency of ~430 blocks per CU overlaps.  Same results and the same
// malformed-block rules as count_block<G, 1024, 0>.
typedef u32x4 __attribute__((aligned(1))) u32x4u;
typedef unsigned __int128 u128;

__device__ __forceinline__ u128 ld16u(const GAS uint8_t* p) {
    const u32x4 v = *(const GAS u32x4u*)p;
    return ((u128)v.w << 96) | ((u128)v.z << 64) | ((u128)v.y << 32) | (u128)v.x;
}
__device__ __forceinline__ void st16u(GAS uint8_t* p, u128 x) {
    u32x4 v;
    v.x = (uint32_t)x; v.y = (uint32_t)(x >> 32); v.z = (uint32_t)(x >> 64); v.w = (uint32_t)(x >> 96);
    *(GAS u32x4u*)p = v;
}
// up to 8 bytes at p, never reading at or past end
__device__ __forceinline__ uint64_t ld8b(const GAS uint8_t* p, const GAS uint8_t* end) {
    if (end - p >= 8) return *(const GAS u64u*)p;
    uint64_t v = 0;
    for (uint32_t i = 0; p + i < end; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
}
// len bytes from src to dst (disjoint, or src < dst with dst - src >= 16), in order
__device__ __forceinline__ void tcopy(GAS uint8_t* dst, const GAS uint8_t* src, uint32_t len) {
    if (len >= 16) {
        uint32_t q = 0;
        for (; q + 16 <= len; q += 16) st16u(dst + q, ld16u(src + q));
        if (q < len) st16u(dst + len - 16, ld16u(src + len - 16));
    } else if (len >= 8) {
        const uint64_t a = *(const GAS u64u*)src, b = *(const GAS u64u*)(src + len - 8);
        *(GAS u64u*)dst = a;
        *(GAS u64u*)(dst + len - 8) = b;
    } else if (len >= 4) {
        const uint32_t a = *(const GAS u32u*)src, b = *(const GAS u32u*)(src + len - 4);
        *(GAS u32u*)dst = a;
        *(GAS u32u*)(dst + len - 4) = b;
    } else {
        for (uint32_t i = 0; i < len; i++) dst[i] = src[i];
    }
}
// out[o, o + len) = out[o - off + (i % off)] (o >= off >= 1); may write up to
// 15 bytes past o + len (slot pad)
__device__ __forceinline__ void tmatch(GAS uint8_t* out, uint32_t o, uint32_t off, uint32_t len) {
    if (off >= 16) {
        tcopy(out + o, out + o - off, len);
        return;
    }
    u128 w = ld16u(out + o - off) & (((u128)1 << (8 * off)) - 1);
    for (uint32_t s = off; s < 16; s *= 2) w |= w << (8 * s);  // period off
    const uint32_t step = (16 / off) * off;
    for (uint32_t q = 0; q < len; q += step) st16u(out + o + q, w);
}

// Snappy body c[p, n) into out[0, ulen); false when malformed (the rules of
// inflate_snappy / winflate_snappy).
__device__ bool tinflate_snappy(const GAS uint8_t* c, uint32_t p, uint32_t n, GAS uint8_t* out, uint32_t ulen) {
    uint32_t o = 0;
    while (p < n) {
        const uint64_t w = ld8b(c + p, c + n);
        const uint32_t tag = (uint32_t)w & 0xFFu;
        p++;
        uint32_t len, off;
        const uint32_t kind = tag & 3u;
        if (kind == 0) {
            len = tag >> 2;
            if (len >= 60) {
                const uint32_t nb = len - 59;
                if (n - p < nb) return false;
                len = (uint32_t)(w >> 8) & (nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1));
                p += nb;
            }
            len += 1;
            if (n - p < len || o + len > ulen) return false;
            tcopy(out + o, c + p, len);
            p += len;
            o += len;
            continue;
        }
        if (kind == 1) {
            if (p >= n) return false;
            len = 4 + ((tag >> 2) & 7u);
            off = ((tag >> 5) << 8) | ((uint32_t)(w >> 8) & 0xFFu);
            p += 1;
        } else if (kind == 2) {
            if (n - p < 2) return false;
            len = 1 + (tag >> 2);
            off = (uint32_t)(w >> 8) & 0xFFFFu;
            p += 2;
        } else {
            if (n - p < 4) return false;
            len = 1 + (tag >> 2);
            off = (uint32_t)(w >> 8);
            p += 4;
        }
        if (off == 0 || off > o || o + len > ulen) return false;
        tmatch(out, o, off, len);
        o += len;
    }
    return o == ulen;
}

__device__ __forceinline__ bool tlz4_ext(const GAS uint8_t* c, uint32_t& p, uint32_t n, uint32_t& v) {
    uint32_t b;
    do {
        if (p >= n) return false;
        b = c[p++];
        v += b;
    } while (b == 255);
    return true;
}
// LZ4 block c[p, n) into out[0, ulen) (the rules of inflate_lz4).
__device__ bool tinflate_lz4(const GAS uint8_t* c, uint32_t p, uint32_t n, GAS uint8_t* out, uint32_t ulen) {
    uint32_t o = 0;
    for (;;) {
        if (p >= n) return false;
        const uint32_t tok = c[p++];
        uint32_t lit = tok >> 4;
        if (lit == 15 && !tlz4_ext(c, p, n, lit)) return false;
        if (n - p < lit || o + lit > ulen) return false;
        tcopy(out + o, c + p, lit);
        p += lit;
        o += lit;
        if (p == n) break;
        if (n - p < 2) return false;
        const uint32_t off = (uint32_t)c[p] | ((uint32_t)c[p + 1] << 8);
        p += 2;
        uint32_t ml = tok & 15u;
        if (ml == 15 && !tlz4_ext(c, p, n, ml)) return false;
        ml += 4;
        if (off == 0 || off > o || o + ml > ulen) return false;
        tmatch(out, o, off, ml);
        o += ml;
    }
    return o == ulen;
}

// Count the entries of the uncompressed block blk[0, n) (readable to
// blk + lim): 1 ok, 0 malformed, 3 an internal key past kKeyCap (wave_walk's rules).
__device__ int twalk(const GAS uint8_t* blk, uint32_t n, const GAS uint8_t* lim, uint64_t& cnt, uint64_t& kbytes,
                     uint64_t& vbytes) {
    cnt = kbytes = vbytes = 0;
    if (n < 4) return 0;
    const uint32_t footer = *(const GAS u32u*)(blk + n - 4);
    const uint32_t nr = footer & 0x7FFFFFFFu;
    uint64_t tail = 4;
    if (footer >> 31) {
        if (n < 6) return 0;
        tail += 2 + (uint32_t)*(const GAS u16u*)(blk + n - 6);
    }
    tail += 4ull * nr;
    if (nr == 0 || tail > n) return 0;
    const uint32_t end = n - (uint32_t)tail;
    uint32_t p = 0, pilen = 0;
    while (p < end) {
        const uint64_t w0 = ld8b(blk + p, lim), w1 = ld8b(blk + p + 8, lim);
        uint32_t v[3], i = 0;
        for (uint32_t k = 0; k < 3; k++) {
            uint32_t r = 0;
            bool done = false;
            for (uint32_t j = 0; j < 5 && !done; j++) {
                if (p + i >= end) return 0;
                const uint32_t byte = (uint32_t)(i < 8 ? w0 >> (8 * i) : w1 >> (8 * (i - 8))) & 0xFFu;
                r |= (byte & 0x7Fu) << (7 * j);
                done = !(byte & 0x80u);
                i++;
            }
            if (!done) return 0;
            v[k] = r;
        }
        p += i;
        const uint32_t shared = v[0], nonshared = v[1], vlen = v[2];
        const uint64_t ilen = (uint64_t)shared + nonshared;
        if (shared > pilen || ilen < 8 || (uint64_t)(end - p) < (uint64_t)nonshared + vlen) return 0;
        if (ilen > kKeyCap) return 3;
        p += nonshared + vlen;
        pilen = (uint32_t)ilen;
        kbytes += ilen - 8;
        vbytes += vlen;
        cnt++;
    }
    return 1;
}

__global__ void __launch_bounds__(256) sst_count_t(SstArgs A) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= A.nblocks) return;
    SstBlock blk = ldblock(A.blocks + b);
    const GAS uint8_t* c = gp(blk.data);
    GAS uint8_t* slot = gp(A.slots) + b * kSstSlot;
    uint64_t cnt = 0, kbytes = 0, vbytes = 0, big_len = 0;
    uint32_t ulen = 0;
    int st = 0;  // unknown compression types, and (device tables) no data, are malformed
    if (blk.size && !blk.data) blk.compression = ~0u;
    if (A.probe & 4) {  // (tuning) pull the stored block's lines into the L2 first
        uint32_t acc = 0;
        for (uint64_t q = 0; q < blk.size; q += 64) acc ^= c[q];
        if (acc == 0x100) sst_report(A.err, b);  // never: keeps the loads
    }
    if (blk.compression == 0) {
        big_len = blk.size;
        if (blk.size > kTier0Raw) {
            st = 2;
        } else {
            ulen = (uint32_t)blk.size;
            st = twalk(c, ulen, c + ulen, cnt, kbytes, vbytes);
        }
    } else if (blk.compression == 1 || blk.compression == 4 || blk.compression == 5) {
        const uint8_t* q = blk.data;
        uint32_t v = 0;
        if (blk.size && varint32(q, blk.data + blk.size, v) && expansion_ok(v, blk.size)) {
            big_len = v;
            if (blk.size > BlockLds<kTier0Raw>::kComp || v > kTier0Raw) {
                st = 2;
            } else {
                ulen = v;
                const uint32_t n = (uint32_t)blk.size, hl = (uint32_t)(q - blk.data);
                const bool ok = (A.probe & 2) ? true
                                : blk.compression == 1 ? tinflate_snappy(c, hl, n, slot, ulen)
                                                       : tinflate_lz4(c, hl, n, slot, ulen);
                st = !ok ? 0 : (A.probe & 3) ? 1 : twalk(slot, ulen, slot + kSstSlot, cnt, kbytes, vbytes);
                if (A.probe & 3) ulen = 0;  // (tuning: an empty block, nothing for the decode)
            }
        }
    }
    if (st == 0) sst_report(A.err, b);
    uint32_t tier = 0;
    if (st == 3) tier = 2;
    if (st == 2) tier = (big_len <= kTier1Raw && blk.size <= BlockLds<kTier1Raw>::kComp) ? 1 : 2;
    if (tier == 1)
        gp(A.list)[__hip_atomic_fetch_add(gp(A.nlist), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)] = (uint32_t)b;
    gp(A.tier)[b] = tier;
    gp(A.rlen)[b] = st == 1 ? ulen : 0;
    gp(A.ulen)[b] = tier == 2 ? (big_len ? big_len : 1) : 0;
    gp(A.ne)[b] = st == 1 ? cnt : 0;
    gp(A.kb)[b] = st == 1 ? kbytes : 0;
    gp(A.vb)[b] = st == 1 ? vbytes : 0;
}

template <uint32_t G>
__global__ void __launch_bounds__(kThreads) sst_count0(SstArgs A) {
    __shared__ BlockLds<kTier0Raw> lds[kThreads / G];
    const uint32_t lane = threadIdx.x % G, slot = threadIdx.x / G;
    const uint64_t b = (uint64_t)blockIdx.x * (kThreads / G) + slot;
    if (b < A.nblocks) count_block<G, kTier0Raw, 0>(A, lds[slot], b, lane);
}

// Tier 1: a wave per block over the tier-1 list (a fixed grid; no work when
// the list is empty).
constexpr uint32_t kTier1Grid = 1024;
__global__ void __launch_bounds__(kThreads) sst_count1(SstArgs A) {
    __shared__ BlockLds<kTier1Raw> lds[kThreads / 64];
    const uint32_t lane = threadIdx.x % 64, slot = threadIdx.x / 64;
    const uint32_t nl = __hip_atomic_load(gp(A.nlist), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t i = blockIdx.x * (kThreads / 64) + slot; i < nl; i += gridDim.x * (kThreads / 64))
        count_block<64, kTier1Raw, 1>(A, lds[slot], gp(A.list)[i], lane);
}

template <uint32_t G, class Lds, bool FROM_SLOT>
__device__ __forceinline__ void decode_block(const SstArgs& A, Lds& L, uint64_t b, uint32_t lane) {
    const SstBlock blk = ldblock(A.blocks + b);
    uint64_t cnt, kbytes, vbytes, big_len;
    uint32_t ulen = 0, r0 = 0;
    int st = 1;
    if (FROM_SLOT) {  // tier 0: the stored block if plain, else its slot (inflated by sst_count)
        ulen = gp(A.rlen)[b];
        r0 = stage<G>(L.raw, blk.compression == 0 ? blk.data : A.slots + b * kSstSlot, ulen, lane);
        wave_sync();
    } else {
        st = wave_inflate<G>(blk, L, r0, ulen, big_len, lane);
    }
    // sst_count accepted the block: this walk repeats it and writes the entries
    if (st == 1)
        (void)wave_walk<G, true>(A, L, r0, ulen, lane, cnt, kbytes, vbytes, gp(A.eoff)[b], gp(A.koff)[b],
                                 gp(A.voff)[b]);
}

template <uint32_t G>
__global__ void __launch_bounds__(kThreads) sst_decode0(SstArgs A) {
    __shared__ BlockLds<kTier0Raw, false> lds[kThreads / G];
    const uint32_t lane = threadIdx.x % G, slot = threadIdx.x / G;
    const uint64_t b = (uint64_t)blockIdx.x * (kThreads / G) + slot;
    if (b < A.nblocks && gp(A.tier)[b] == 0) decode_block<G, BlockLds<kTier0Raw, false>, true>(A, lds[slot], b, lane);
}

__global__ void __launch_bounds__(kThreads) sst_decode1(SstArgs A) {
    __shared__ BlockLds<kTier1Raw> lds[kThreads / 64];
    const uint32_t lane = threadIdx.x % 64, slot = threadIdx.x / 64;
    const uint32_t nl = __hip_atomic_load(gp(A.nlist), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t i = blockIdx.x * (kThreads / 64) + slot; i < nl; i += gridDim.x * (kThreads / 64)) {
        const uint32_t b = gp(A.list)[i];
        if (gp(A.tier)[b] == 1) decode_block<64, BlockLds<kTier1Raw>, false>(A, lds[slot], b, lane);
    }
}

// Exclusive scans of u64 arrays (ScanSet): chunk scans of 1024 (sums into
// part[]), one workgroup per array over its chunk sums, then the add-back.
__device__ uint64_t block_scan1024(uint64_t v, uint64_t* s_w, uint64_t* total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = (uint64_t)__shfl_up((unsigned long long)inc, d, 64);
        if (lane >= (uint32_t)d) inc += o;
    }
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
    for (uint32_t w = 0; w < 16; w++) {
        before += w < wave ? s_w[w] : 0;
        all += s_w[w];
    }
    __syncthreads();
    *total = all;
    return before + inc - v;
}
// The same over up to four arrays at once (blockIdx.y picks the array): three
// launches for the count pass's four scans instead of twelve.
__global__ void __launch_bounds__(1024) scan_chunks_n(ScanSet S, uint64_t n, uint64_t nparts) {
    __shared__ uint64_t s_w[16];
    const uint32_t k = blockIdx.y;
    const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    const uint64_t v = i < n ? gp(S.x[k])[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_scan1024(v, s_w, &tot);
    if (i < n) gp(S.y[k])[i] = ex;
    if (threadIdx.x == 0) gp(S.part)[k * nparts + blockIdx.x] = tot;
}
__global__ void __launch_bounds__(1024) scan_parts_n(ScanSet S, uint64_t nparts) {
    __shared__ uint64_t s_w[16];
    const uint32_t k = blockIdx.x;
    uint64_t* part = S.part + k * nparts;
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nparts; base += 1024) {
        const uint64_t j = base + threadIdx.x;
        const uint64_t v = j < nparts ? gp(part)[j] : 0;
        uint64_t tot;
        const uint64_t ex = block_scan1024(v, s_w, &tot);
        if (j < nparts) gp(part)[j] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) gp(S.total[k])[0] = carry;
}
__global__ void __launch_bounds__(1024) scan_add_n(ScanSet S, uint64_t n, uint64_t nparts) {
    const uint32_t k = blockIdx.y;
    const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    if (i < n) gp(S.y[k])[i] += gp(S.part)[k * nparts + blockIdx.x];
}

}  // namespace

// Tier-0 count: the thread-per-block kernel (sst_count_t); tuning builds can
// pick the lane-group one (MURR_SST_LANES 4 to 64).  Lanes per tier-0 block of
// sst_decode: kDecodeLanes (MURR_SST_DLANES).
constexpr uint32_t kDecodeLanes = 8;
uint32_t lanes_env(const char* name, uint32_t dflt) {
#ifdef MURR_TUNING
    const char* e = std::getenv(name);
    const uint32_t v = e ? (uint32_t)std::atoi(e) : dflt;
    return (v == 1 || v == 4 || v == 8 || v == 16 || v == 32 || v == 64) ? v : dflt;
#else
    (void)name;
    return dflt;
#endif
}
template <uint32_t G>
hipError_t launch_tier0(bool decode, const SstArgs& a, hipStream_t s) {
    const dim3 grid((uint32_t)((a.nblocks + kThreads / G - 1) / (kThreads / G)));
    if (decode) hipLaunchKernelGGL(sst_decode0<G>, grid, dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL(sst_count0<G>, grid, dim3(kThreads), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_tiers(bool decode, const SstArgs& a_in, hipStream_t s) {
    SstArgs a = a_in;
#ifdef MURR_TUNING
    // phase ablations of sst_count_t (compressed blocks then read as empty):
    // 1 no walk, 2 no inflate and no walk, 4 prefetch the stored block
    static const uint32_t probe = std::getenv("MURR_SST_PROBE") ? (uint32_t)std::atoi(std::getenv("MURR_SST_PROBE")) : 0;
    a.probe = probe;
#endif
    static const uint32_t gc = lanes_env("MURR_SST_LANES", 1);  // 1: the thread-per-block count
    static const uint32_t gd = lanes_env("MURR_SST_DLANES", kDecodeLanes);
    hipError_t e;
    if (!decode && gc == 1) {
        hipLaunchKernelGGL(sst_count_t, dim3((uint32_t)((a.nblocks + 255) / 256)), dim3(256), 0, s, a);
        e = hipGetLastError();
    } else switch (decode ? gd : gc) {
    case 4: e = launch_tier0<4>(decode, a, s); break;
    case 8: e = launch_tier0<8>(decode, a, s); break;
    case 32: e = launch_tier0<32>(decode, a, s); break;
    case 64: e = launch_tier0<64>(decode, a, s); break;
    default: e = launch_tier0<16>(decode, a, s); break;
    }
    if (e != hipSuccess) return e;
    // tier 1 right behind tier 0, over the list tier 0's count made
    if (decode) hipLaunchKernelGGL(sst_decode1, dim3(kTier1Grid), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL(sst_count1, dim3(kTier1Grid), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_sst_count(const SstArgs& a, hipStream_t s) { return launch_tiers(false, a, s); }
hipError_t launch_sst_big_count(const SstArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(sst_big_count, dim3((uint32_t)((a.nblocks + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_sst_decode(const SstArgs& a, hipStream_t s) { return launch_tiers(true, a, s); }
hipError_t launch_sst_big_decode(const SstArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(sst_big_decode, dim3((uint32_t)((a.nblocks + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_scan_u64_n(const ScanSet& S, uint64_t n, hipStream_t s) {
    const uint64_t nparts = (n + 1023) / 1024;
    if (nparts) hipLaunchKernelGGL(scan_chunks_n, dim3((uint32_t)nparts, S.k), dim3(1024), 0, s, S, n, nparts);
    hipLaunchKernelGGL(scan_parts_n, dim3(S.k), dim3(1024), 0, s, S, nparts);
    if (nparts) hipLaunchKernelGGL(scan_add_n, dim3((uint32_t)nparts, S.k), dim3(1024), 0, s, S, n, nparts);
    return hipGetLastError();
}

}  // namespace murr
