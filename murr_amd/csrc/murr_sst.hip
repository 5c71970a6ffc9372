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
// One thread per block (blocks are ~512 B and a launch holds many): the
// uncompressed length, the decompression, the entry count and the entry
// decode are four passes, with device scans between them placing every
// block's bytes and entries.  HBM-bound in principle; byte-serial per thread
// in practice.
#include "murr_device.h"

namespace murr {

namespace {

using namespace dev;

constexpr uint32_t kSstCorrupt = 5;  // err_key status: MURR_E_MALFORMED_ROW (row = block index)

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

// Pass 1: uncompressed length of every block.
__global__ void __launch_bounds__(256) sst_len(SstArgs A) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= A.nblocks) return;
    const SstBlock blk = ldblock(A.blocks + b);
    uint64_t len = blk.size;
    if (blk.compression == 1 || blk.compression == 4 || blk.compression == 5) {  // Snappy, LZ4, LZ4HC
        const uint8_t* p = blk.data;
        uint32_t v = 0;
        if (!varint32(p, blk.data + blk.size, v)) {
            sst_report(A.err, b);
            v = 0;
        }
        len = v;
    } else if (blk.compression != 0) {
        sst_report(A.err, b);
        len = 0;
    }
    gp(A.ulen)[b] = len;
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

// Pass 2: decompress (or copy) block b to raw + uoff[b].
__global__ void __launch_bounds__(256) sst_inflate(SstArgs A) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= A.nblocks) return;
    const SstBlock blk = ldblock(A.blocks + b);
    GAS uint8_t* dst = gp(A.raw) + gp(A.uoff)[b];
    const uint64_t ulen = gp(A.ulen)[b];
    bool ok = true;
    if (blk.compression == 0)
        for (uint64_t i = 0; i < ulen; i++) dst[i] = gp(blk.data)[i];
    else if (blk.compression == 1)
        ok = inflate_snappy(blk.data, blk.data + blk.size, dst, ulen);
    else if (blk.compression == 4 || blk.compression == 5)
        ok = inflate_lz4(blk.data, blk.data + blk.size, dst, ulen);
    // other types were reported by sst_len
    if (!ok) sst_report(A.err, b);
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

// Passes 3 and 4: walk block b's entries; count (emit false) or write them.
template <bool EMIT>
__device__ void sst_walk(const SstArgs& A, uint64_t b) {
    const uint8_t* blk = A.raw + gp(A.uoff)[b];
    const uint64_t n = gp(A.ulen)[b];
    uint64_t limit = 0;
    if (!block_layout(blk, n, limit)) {
        if (!EMIT) sst_report(A.err, b);
        if (!EMIT) gp(A.ne)[b] = gp(A.kb)[b] = gp(A.vb)[b] = 0;
        return;
    }
    const uint8_t* p = blk;
    const uint8_t* end = blk + limit;
    uint64_t cnt = 0, kbytes = 0, vbytes = 0;
    uint64_t e0 = 0, k0 = 0, v0 = 0;
    if (EMIT) {
        e0 = gp(A.ne)[b];
        k0 = gp(A.kb)[b];
        v0 = gp(A.vb)[b];
    }
    uint64_t pstart = 0;     // previous user key: output position and length
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

__global__ void __launch_bounds__(256) sst_count(SstArgs A) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b < A.nblocks) sst_walk<false>(A, b);
}
__global__ void __launch_bounds__(256) sst_decode(SstArgs A) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b < A.nblocks) sst_walk<true>(A, b);
}

// Exclusive scan of u64 x[0..n) in place, total at x[n]: chunk scans of 1024
// (sums into part[]), one workgroup over the chunk sums, then the add-back.
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
__global__ void __launch_bounds__(1024) scan_chunks(uint64_t* x, uint64_t n, uint64_t* part) {
    __shared__ uint64_t s_w[16];
    const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    const uint64_t v = i < n ? gp(x)[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_scan1024(v, s_w, &tot);
    if (i < n) gp(x)[i] = ex;
    if (threadIdx.x == 0) gp(part)[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(1024) scan_parts(uint64_t* part, uint64_t nparts, uint64_t* total) {
    __shared__ uint64_t s_w[16];
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nparts; base += 1024) {
        const uint64_t j = base + threadIdx.x;
        const uint64_t v = j < nparts ? gp(part)[j] : 0;
        uint64_t tot;
        const uint64_t ex = block_scan1024(v, s_w, &tot);
        if (j < nparts) gp(part)[j] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) gp(total)[0] = carry;
}
__global__ void __launch_bounds__(1024) scan_add(uint64_t* x, uint64_t n, const uint64_t* part) {
    const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    if (i < n) gp(x)[i] += gp(part)[blockIdx.x];
}

}  // namespace

hipError_t launch_sst_len(const SstArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(sst_len, dim3((uint32_t)((a.nblocks + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_sst_inflate(const SstArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(sst_inflate, dim3((uint32_t)((a.nblocks + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_sst_count(const SstArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(sst_count, dim3((uint32_t)((a.nblocks + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_sst_decode(const SstArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(sst_decode, dim3((uint32_t)((a.nblocks + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}
// x[0..n) -> exclusive prefix, total -> *total; part: ceil(n / 1024) scratch.
hipError_t launch_scan_u64(uint64_t* x, uint64_t n, uint64_t* part, uint64_t* total, hipStream_t s) {
    const uint64_t nparts = (n + 1023) / 1024;
    if (nparts) hipLaunchKernelGGL(scan_chunks, dim3((uint32_t)nparts), dim3(1024), 0, s, x, n, part);
    hipLaunchKernelGGL(scan_parts, dim3(1), dim3(1024), 0, s, part, nparts, total);
    if (nparts) hipLaunchKernelGGL(scan_add, dim3((uint32_t)nparts), dim3(1024), 0, s, x, n, (const uint64_t*)part);
    return hipGetLastError();
}

}  // namespace murr
