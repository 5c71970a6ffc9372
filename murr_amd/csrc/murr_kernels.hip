// murr_kernels.hip — gfx950 encode kernel: Arrow buffers -> row blobs.
//
// Replaces Table::write's row loop with WriteRow + ColumnDecoders
// (src/io/table/mod.rs:97-109, src/io/row/write.rs:19-52, primitive.rs:85-95,
// bool_.rs:111-117, utf8.rs:113-119).  The decode kernel is in murr_decode.hip.
//
// Byte movement: HBM-bound, no MFMA.  One workgroup = 4 waves = one 256-row
// tile, thread-per-row.  Row sizes are scanned (wave scan, LDS combine across
// the 4 waves, one-hop window sum across tiles: window_prefix); rows are
// assembled in LDS and written out with 16-B coalesced stores.  Tiles are
// assigned round-robin to a persistent grid that fits on the chip at once, so
// every tile a prefix waits on is resident or finished.
#include "murr_device.h"

namespace murr {

namespace {

using namespace dev;

// Block-wide (256 threads) inclusive scan; returns inclusive value, sets *agg.
__device__ __forceinline__ uint64_t block_incl_scan(uint64_t x, uint64_t* s_w, uint64_t* agg) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = wave_incl_scan64(x, lane);
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
            A.row_off[row] = A.row_base + start;
            if (row + 1 == A.n_rows) A.row_off[row + 1] = A.row_base + start + size;
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


// ---- segment copies over PCIe (streaming host decode, murr_abi.cpp hstream) ----
// A list of (src, dst, bytes) copies done by one grid of 256-thread
// workgroups: pinned host -> device (the batch's blob and row offsets, and
// the decode's descriptors) or device -> pinned host (the decoded buffers and
// the decode's counters), the other side of PCIe read or written directly by
// the CUs -- no copy engine, no per-copy command, no cross-stream event.  A
// segment may take its length from a device int32 (a utf8 column's final
// offset: exactly its decoded bytes, clamped to `bytes`).  Each workgroup step
// moves one 16 KiB chunk: four 16-B loads per lane issued before their
// stores, so a wave keeps 4 KiB of PCIe reads in flight.
constexpr uint64_t kCopyChunk = 256 * 4 * 16;

__device__ __forceinline__ uint64_t seg_bytes(const CopySeg& g) {
    if (!g.len) return g.bytes;
    const int32_t v = *(const CAS int32_t*)g.len;
    return v <= 0 ? 0 : ((uint64_t)v < g.bytes ? (uint64_t)v : g.bytes);
}

__global__ void __launch_bounds__(256) copy_segs_kernel(CopyArgs A) {
    const uint32_t tid = threadIdx.x;
    for (uint64_t c = blockIdx.x;; c += gridDim.x) {
        // the segment holding chunk c (uniform; at most kMaxCopySegs steps)
        uint32_t s = 0;
        uint64_t base = 0, nb = 0;
        for (; s < A.nseg; s++) {
            nb = seg_bytes(A.seg[s]);
            const uint64_t nc = (nb + kCopyChunk - 1) / kCopyChunk;
            if (c < base + nc) break;
            base += nc;
        }
        if (s >= A.nseg) break;
        const uint64_t off = (c - base) * kCopyChunk;
        const uint64_t n = nb - off < kCopyChunk ? nb - off : kCopyChunk;
        const uint8_t* src = A.seg[s].src + off;
        uint8_t* dst = A.seg[s].dst + off;
        if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
            const uint64_t nv = n >> 4;
            const u32x4* sv = (const u32x4*)src;
            u32x4* dv = (u32x4*)dst;
            u32x4 v[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint64_t i = tid + 256 * k;
                if (i < nv) v[k] = __builtin_nontemporal_load(sv + i);
            }
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint64_t i = tid + 256 * k;
                if (i < nv) __builtin_nontemporal_store(v[k], dv + i);
            }
            const uint64_t t0 = nv << 4;
            if (t0 + tid < n) dst[t0 + tid] = src[t0 + tid];
        } else if ((((uintptr_t)src | (uintptr_t)dst) & 7) == 0) {
            const uint64_t nq = n >> 3;
            for (uint64_t i = tid; i < nq; i += 256) ((uint64_t*)dst)[i] = ((const uint64_t*)src)[i];
            const uint64_t t0 = nq << 3;
            if (t0 + tid < n) dst[t0 + tid] = src[t0 + tid];
        } else {
            for (uint64_t i = tid; i < n; i += 256) dst[i] = src[i];
        }
    }
}

// ---- row-offset widths (murr_block_t.row_off32) -------------------------------
// u64 -> u32 (murr_row_off_narrow).  Both decode kernels read either width
// natively.  Every offset is checked, not only the last (a malformed block's
// interior offset would otherwise be truncated into a plausible row span):
// bit 0 of *bad = some offset >= 2^32, bit 1 = some offset below its
// predecessor.  *bad is zeroed by the host before the launch.
__global__ void __launch_bounds__(256) narrow_kernel(const uint64_t* __restrict__ in, uint32_t* __restrict__ out,
                                                     uint64_t n, unsigned int* __restrict__ bad) {
    unsigned int f = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t v = in[i];
        out[i] = (uint32_t)v;
        f |= (v >> 32) ? 1u : 0u;
        f |= i && v < in[i - 1] ? 2u : 0u;
    }
    if (__any(f != 0)) atomicOr(bad, f);
}

}  // namespace

hipError_t launch_row_off_narrow(const uint64_t* in, uint32_t* out, uint64_t n, unsigned int* bad, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint64_t g = (n + 255) / 256;
    hipLaunchKernelGGL(narrow_kernel, dim3((uint32_t)(g < 4096 ? g : 4096)), dim3(256), 0, s, in, out, n, bad);
    return hipGetLastError();
}

hipError_t launch_encode(const EncodeArgs& a, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(encode_kernel, dim3(grid), dim3(kTile), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_copy_segs(const CopySeg* segs, uint32_t n, uint32_t grid, hipStream_t s) {
    for (uint32_t i = 0; i < n; i += kMaxCopySegs) {
        CopyArgs a{};
        a.nseg = n - i < kMaxCopySegs ? n - i : kMaxCopySegs;
        uint64_t bound = 0;
        for (uint32_t k = 0; k < a.nseg; k++) {
            a.seg[k] = segs[i + k];
            bound += (segs[i + k].bytes + kCopyChunk - 1) / kCopyChunk;
        }
        if (!bound) continue;
        hipLaunchKernelGGL(copy_segs_kernel, dim3((uint32_t)(bound < grid ? bound : grid)), dim3(256), 0, s, a);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

int encode_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, encode_kernel, kTile, 0) != hipSuccess) return 1;
    return n;
}

}  // namespace murr
