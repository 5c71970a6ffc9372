// murr_index.hip — device-resident key index and row gather (SURVEY.md §8(f)
// rank 1): the point lookups of Store::read for a table held in HBM.
//
// Replaces, for a resident table, RocksDBStore::read's key lookups and its
// serial present/missing feed (src/io/store/rocksdb/mod.rs:241-267;
// MemoryStore::read, src/io/store/memory.rs:28-45): every query key is looked
// up in an open-addressing hash table, and the hit rows are gathered back to
// back into a block in caller order (a miss = an empty row, which the decode
// turns into ReadBatchBuilder::add_empty, src/io/row/read.rs:93-98).  Writes
// follow put semantics: of equal keys the later row wins (memory.rs:47-56,
// RocksDB's newest sequence number).
//
// Table: capacity = 2^k >= 3n slots of u64 {hash tag (32) | row (32)}, empty
// = ~0, and beside each slot the key's {start (32) | length (32)} in the
// index's key copy, so a probe reads slot and key location together and then
// the key bytes.  Insert is lock-free: CAS into the first empty slot of the linear
// probe sequence, or atomicMax onto the slot of an equal key (same tag, so
// the max picks the larger row = the later write).  Two inserts of one key
// see the same probe sequence and meet at the same slot, so keys stay unique.
// All integer work; the lookup is latency-bound (query key, slot + location,
// stored key: three dependent memory round trips per probe), the gather an
// HBM-bound byte copy.
#include "murr_device.h"

namespace murr {

namespace {

using namespace dev;

constexpr uint64_t kEmpty = ~0ull;

// Keys are read as the aligned dwords that cover them (an aligned dword never
// crosses a page, so the bytes around a key are safe to load whatever buffer
// it sits in) and realigned with v_alignbyte into key words: word j = key
// bytes [4j, 4j + 4), the last one zero-padded.  Eight words (32 bytes) per
// chunk with their loads issued together, so a short key costs one memory
// round trip instead of one per byte.
constexpr uint32_t kChunkWords = 8;

struct KeyChunk {
    uint32_t w[kChunkWords];
};

// Words [8c, 8c + 8) of the key at p (n bytes); words past the end are 0.
__device__ __forceinline__ KeyChunk key_chunk(const GAS uint8_t* p, uint32_t n, uint32_t c) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t sa = (uint32_t)(a & 3);
    const GAS uint32_t* al = (const GAS uint32_t*)(a - sa);
    const uint32_t nal = (sa + n + 3) >> 2;  // aligned dwords covering the key
    uint32_t raw[kChunkWords + 1];
#pragma unroll
    for (uint32_t k = 0; k <= kChunkWords; k++) {
        const uint32_t idx = kChunkWords * c + k;
        raw[k] = idx < nal ? al[idx] : 0u;
    }
    KeyChunk out;
#pragma unroll
    for (uint32_t k = 0; k < kChunkWords; k++) {
        uint32_t v = __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sa);
        const int32_t left = (int32_t)n - 4 * (int32_t)(kChunkWords * c + k);  // key bytes in this word
        if (left <= 0) v = 0;
        else if (left < 4) v &= (1u << (8 * left)) - 1u;
        out.w[k] = v;
    }
    return out;
}

__device__ __forceinline__ uint64_t mix_words(uint64_t h, const KeyChunk& k) {
#pragma unroll
    for (uint32_t j = 0; j < kChunkWords; j++) h = (h ^ k.w[j]) * 0x100000001b3ull;
    return h;
}

// Hash of the key bytes (whatever their alignment): FNV-style over the
// zero-padded key words and the length, finished with the murmur3 avalanche
// (fmix64) so the low bits (slot) and high bits (tag) are both well mixed.
// *first gets the first chunk (all a short key's comparison needs).
__device__ __forceinline__ uint64_t key_hash(const GAS uint8_t* k, uint32_t n, KeyChunk* first) {
    uint64_t h = 0xcbf29ce484222325ull ^ n;
    *first = key_chunk(k, n, 0);
    h = mix_words(h, *first);
    for (uint32_t c = 1; kChunkWords * 4 * c < n; c++) h = mix_words(h, key_chunk(k, n, c));
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return h;
}

__device__ __forceinline__ bool chunk_eq(const KeyChunk& a, const KeyChunk& b) {
    uint32_t d = 0;
#pragma unroll
    for (uint32_t j = 0; j < kChunkWords; j++) d |= a.w[j] ^ b.w[j];
    return d == 0;
}

// Keys a and q of the same length n; qc = q's first chunk.
__device__ __forceinline__ bool key_eq(const GAS uint8_t* a, const KeyChunk& qc, const GAS uint8_t* q, uint32_t n) {
    if (!chunk_eq(key_chunk(a, n, 0), qc)) return false;
    for (uint32_t c = 1; kChunkWords * 4 * c < n; c++)
        if (!chunk_eq(key_chunk(a, n, c), key_chunk(q, n, c))) return false;
    return true;
}

__global__ void __launch_bounds__(256) index_insert(IndexArgs A) {
    const uint64_t i = A.base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // key i is row i
    if (i >= A.base + A.n) return;
    const GAS int32_t* ko = gp(A.key_off);
    const int32_t k0 = ko[i], k1 = ko[i + 1];
    const uint32_t len = (uint32_t)(k1 - k0);
    const GAS uint8_t* key = gp(A.key_data) + k0;
    KeyChunk kc;
    const uint64_t h = key_hash(key, len, &kc);
    const uint64_t mine = (h & 0xFFFFFFFF00000000ull) | i;
    GAS unsigned long long* slots = (GAS unsigned long long*)gp(A.slots);
    uint64_t s = h & A.mask;
    for (uint64_t probe = 0; probe <= A.mask; probe++, s = (s + 1) & A.mask) {
        unsigned long long e = __hip_atomic_load(slots + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (e == kEmpty) {
            unsigned long long want = kEmpty;
            if (__hip_atomic_compare_exchange_strong(slots + s, &want, (unsigned long long)mine, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                // where a probe finds the key bytes; equal keys share them, so
                // the row a later atomicMax installs needs no update here
                gp(A.loc)[s] = ((uint64_t)(uint32_t)k0 << 32) | len;
                if (A.kp) {  // the key's first 16 bytes (a key of <= 16 compares here alone)
                    gp(A.kp)[2 * s] = ((uint64_t)kc.w[1] << 32) | kc.w[0];
                    gp(A.kp)[2 * s + 1] = ((uint64_t)kc.w[3] << 32) | kc.w[2];
                }
                return;
            }
            e = want;  // another key took it first
        }
        if ((e >> 32) == (mine >> 32)) {
            // (loc[s] may not be written yet: compare through the row's offsets)
            const uint32_t r = (uint32_t)e;
            const int32_t o0 = ko[r];
            if ((uint32_t)(ko[r + 1] - o0) == len && key_eq(gp(A.key_data) + o0, kc, key, len)) {
                __hip_atomic_fetch_max(slots + s, (unsigned long long)mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
        }
    }
    report(A.err, err_key(0, i, 0, kStInternal));  // table full: cannot happen at load <= 1/3
}

// Slot holding stored key i (inserted already): index_probe's walk over the
// index's own key copy.
__device__ __forceinline__ uint64_t slot_of(const IndexArgs& A, uint64_t i) {
    const GAS int32_t* ko = gp(A.key_off);
    const int32_t k0 = ko[i];
    const uint32_t len = (uint32_t)(ko[i + 1] - k0);
    const GAS uint8_t* key = gp(A.key_data) + k0;
    KeyChunk kc;
    const uint64_t h = key_hash(key, len, &kc);
    const GAS uint64_t* slots = gp(A.slots);
    const GAS uint64_t* loc = gp(A.loc);
    uint64_t s = h & A.mask;
    for (uint64_t probe = 0; probe <= A.mask; probe++, s = (s + 1) & A.mask) {
        const uint64_t e = slots[s], l = loc[s];
        if (e == kEmpty) break;
        if ((e >> 32) == (h >> 32) && (uint32_t)l == len && key_eq(gp(A.key_data) + (uint32_t)(l >> 32), kc, key, len))
            return s;
    }
    return kEmpty;
}

// Equal keys resolved by sequence number instead of row (SST entries: RocksDB
// keeps a user key's versions newest first, and overlapping files repeat
// keys in any order; the version with the highest sequence number is the
// live one, DBImpl's read path).  Phase 0, per row: best[slot] = max seq;
// phase 1, per row holding that seq: win[slot] = max row + 1 (equal seqs:
// the later row); phase 2, per slot: install the winner.
__global__ void __launch_bounds__(256) index_seq(IndexArgs A, const uint64_t* seqs, unsigned long long* best,
                                                 unsigned long long* win, uint32_t phase) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (phase == 2) {
        if (i > A.mask) return;
        const uint64_t w = gp(win)[i];
        if (w) gp(A.slots)[i] = (gp(A.slots)[i] & 0xFFFFFFFF00000000ull) | (w - 1);
        return;
    }
    if (i >= A.n) return;
    const uint64_t s = slot_of(A, i);
    if (s == kEmpty) {
        report(A.err, err_key(0, i, 0, kStInternal));
        return;
    }
    const uint64_t q = gp(seqs)[i];
    if (phase == 0) __hip_atomic_fetch_max(gp(best) + s, (unsigned long long)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (q == gp(best)[s])
        __hip_atomic_fetch_max(gp(win) + s, (unsigned long long)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The slot cache of row i (i in [from, n)): its slot's row offset, size and
// utf8 string bytes, written only when the slot holds row i (a key written
// again: its later row is the one in the slot, and that row's thread writes).
__global__ void __launch_bounds__(256) index_cache_rows(IndexArgs A, const uint64_t* row_off, const uint32_t* ulen,
                                                        uint64_t from) {
    const uint64_t i = from + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n) return;
    const uint64_t s = slot_of(A, i);
    if (s == kEmpty || (uint32_t)gp(A.slots)[s] != (uint32_t)i) return;
    const uint64_t o0 = gp(row_off)[i], o1 = gp(row_off)[i + 1];
    gp(A.rc)[2 * s] = o0;
    gp(A.rc)[2 * s + 1] = o1 - o0;
    for (uint32_t u = 0; u < A.nu_rc; u++) gp(A.ru)[s * A.nu_rc + u] = gp(ulen)[i * A.nu_rc + u];
}

// Row of query i, or kMissing.  With `size` (a gather): the row's blob
// length too, its two row offsets loaded beside the candidate's key bytes --
// a tag match is the row with near certainty, so the lengths need no round
// trip of their own after the compare (query key, slot + location, stored key
// and row offsets: three dependent round trips, not four).
template <bool SIZED = false>
__device__ __forceinline__ uint32_t probe_one(const IndexArgs& A, uint64_t i, uint64_t* size = nullptr,
                                              uint64_t* start = nullptr, uint32_t* ul = nullptr) {
    const GAS int32_t* qo = gp(A.q_off);
    const int32_t q0 = qo[i];
    const uint32_t len = (uint32_t)(qo[i + 1] - q0);
    const GAS uint8_t* q = gp(A.q_data) + q0;
    KeyChunk qc;
    const uint64_t h = key_hash(q, len, &qc);
    const GAS uint64_t* slots = gp(A.slots);
    const GAS uint64_t* loc = gp(A.loc);
    uint32_t row = kMissing;
    uint64_t s = h & A.mask;
    if constexpr (SIZED) {
        if (A.rc) {
            // slot cache (murr_index_cache_rows): the slot's key prefix, row
            // offset, size and string bytes come with the slot, so a key of
            // <= 16 bytes resolves in this round trip
            const uint64_t q0 = ((uint64_t)qc.w[1] << 32) | qc.w[0], q1 = ((uint64_t)qc.w[3] << 32) | qc.w[2];
            for (uint64_t probe = 0; probe <= A.mask; probe++, s = (s + 1) & A.mask) {
                const uint64_t e = slots[s], l = loc[s];  // independent loads
                const uint64_t p0 = gp(A.kp)[2 * s], p1 = gp(A.kp)[2 * s + 1];
                const uint64_t c0 = gp(A.rc)[2 * s], c1 = gp(A.rc)[2 * s + 1];
                uint32_t u4[kGatherMaxU] = {0, 0, 0, 0};
                if (ul) {
#pragma unroll
                    for (uint32_t u = 0; u < kGatherMaxU; u++)
                        if (u < A.nu_rc) u4[u] = gp(A.ru)[s * A.nu_rc + u];
                }
                if (e == kEmpty) break;
                if ((e >> 32) == (h >> 32) && (uint32_t)l == len && p0 == q0 && p1 == q1 &&
                    (len <= 16 || key_eq(gp(A.key_data) + (uint32_t)(l >> 32), qc, q, len))) {
                    row = (uint32_t)e;
                    *size = c1;
                    if (start) *start = c0;
                    if (ul) {
#pragma unroll
                        for (uint32_t u = 0; u < kGatherMaxU; u++) ul[u] = u4[u];
                    }
                    break;
                }
            }
            return row;
        }
    }
    for (uint64_t probe = 0; probe <= A.mask; probe++, s = (s + 1) & A.mask) {
        const uint64_t e = slots[s], l = loc[s];  // independent loads
        if (e == kEmpty) break;
        if ((e >> 32) == (h >> 32) && (uint32_t)l == len) {
            uint64_t o0 = 0, o1 = 0;
            uint32_t u4[kGatherMaxU] = {0, 0, 0, 0};
            if constexpr (SIZED) {
                o0 = gp(A.row_off)[(uint32_t)e];
                o1 = gp(A.row_off)[(uint32_t)e + 1];
                if (ul) {  // (the row's utf8 string bytes, in the same round trip)
#pragma unroll
                    for (uint32_t u = 0; u < kGatherMaxU; u++)
                        if (u < A.nu) u4[u] = gp(A.ulen)[(uint64_t)(uint32_t)e * A.nu + u];
                }
            }
            if (key_eq(gp(A.key_data) + (uint32_t)(l >> 32), qc, q, len)) {
                row = (uint32_t)e;
                if constexpr (SIZED) {
                    *size = o1 - o0;
                    if (start) *start = o0;
                    if (ul) {
#pragma unroll
                        for (uint32_t u = 0; u < kGatherMaxU; u++) ul[u] = u4[u];
                    }
                }
                break;
            }
        }
    }
    return row;
}


// One query per thread: rows[i] = the key's row or kMissing; sizes[i] = its
// blob length (0 for a miss) when a gather follows.
// Queries that are looked up: [0, nq_live) when nq_live is set (a prepared
// read padded to its capacity: the rest are misses), else all nq.
__device__ __forceinline__ uint64_t live_queries(const IndexArgs& A) { return A.nq_live ? A.nq_live : A.nq; }

__global__ void __launch_bounds__(256) index_probe(IndexArgs A) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.nq) return;
    uint64_t sz = 0;
    uint32_t row = kMissing;
    if (i < live_queries(A)) row = A.sizes ? probe_one<true>(A, i, &sz) : probe_one(A, i);
    if (A.rows) gp(A.rows)[i] = row;
    if (A.sizes) gp(A.sizes)[i] = sz;
}

// Exclusive scan of sizes[0..nq) in place into block row offsets, in groups
// of kScanGroup entries per 1024-thread workgroup:
//   pass 0: group sums -> sums[g];
//   pass 2: one workgroup scans sums[] (exclusive) and writes the total;
//   pass 1: each group rewrites its entries as offsets (sums[g] + local prefix).
// A single group runs pass 1 alone with a zero group prefix.  Offsets are
// clamped to out_cap so the block never points past its buffer; the true
// total goes to *needed.
constexpr uint32_t kScanThreads = 1024, kScanPer = 4, kScanGroup = kScanThreads * kScanPer;

__device__ uint64_t block_excl1024(uint64_t x, uint64_t* s_t, uint64_t* total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t inc = wave_incl_scan64(x, lane);
    if (lane == 63) s_t[wave] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kScanThreads / 64; w++) {
        const uint64_t v = s_t[w];
        before += w < wave ? v : 0u;
        all += v;
    }
    __syncthreads();
    *total = all;
    return before + inc - x;
}

__global__ void __launch_bounds__(kScanThreads) gather_scan(IndexArgs A, uint32_t pass) {
    __shared__ uint64_t s_t[kScanThreads / 64];
    const uint32_t tid = threadIdx.x;
    GAS uint64_t* v = gp(A.sizes);
    GAS uint64_t* sums = gp(A.scratch);
    const uint64_t nq = A.nq, ngroups = (nq + kScanGroup - 1) / kScanGroup;
    if (pass == 2) {
        uint64_t carry = 0;
        for (uint64_t g0 = 0; g0 < ngroups; g0 += kScanThreads) {
            const uint64_t g = g0 + tid;
            const uint64_t x = g < ngroups ? sums[g] : 0;
            uint64_t tot;
            const uint64_t ex = block_excl1024(x, s_t, &tot);
            if (g < ngroups) sums[g] = carry + ex;
            carry += tot;
        }
        if (tid == 0) {
            v[nq] = min(carry, A.out_cap);
            if (A.needed) gp(A.needed)[0] = carry;
        }
        return;
    }
    const uint64_t g = blockIdx.x, lo = g * kScanGroup, hi = min(nq, lo + kScanGroup);
    uint64_t x[kScanPer], s = 0;
#pragma unroll
    for (uint32_t q = 0; q < kScanPer; q++) {
        const uint64_t j = lo + tid * kScanPer + q;
        x[q] = j < hi ? v[j] : 0;
        s += x[q];
    }
    uint64_t tot;
    const uint64_t ex = block_excl1024(s, s_t, &tot);
    if (pass == 0) {
        if (tid == 0) sums[g] = tot;
        return;
    }
    const bool single = ngroups == 1;
    uint64_t run = (single ? 0 : sums[g]) + ex;
#pragma unroll
    for (uint32_t q = 0; q < kScanPer; q++) {
        const uint64_t j = lo + tid * kScanPer + q;
        if (j < hi) v[j] = min(run, A.out_cap);
        run += x[q];
    }
    if (single && tid == kScanThreads - 1) {
        v[nq] = min(run, A.out_cap);
        if (A.needed) gp(A.needed)[0] = run;
    }
}

// nq <= kScanThreads: probe, sizes and their scan in one workgroup (one
// launch instead of two for a small read).
__global__ void __launch_bounds__(kScanThreads) gather_probe_scan(IndexArgs A) {
    __shared__ uint64_t s_t[kScanThreads / 64];
    const uint32_t tid = threadIdx.x;
    uint32_t row = kMissing;
    uint64_t sz = 0;
    if (tid < live_queries(A)) row = probe_one<true>(A, tid, &sz);
    uint64_t tot;
    const uint64_t ex = block_excl1024(sz, s_t, &tot);
    if (tid < A.nq) {
        gp(A.rows)[tid] = row;
        gp(A.sizes)[tid] = min(ex, A.out_cap);
    }
    if (tid == 0) {
        gp(A.sizes)[A.nq] = min(tot, A.out_cap);
        if (A.needed) gp(A.needed)[0] = tot;
    }
}

// Eight lanes per query row, eight rows per wave: copy the row's blob bytes
// to the block (rows clamped by the scan copy only what fits).  A lane owns
// 16-B destination blocks b = lane%8, +8, ... aligned to the block buffer; it
// loads the five aligned source dwords that cover the block (only the words
// that overlap the row, so nothing outside the blob is read) and realigns them
// with v_alignbyte.  Interior blocks are one 16-B store, the row's first and
// last blocks byte stores.  One row per wave (the first version) spent most of
// its time creating waves: ~100-B rows gave a wave one load and one store.
// Lane j of kCopyLanes copies the row at blob[s0 ..) to out[d0, d1).
template <uint32_t kCopyLanes>
__device__ __forceinline__ void copy_row(const GAS uint8_t* blob, uint64_t s0, GAS uint8_t* out, uint64_t d0,
                                         uint64_t d1, uint32_t j) {
    const uint64_t first = d0 & ~(uint64_t)15;
    for (uint64_t D = first + 16 * (uint64_t)j; D < d1; D += 16 * kCopyLanes) {
        const uint64_t lo = D > d0 ? D : d0, hi = D + 16 < d1 ? D + 16 : d1;
        // source bytes of [lo, hi): [s0 + lo - d0, s0 + hi - d0); of D: S (may precede the row)
        const uint64_t slo = s0 + (lo - d0), shi = s0 + (hi - d0);
        const uint64_t S = slo - (lo - D);  // = s0 - d0 + D, computed without underflow past lo
        const uint32_t sh = (uint32_t)(S & 3);
        const uint64_t wb = S & ~(uint64_t)3;
        uint32_t w[5];
#pragma unroll
        for (int t = 0; t < 5; t++) {
            const uint64_t a = wb + 4 * t;
            w[t] = (a < shi && a + 4 > slo) ? *(const GAS uint32_t*)(blob + a) : 0u;
        }
        uint32_t q[4];
#pragma unroll
        for (int t = 0; t < 4; t++) q[t] = __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
        if (lo == D && hi == D + 16) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4 v = {q[0], q[1], q[2], q[3]};
            *(GAS u32x4*)(out + D) = v;
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint64_t b = D + k;
                if (b >= lo && b < hi) out[b] = (uint8_t)(q[k >> 2] >> (8 * (k & 3)));
            }
        }
    }
}

template <uint32_t kCopyLanes>
__global__ void __launch_bounds__(256) gather_copy(IndexArgs A) {
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kCopyLanes;
    const uint32_t j = threadIdx.x % kCopyLanes;
    if (i >= A.nq) return;
    const uint32_t row = gp(A.rows)[i];
    if (row == kMissing) return;
    const uint64_t d0 = gp(A.sizes)[i], d1 = gp(A.sizes)[i + 1];
    if (d1 <= d0) return;
    copy_row<kCopyLanes>(gp(A.blob), gp(A.row_off)[row], gp(A.out), d0, d1, j);
}

// A small gather in one launch (nq <= 1024, A.lb set; launch_gather): one
// workgroup per 64 queries.  Its first wave probes them (rows, sizes and
// source offsets into LDS) and scans the sizes; lane 0 publishes the group's
// byte total in its look-back word (bit 63 set), and the group's base is the
// sum of the words of the groups before it -- workgroups of lower index are
// dispatched first and never wait on a later one, so the spin always ends
// (bounded anyway).  Then all 512 threads copy the group's rows, 8 lanes a
// row, in one pass.  The words come in two sets used by alternate launches
// (the host flips A.lb); a launch's workgroup 0 zeroes the other set for the
// next one, so no launch waits on a ticket at its end.
// With A.ulen (a resident table's per-row utf8 string bytes), the same probe
// loads each row's string bytes beside its offsets, the look-back carries
// their group totals too, and the gather writes the gathered block's utf8
// index at stride 64 (A.uidx): the decode then cuts the block into one-pass
// virtual blocks instead of split mode's two passes and look-back.
constexpr unsigned long long kLbSet = 1ull << 63;
// Phase clocks of tuning builds (100 MHz s_memrealtime, workgroup's thread 0,
// after a wait for every memory operation in flight; murr_abi.cpp prints them
// with MURR_GATHER_STAMPS=1).
#ifdef MURR_TUNING
#define GF_STAMP(k)                                                                                 \
    if (A.stamps) {                                                                                 \
        __builtin_amdgcn_s_waitcnt(0); /* (the phase's loads land before its clock) */              \
        if (tid == 0) gp(A.stamps)[(uint64_t)g * kGatherStamps + (k)] = __builtin_amdgcn_s_memrealtime(); \
    }
#else
#define GF_STAMP(k)
#endif
constexpr uint32_t kLbW = 1 + kGatherMaxU;  // words per group: bytes, then each utf8 column's string bytes
__global__ void __launch_bounds__(512) gather_fused(IndexArgs A, unsigned long long* other) {
    __shared__ uint64_t s_off[65], s_src[64];
    __shared__ uint32_t s_row[64];
    const uint32_t tid = threadIdx.x, g = blockIdx.x;
    const uint64_t nq = A.nq, i0 = (uint64_t)g * 64;
    const uint32_t nu = A.ulen ? A.nu : 0u;
    GAS unsigned long long* lb = (GAS unsigned long long*)A.lb;
    GF_STAMP(0);
    if (g == 0 && tid >= 64 && tid < 64 + kGatherWords) gp(other)[tid - 64] = 0ull;
    if (tid < 64) {
        const uint64_t i = i0 + tid;
        uint64_t sz = 0, src = 0;
        uint32_t ul[kGatherMaxU] = {0, 0, 0, 0};
        uint32_t row = kMissing;
        if (i < live_queries(A)) row = probe_one<true>(A, i, &sz, &src, nu ? ul : nullptr);
        GF_STAMP(1);
        uint64_t x[kLbW], inc[kLbW];
        x[0] = sz;
#pragma unroll
        for (uint32_t u = 0; u < kGatherMaxU; u++) x[1 + u] = ul[u];
#pragma unroll
        for (uint32_t k = 0; k < kLbW; k++) {
            inc[k] = 0;
            if (k <= nu) {
                inc[k] = wave_incl_scan64(x[k], tid);
                const uint64_t tot = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(inc[k] >> 32), 63) << 32) |
                                     __builtin_amdgcn_readlane((uint32_t)inc[k], 63);
                if (tid == 0) __hip_atomic_store(lb + g * kLbW + k, kLbSet | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        // the groups before this one: lane j < g spins on group j's words,
        // all of them loaded together each time round
        uint64_t v[kLbW], base[kLbW];
#pragma unroll
        for (uint32_t k = 0; k < kLbW; k++) v[k] = kLbSet;
        if (tid < g) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                bool all = true;
#pragma unroll
                for (uint32_t k = 0; k < kLbW; k++)
                    if (k <= nu) v[k] = __hip_atomic_load(lb + tid * kLbW + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (uint32_t k = 0; k < kLbW; k++) all &= !(k <= nu) || (v[k] & kLbSet) != 0;
                if (all) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {  // 50 ms: cannot happen
                    if (A.err) __hip_atomic_fetch_max(gp(A.err), ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        GF_STAMP(2);
#pragma unroll
        for (uint32_t k = 0; k < kLbW; k++) base[k] = k <= nu ? wave_sum64(tid < g ? v[k] & ~kLbSet : 0ull) : 0;
        s_off[tid] = base[0] + inc[0] - sz;
        s_src[tid] = src;
        s_row[tid] = row;
        if (i < nq) {
            gp(A.rows)[i] = row;
            gp(A.sizes)[i] = min(base[0] + inc[0] - sz, A.out_cap);
        }
        const bool last = i0 + 64 >= nq;
        if (tid == 0) {  // utf8 index entry g: the string bytes of the rows before row 64 g
#pragma unroll
            for (uint32_t u = 0; u < kGatherMaxU; u++)
                if (u < nu) gp(A.uidx)[(uint64_t)g * nu + u] = base[1 + u];
        }
        if (tid == 63) {
            s_off[64] = base[0] + inc[0];
            if (last) {  // the block's end, the exact size and the index's last entry
                gp(A.sizes)[nq] = min(base[0] + inc[0], A.out_cap);
                if (A.needed) gp(A.needed)[0] = base[0] + inc[0];
#pragma unroll
                for (uint32_t u = 0; u < kGatherMaxU; u++)
                    if (u < nu) gp(A.uidx)[(uint64_t)(g + 1) * nu + u] = base[1 + u] + inc[1 + u];
            }
        }
    }
    __syncthreads();
    GF_STAMP(3);
    const uint32_t r = tid / 8;
    if (i0 + r < nq && s_row[r] != kMissing) {
        const uint64_t d0 = min(s_off[r], A.out_cap), d1 = min(s_off[r + 1], A.out_cap);
        if (d1 > d0) copy_row<8>(gp(A.blob), s_src[r], gp(A.out), d0, d1, tid % 8);
    }
#ifdef MURR_TUNING
    if (A.stamps) {
        __syncthreads();
        GF_STAMP(4);
    }
#endif
}

// ---- one read over a table sharded across GPUs (murr_multi_gather) ----------------
// The caller's queries are grouped by owner shard (shard s holds grouped
// positions [q_end[s - 1], q_end[s])); src[i] = grouped position of caller
// query i; rows[p] = the row shard s's lookup found for grouped position p.
// Each query's row is read straight from its shard's arena (peer memory over
// xGMI when the shard lives on another GPU).
__device__ __forceinline__ uint32_t multi_shard(const MultiTab& T, uint64_t p) {
    uint32_t s = 0;
    while (s + 1 < T.n && p >= T.q_end[s]) s++;
    return s;
}

__global__ void __launch_bounds__(256) multi_sizes(IndexArgs A, MultiTab T) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.nq) return;
    const uint64_t p = gp(A.src)[i];
    const uint32_t row = gp(A.rows)[p];
    const uint32_t s = multi_shard(T, p);
    gp(A.sizes)[i] = row == kMissing ? 0 : gp(T.row_off[s])[row + 1] - gp(T.row_off[s])[row];
}

template <uint32_t kCopyLanes>
__global__ void __launch_bounds__(256) multi_copy(IndexArgs A, MultiTab T) {
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kCopyLanes;
    const uint32_t j = threadIdx.x % kCopyLanes;
    if (i >= A.nq) return;
    const uint64_t p = gp(A.src)[i];
    const uint32_t row = gp(A.rows)[p];
    if (row == kMissing) return;
    const uint64_t d0 = gp(A.sizes)[i], d1 = gp(A.sizes)[i + 1];
    if (d1 <= d0) return;
    const uint32_t s = multi_shard(T, p);
    copy_row<kCopyLanes>(gp(T.arena[s]), gp(T.row_off[s])[row], gp(A.out), d0, d1, j);
}

}  // namespace

hipError_t launch_index_insert(const IndexArgs& a, hipStream_t s) {
    if (!a.n) return hipSuccess;
    hipLaunchKernelGGL(index_insert, dim3((uint32_t)((a.n + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_index_cache_rows(const IndexArgs& a, const uint64_t* row_off, const uint32_t* ulen, uint64_t from,
                                   hipStream_t s) {
    if (a.n > from)
        hipLaunchKernelGGL(index_cache_rows, dim3((uint32_t)((a.n - from + 255) / 256)), dim3(256), 0, s, a, row_off,
                           ulen, from);
    return hipGetLastError();
}

hipError_t launch_index_probe(const IndexArgs& a, hipStream_t s) {
    if (!a.nq) return hipSuccess;
    hipLaunchKernelGGL(index_probe, dim3((uint32_t)((a.nq + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_index_seq(const IndexArgs& a, const uint64_t* seqs, unsigned long long* best,
                            unsigned long long* win, hipStream_t s) {
    if (!a.n) return hipSuccess;
    for (uint32_t ph = 0; ph < 3; ph++) {
        const uint64_t n = ph == 2 ? a.mask + 1 : a.n;
        hipLaunchKernelGGL(index_seq, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, a, seqs, best, win, ph);
    }
    return hipGetLastError();
}

uint64_t gather_scan_groups(uint64_t nq) { return (nq + kScanGroup - 1) / kScanGroup; }

hipError_t launch_gather_scan(const IndexArgs& a, hipStream_t s) {
    const uint64_t groups = gather_scan_groups(a.nq);
    if (a.nq <= kScanThreads) {
        hipLaunchKernelGGL(gather_probe_scan, dim3(1), dim3(kScanThreads), 0, s, a);
    } else {
        const hipError_t e = launch_index_probe(a, s);
        if (e != hipSuccess) return e;
        if (groups <= 1) {
            hipLaunchKernelGGL(gather_scan, dim3(1), dim3(kScanThreads), 0, s, a, 1u);
        } else {
            hipLaunchKernelGGL(gather_scan, dim3((uint32_t)groups), dim3(kScanThreads), 0, s, a, 0u);
            hipLaunchKernelGGL(gather_scan, dim3(1), dim3(kScanThreads), 0, s, a, 2u);
            hipLaunchKernelGGL(gather_scan, dim3((uint32_t)groups), dim3(kScanThreads), 0, s, a, 1u);
        }
    }
    return hipGetLastError();
}

hipError_t launch_gather_copy(const IndexArgs& a, hipStream_t s) {
    if (a.nq) {
        // eight lanes per row (measured best of 4 / 8 / 16 on config C rows)
        constexpr uint32_t rows_per_wg = 256 / 8;
        const dim3 grid((uint32_t)((a.nq + rows_per_wg - 1) / rows_per_wg));
        hipLaunchKernelGGL(gather_copy<8>, grid, dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

// Sizes of the caller-order block (each query's row in its shard) and their
// scan into A.sizes; then, when A.out is set, the rows copied.
hipError_t launch_multi_gather(const IndexArgs& a, const MultiTab& t, bool copy, hipStream_t s) {
    if (!a.nq) return hipSuccess;
    hipLaunchKernelGGL(multi_sizes, dim3((uint32_t)((a.nq + 255) / 256)), dim3(256), 0, s, a, t);
    const uint64_t groups = gather_scan_groups(a.nq);
    if (groups <= 1) {
        hipLaunchKernelGGL(gather_scan, dim3(1), dim3(kScanThreads), 0, s, a, 1u);
    } else {
        hipLaunchKernelGGL(gather_scan, dim3((uint32_t)groups), dim3(kScanThreads), 0, s, a, 0u);
        hipLaunchKernelGGL(gather_scan, dim3(1), dim3(kScanThreads), 0, s, a, 2u);
        hipLaunchKernelGGL(gather_scan, dim3((uint32_t)groups), dim3(kScanThreads), 0, s, a, 1u);
    }
    if (copy) {
        constexpr uint32_t rows_per_wg = 256 / 8;
        hipLaunchKernelGGL(multi_copy<8>, dim3((uint32_t)((a.nq + rows_per_wg - 1) / rows_per_wg)), dim3(256), 0, s,
                           a, t);
    }
    return hipGetLastError();
}

hipError_t launch_multi_copy(const IndexArgs& a, const MultiTab& t, hipStream_t s) {
    if (!a.nq) return hipSuccess;
    constexpr uint32_t rows_per_wg = 256 / 8;
    hipLaunchKernelGGL(multi_copy<8>, dim3((uint32_t)((a.nq + rows_per_wg - 1) / rows_per_wg)), dim3(256), 0, s, a, t);
    return hipGetLastError();
}

uint64_t gather_scratch_words(uint64_t nq) { return gather_scan_groups(nq) + 1; }

hipError_t launch_gather(const IndexArgs& a, hipStream_t s) {
    if (a.nq && a.nq <= 64 * kGatherGroups && a.lb) {  // (a.lb: this launch's word set; a.lb_other: the next's)
        hipLaunchKernelGGL(gather_fused, dim3((uint32_t)((a.nq + 63) / 64)), dim3(512), 0, s, a, a.lb_other);
        return hipGetLastError();
    }
    const hipError_t e = launch_gather_scan(a, s);
    if (e != hipSuccess) return e;
    return launch_gather_copy(a, s);
}

namespace {
__global__ void __launch_bounds__(256) offsets_rebase(int32_t* dst, const int32_t* src, uint64_t n, int64_t add) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) gp(dst)[i] = (int32_t)((int64_t)gp(src)[i] + add);
}
}  // namespace

// dst[i] = src[i] + add for i < n (an appended key column's offsets into the
// index's key copy).
hipError_t launch_offsets_rebase(int32_t* dst, const int32_t* src, uint64_t n, int64_t add, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(offsets_rebase, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, dst, src, n, add);
    return hipGetLastError();
}

// ---- utf8 index of a block (murr_utf8_index) -------------------------------------
// For every utf8 column u of the layout, the string bytes of the rows before
// row j * stride: what the decode's utf8 offsets reach at that row
// (Utf8Encoder::add_row, src/io/codec/utf8.rs:86-96), by the decode's own
// cell rules (read.rs:45-55 bounds; a null, missing, short or malformed cell
// adds nothing).  With it, a block can be decoded by many workgroups at once,
// each from a known starting offset.
namespace {
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// One workgroup per stride window: window k (from floor(from / stride)) is
// the rows [max(k * stride, from), min((k + 1) * stride, n)); its string bytes
// per column go to part[k - k0].
__global__ void __launch_bounds__(256) uidx_sums(Utf8IndexArgs A) {
    __shared__ uint64_t part[4];
    const uint64_t k = A.from / A.stride + blockIdx.x;
    const uint64_t w0 = k * A.stride, r0 = w0 > A.from ? w0 : A.from;
    const uint64_t r1 = w0 + A.stride < A.n ? w0 + A.stride : A.n;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t u = 0; u < A.nu; u++) {
        const uint32_t c = A.col[u], fo = A.fo[u];
        uint64_t sum = 0;
        for (uint64_t i = r0 + threadIdx.x; i < r1; i += 256) {
            const uint64_t a = A.row_off32 ? (uint64_t)gp(A.row_off32)[i] : gp(A.row_off)[i];
            const uint64_t e = A.row_off32 ? (uint64_t)gp(A.row_off32)[i + 1] : gp(A.row_off)[i + 1];
            if (e < a || e - a > 0xFFFFFFFFull) continue;  // the decode reports such a row
            const uint32_t rl = (uint32_t)(e - a);
            const uint8_t* row = A.data + a;
            if (rl < A.bs || ((row[c >> 3] >> (c & 7)) & 1)) continue;  // short row / null cell
            if (fo + 4 > rl) continue;
            const uint32_t sl = ld32u(row + fo), vlen = rl - A.bs;
            if (sl > vlen - 4) continue;
            const uint32_t l = ld32u(row + A.bs + sl);
            if (l > vlen - 4 - sl) continue;
            sum += l;
        }
        for (int m = 32; m >= 1; m >>= 1) sum += (uint64_t)__shfl_xor((unsigned long long)sum, m, 64);
        if (lane == 0) part[wave] = sum;
        __syncthreads();
        if (threadIdx.x == 0) gp(A.part)[(uint64_t)blockIdx.x * A.nu + u] = part[0] + part[1] + part[2] + part[3];
        __syncthreads();
    }
}

// Per row: out[i * nu + u] = the string bytes row i's u-th utf8 column adds
// to the decode's offsets, by the same cell rules (rows [from, n)).  A
// resident table keeps these beside its arena for the fused gather.
__global__ void __launch_bounds__(256) utf8_row_lengths(Utf8IndexArgs A, uint32_t* out) {
    const uint64_t i = A.from + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n) return;
    const uint64_t a = A.row_off32 ? (uint64_t)gp(A.row_off32)[i] : gp(A.row_off)[i];
    const uint64_t e = A.row_off32 ? (uint64_t)gp(A.row_off32)[i + 1] : gp(A.row_off)[i + 1];
    const bool span_ok = !(e < a || e - a > 0xFFFFFFFFull);
    const uint32_t rl = span_ok ? (uint32_t)(e - a) : 0u;
    const uint8_t* row = A.data + a;
    for (uint32_t u = 0; u < A.nu; u++) {
        const uint32_t c = A.col[u], fo = A.fo[u];
        uint32_t l = 0;
        if (span_ok && rl >= A.bs && !((row[c >> 3] >> (c & 7)) & 1) && fo + 4 <= rl) {
            const uint32_t sl = ld32u(row + fo), vlen = rl - A.bs;
            if (sl <= vlen - 4) {
                const uint32_t len = ld32u(row + A.bs + sl);
                if (len <= vlen - 4 - sl) l = len;
            }
        }
        gp(out)[i * A.nu + u] = l;
    }
}

// One workgroup: entries k0 + 1 .. k0 + nwin = the total before `from` (the
// index's old total, entry ceil(from / stride), read before any entry is
// written) plus the inclusive prefix of the window sums; entry 0 = 0 for a
// fresh index.  The last of them is the new total.
__global__ void __launch_bounds__(1024) uidx_scan(uint64_t* out, const uint64_t* part, uint64_t nwin, uint32_t nu,
                                                  uint64_t k0, uint64_t from, uint64_t stride) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t base_s;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t u = 0; u < nu; u++) {
        if (threadIdx.x == 0) base_s = from ? gp(out)[((from + stride - 1) / stride) * nu + u] : 0;
        __syncthreads();
        uint64_t carry = base_s;
        if (from == 0 && threadIdx.x == 0) gp(out)[u] = 0;
        for (uint64_t base = 0; base < nwin; base += 1024) {
            const uint64_t j = base + threadIdx.x;
            const uint64_t v = j < nwin ? gp(part)[j * nu + u] : 0;
            uint64_t inc = v;
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t o = (uint64_t)__shfl_up((unsigned long long)inc, d, 64);
                if (lane >= (uint32_t)d) inc += o;
            }
            if (lane == 63) wsum[wave] = inc;
            __syncthreads();
            uint64_t before = 0, total = 0;
            for (uint32_t w = 0; w < 16; w++) {
                before += w < wave ? wsum[w] : 0;
                total += wsum[w];
            }
            if (j < nwin) gp(out)[(k0 + 1 + j) * nu + u] = carry + before + inc;
            carry += total;
            __syncthreads();
        }
        __syncthreads();  // every thread has its base before thread 0 reads the next column's
    }
}
}  // namespace

uint64_t utf8_index_windows(uint64_t from, uint64_t n, uint64_t stride) {
    return n > from ? (n + stride - 1) / stride - from / stride : 0;
}

hipError_t launch_utf8_row_lengths(const Utf8IndexArgs& a, uint32_t* out, hipStream_t s) {
    if (a.n > a.from)
        hipLaunchKernelGGL(utf8_row_lengths, dim3((uint32_t)((a.n - a.from + 255) / 256)), dim3(256), 0, s, a, out);
    return hipGetLastError();
}

hipError_t launch_utf8_index(const Utf8IndexArgs& a, hipStream_t s) {
    const uint64_t nwin = utf8_index_windows(a.from, a.n, a.stride);
    if (nwin) hipLaunchKernelGGL(uidx_sums, dim3((uint32_t)nwin), dim3(256), 0, s, a);
    if (nwin || a.from == 0)
        hipLaunchKernelGGL(uidx_scan, dim3(1), dim3(1024), 0, s, a.out, (const uint64_t*)a.part, nwin, a.nu,
                           a.from / a.stride, a.from, a.stride);
    return hipGetLastError();
}

}  // namespace murr
