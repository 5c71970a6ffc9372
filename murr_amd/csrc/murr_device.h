// murr_device.h — device helpers shared by the decode (murr_decode.hip) and
// encode (murr_kernels.hip) kernels: address-space views, wave64 scans on DPP,
// the cross-workgroup one-hop window prefix, and the UTF-8 DFA.
#pragma once
#include "murr_internal.h"

namespace murr {
namespace dev {

#define GAS __attribute__((address_space(1)))
#define LAS __attribute__((address_space(3)))
#define CAS __attribute__((address_space(4)))

// Global-address-space views of generic pointers: global_* instead of flat_*
// instructions (flat ones also tie up lgkmcnt and cost issue slots).
template <class T> __device__ __forceinline__ GAS T* gp(T* p) { return (GAS T*)p; }
template <class T> __device__ __forceinline__ const GAS T* gp(const T* p) { return (const GAS T*)p; }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Unaligned views for global memory: gfx9 serves unaligned global dword
// loads/stores at any byte address.  (Unaligned LDS reads are correct too but
// ~25x slower than aligned ones: tools/ubench/lds_unaligned.hip.)
typedef uint16_t __attribute__((aligned(1))) u16u;
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;

constexpr uint32_t kUtf8 = 0, kBool = 1;
constexpr uint32_t kSpinLimit = 1u << 22;
enum : uint32_t { kStUtf8 = 1, kStOverflow = 4, kStMalformed = 5, kStCapacity = 6, kStInternal = 10 };

__device__ __forceinline__ void report(unsigned long long* err, uint64_t key) {
    __hip_atomic_fetch_max(gp(err), (unsigned long long)~key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t sgpr(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t sgpr64(uint64_t v) {
    return ((uint64_t)sgpr((uint32_t)(v >> 32)) << 32) | sgpr((uint32_t)v);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int m) {
    uint32_t lo = __shfl_xor((uint32_t)x, m, 64), hi = __shfl_xor((uint32_t)(x >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t x, int d) {
    uint32_t lo = __shfl_up((uint32_t)x, d, 64), hi = __shfl_up((uint32_t)(x >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = shfl_up64(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
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

// threadIdx.x made opaque at each use: stops the compiler from hoisting the
// many lane masks derived from it out of a tile loop into SGPR pairs.
__device__ __forceinline__ uint32_t tidx() {
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops,
// not for its vector-memory ops, so LDS-DMA in flight survives it
// (__syncthreads() emits s_waitcnt vmcnt(0) and would drain it).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void publish(uint64_t* p, uint64_t v) {
    __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Cross-tile prefix by a one-hop window sum.  Tiles are dealt round-robin to
// a persistent grid of G workgroups, so tile t's workgroup processed tile t-G
// itself and kept its inclusive prefix (`base`).  What lies between is the
// aggregate of tiles (t-G, t): each tile publishes its aggregate (+1, so 0 =
// not yet) in one 8-byte agent-scope store as soon as it is known, and the
// whole workgroup sums the <= G-1 granules in parallel (agent-scope relaxed
// loads = sc1: bypass this CU's L1; MI355X_MICROARCH.md R2 hand-off form).
// Only tiles that are resident or done are ever waited on; spins are bounded.
template <int NW>  // waves in the workgroup
__device__ __forceinline__ uint64_t window_prefix(const uint64_t* st, uint64_t lo, uint64_t t, uint64_t base,
                                                  LAS uint64_t* s_w, unsigned long long* err, uint64_t ekey) {
    constexpr int K = 4;  // granules per thread per pass
    constexpr uint32_t NT = 64 * NW;
    const uint32_t tid = tidx(), lane = tid & 63, wave = tid >> 6;
    uint64_t sum = 0;
    for (uint64_t j0 = lo; j0 < t; j0 += NT * K) {
        uint64_t v[K];
#pragma unroll
        for (int i = 0; i < K; i++) {  // every load in flight before the first check
            const uint64_t j = j0 + i * NT + tid;
            v[i] = j < t ? __hip_atomic_load(gp(st) + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1;
        }
#pragma unroll
        for (int i = 0; i < K; i++) {
            const uint64_t j = j0 + i * NT + tid;
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
    sum = wave_sum64(sum);
    if (lane == 0) s_w[wave] = sum;
    lds_barrier();
    uint64_t tot = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) tot += s_w[w];
    lds_barrier();
    return base + tot;
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

}  // namespace dev
}  // namespace murr
