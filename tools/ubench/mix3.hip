// Ceiling probe for the headline decode's HBM traffic, with ideal access (16-B
// per lane, fully coalesced, no LDS, no decode work):
//   copy    1:1 float4 copy (the guide's 6.29 TB/s reference point)
//   mix21   two read streams + one write stream of half their size
//   blocks  the decode's stream structure: K = 1000 blocks, each a blob
//           (17.89 B/row), row offsets (8 B/row) read and three outputs
//           (4 + 4 + 4.89 B/row) written, tile by tile (TR rows); workgroup g
//           owns whole blocks g, g + G, ... (local mode) or takes tiles of all
//           blocks round-robin (interleaved).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 mix3.hip -o mix3
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n) {
    const size_t nt = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += nt * U) {
        u32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++)
            if (i + k * nt < n) v[k] = NT ? __builtin_nontemporal_load(in + i + k * nt) : in[i + k * nt];
#pragma unroll
        for (int k = 0; k < U; k++)
            if (i + k * nt < n) out[i + k * nt] = v[k];
    }
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) mix21(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                             u32x4* __restrict__ out, size_t n) {
    const size_t nt = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += nt * U) {
        u32x4 v[U], w[U];
#pragma unroll
        for (int k = 0; k < U; k++)
            if (i + k * nt < n) {
                v[k] = NT ? __builtin_nontemporal_load(a + i + k * nt) : a[i + k * nt];
                w[k] = NT ? __builtin_nontemporal_load(b + i + k * nt) : b[i + k * nt];
            }
#pragma unroll
        for (int k = 0; k < U; k++)
            if (i + k * nt < n) out[i + k * nt] = v[k] ^ w[k];
    }
}

struct Blk {
    const uint8_t* blob;
    const uint8_t* ro;
    uint8_t* f;
    uint8_t* o;
    uint8_t* s;
};
constexpr uint32_t N = 100000;
constexpr double BLOB = 17.8889, STR = 4.8889;

// one tile [r0, r1) of block k: read blob + ro spans, write f/o/s spans
__device__ __forceinline__ void tile(const Blk& B, uint32_t r0, uint32_t r1, u32x4& acc) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint64_t b0 = (uint64_t)(r0 * BLOB) & ~15ull, b1 = (uint64_t)(r1 * BLOB) & ~15ull;
    const u32x4* bp = (const u32x4*)(B.blob + b0);
    for (uint64_t q = tid; q < (b1 - b0) / 16; q += nt) acc ^= bp[q];
    const u32x4* rp = (const u32x4*)(B.ro + 8ull * r0);
    for (uint64_t q = tid; q < (r1 - r0) / 2; q += nt) acc ^= rp[q];
    u32x4* fp = (u32x4*)(B.f + 4ull * r0);
    u32x4* op = (u32x4*)(B.o + 4ull * r0);
    for (uint64_t q = tid; q < (r1 - r0) / 4; q += nt) {
        fp[q] = acc;
        op[q] = acc;
    }
    const uint64_t s0 = (uint64_t)(r0 * STR) & ~15ull, s1 = (uint64_t)(r1 * STR) & ~15ull;
    u32x4* sp = (u32x4*)(B.s + s0);
    for (uint64_t q = tid; q < (s1 - s0) / 16; q += nt) sp[q] = acc;
}

// MODE 0: workgroup g owns blocks g, g + G, ...; MODE 1: tiles of every block
// round-robin over the grid (tile t of the whole launch -> workgroup t % G).
template <int MODE>
__global__ void __launch_bounds__(256) blocks(const Blk* __restrict__ bl, uint32_t K, uint32_t TR, u32x4* sink) {
    u32x4 acc = {0, 0, 0, 0};
    const uint32_t tpb = (N + TR - 1) / TR;
    if (MODE == 0) {
        for (uint32_t k = blockIdx.x; k < K; k += gridDim.x) {
            const Blk B = bl[k];
            for (uint32_t r = 0; r < N; r += TR) tile(B, r, r + TR < N ? r + TR : N, acc);
        }
    } else {
        for (uint64_t t = blockIdx.x; t < (uint64_t)K * tpb; t += gridDim.x) {
            const uint32_t k = (uint32_t)(t / tpb), r = (uint32_t)(t % tpb) * TR;
            tile(bl[k], r, r + TR < N ? r + TR : N, acc);
        }
    }
    if (acc.x == 0x12345678u) sink[threadIdx.x] = acc;
}

int main() {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto timeit = [&](auto launch) {
        float best = 1e9, sum = 0;
        for (int rep = 0; rep < 13; rep++) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 3) { best = ms < best ? ms : best; sum += ms; }
        }
        return sum / 10;
    };
    {  // copy and 2:1 mix over 1.29 GB units (the headline's write volume)
        const size_t n = 1288894000ull / 16;
        u32x4 *a, *b, *o;
        CK(hipMalloc(&a, 16 * n));
        CK(hipMalloc(&b, 16 * n));
        CK(hipMalloc(&o, 16 * n));
        CK(hipMemset(a, 1, 16 * n));
        CK(hipMemset(b, 2, 16 * n));
        for (uint32_t g : {2048u, 4096u, 8192u, 16384u}) {
            float ms = timeit([&] { copy<4, false><<<g, 256>>>(a, o, n); });
            std::printf("copy   U4    grid %5u: %.4f ms = %.0f GB/s (frac %.3f)\n", g, ms, 32.0 * n / ms / 1e6, 32.0 * n / ms / 8e9);
            ms = timeit([&] { copy<4, true><<<g, 256>>>(a, o, n); });
            std::printf("copy   U4 nt grid %5u: %.4f ms = %.0f GB/s (frac %.3f)\n", g, ms, 32.0 * n / ms / 1e6, 32.0 * n / ms / 8e9);
            ms = timeit([&] { mix21<2, false><<<g, 256>>>(a, b, o, n); });
            std::printf("mix21  U2    grid %5u: %.4f ms = %.0f GB/s (frac %.3f)\n", g, ms, 48.0 * n / ms / 1e6, 48.0 * n / ms / 8e9);
            ms = timeit([&] { mix21<2, true><<<g, 256>>>(a, b, o, n); });
            std::printf("mix21  U2 nt grid %5u: %.4f ms = %.0f GB/s (frac %.3f)\n", g, ms, 48.0 * n / ms / 1e6, 48.0 * n / ms / 8e9);
            ms = timeit([&] { mix21<4, false><<<g, 256>>>(a, b, o, n); });
            std::printf("mix21  U4    grid %5u: %.4f ms = %.0f GB/s (frac %.3f)\n", g, ms, 48.0 * n / ms / 1e6, 48.0 * n / ms / 8e9);
        }
        CK(hipFree(a));
        CK(hipFree(b));
        CK(hipFree(o));
    }
    {  // the decode's stream structure
        const uint32_t K = 1000;
        std::vector<Blk> hb(K);
        std::vector<void*> fr;
        auto al = [&](size_t n) { void* p; CK(hipMalloc(&p, n)); fr.push_back(p); CK(hipMemset(p, 3, n)); return (uint8_t*)p; };
        for (uint32_t k = 0; k < K; k++)
            hb[k] = Blk{al((size_t)(N * BLOB) + 64), al(8ull * N + 64), al(4ull * N + 64), al(4ull * N + 64), al((size_t)(N * STR) + 64)};
        Blk* db;
        CK(hipMalloc(&db, sizeof(Blk) * K));
        CK(hipMemcpy(db, hb.data(), sizeof(Blk) * K, hipMemcpyHostToDevice));
        u32x4* sink;
        CK(hipMalloc(&sink, 4096));
        const double by = K * (double)N * (BLOB + 8 + 4 + 4 + STR);
        for (uint32_t TR : {768u, 1536u, 4096u}) {
            for (uint32_t wpc : {2u, 4u, 8u}) {
                const uint32_t G = cus * wpc;
                float ms = timeit([&] { blocks<0><<<K < G ? K : G, 256>>>(db, K, TR, sink); });
                std::printf("blocks local       TR %4u wg/CU %u: %.4f ms = %.0f GB/s (frac %.3f)\n", TR, wpc, ms, by / ms / 1e6, by / ms / 8e9);
                ms = timeit([&] { blocks<1><<<G, 256>>>(db, K, TR, sink); });
                std::printf("blocks interleaved TR %4u wg/CU %u: %.4f ms = %.0f GB/s (frac %.3f)\n", TR, wpc, ms, by / ms / 1e6, by / ms / 8e9);
            }
        }
        for (void* p : fr) CK(hipFree(p));
    }
    return 0;
}
