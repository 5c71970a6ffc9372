// Store-shape probe (round 4): what one wave store instruction costs the CU's
// memory pipeline (TA/TD/TCP) by shape -- the decode writes narrow columns
// (1-2 B per lane), unaligned string pieces and 4/8-B values, one row per lane.
// Every CU streams stores only (no loads); each variant reports ns per
// wave-instruction per CU and the bytes it moves.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 stshape.hip -o stshape
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint16_t __attribute__((aligned(1))) u16u;
typedef uint64_t __attribute__((aligned(1))) u64u;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// SHAPE: 0 byte, 1 short, 2 dword, 3 dword at base+1 (unaligned, contiguous),
// 4 "strings": lane i writes dwords at 5i and 5i+1 (two overlapping unaligned
// pieces per lane, 5-B pitch), 5 dwordx2, 6 dwordx4, 7 dword at 8-B pitch,
// 8 "strings" at 13-B pitch with 8-B pieces (u64 unaligned)
template <int SHAPE>
__global__ void __launch_bounds__(256) st(uint8_t* __restrict__ out, uint64_t iters, uint64_t span) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + wave, nw = (uint64_t)gridDim.x * 4;
    constexpr uint32_t pitch = SHAPE == 0 ? 64 : SHAPE == 1 ? 128 : SHAPE == 2 || SHAPE == 3 ? 256 : SHAPE == 4 ? 328
                             : SHAPE == 5 ? 512 : SHAPE == 6 ? 1024 : SHAPE == 7 ? 512 : 840;
    for (uint64_t k = 0; k < iters; k++) {
        const uint64_t base = ((w + k * nw) * pitch) % span;
        uint8_t* p = out + base;
        const uint32_t v = lane * 0x01010101u + (uint32_t)k;
        if constexpr (SHAPE == 0) p[lane] = (uint8_t)v;
        else if constexpr (SHAPE == 1) ((uint16_t*)p)[lane] = (uint16_t)v;
        else if constexpr (SHAPE == 2) ((uint32_t*)p)[lane] = v;
        else if constexpr (SHAPE == 3) *(u32u*)(p + 1 + 4 * lane) = v;
        else if constexpr (SHAPE == 4) {
            *(u32u*)(p + 5 * lane) = v;
            *(u32u*)(p + 5 * lane + 1) = v;
        } else if constexpr (SHAPE == 5) ((u32x2*)p)[lane] = u32x2{v, v};
        else if constexpr (SHAPE == 6) ((u32x4*)p)[lane] = u32x4{v, v, v, v};
        else if constexpr (SHAPE == 7) ((uint32_t*)p)[2 * lane] = v;
        else {
            *(u64u*)(p + 13 * lane) = ((uint64_t)v << 32) | v;
        }
    }
}

int main() {
    const uint64_t span = 1ull << 30;
    uint8_t* out;
    CK(hipMalloc(&out, span + 4096));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"byte", "short", "dword", "dword+1 unaligned", "2x dword overlapping @5B pitch", "dwordx2",
                           "dwordx4", "dword @8B pitch", "u64 unaligned @13B pitch"};
    const double bytes_per[] = {64, 128, 256, 256, 320, 512, 1024, 256, 512};
    const double insts_per[] = {1, 1, 1, 1, 2, 1, 1, 1, 1};
    for (int wpc : {4, 8}) {
        const uint32_t grid = cus * wpc;
        const uint64_t iters = 2048;
        for (int s = 0; s < 9; s++) {
            auto launch = [&] {
                switch (s) {
                    case 0: st<0><<<grid, 256>>>(out, iters, span); break;
                    case 1: st<1><<<grid, 256>>>(out, iters, span); break;
                    case 2: st<2><<<grid, 256>>>(out, iters, span); break;
                    case 3: st<3><<<grid, 256>>>(out, iters, span); break;
                    case 4: st<4><<<grid, 256>>>(out, iters, span); break;
                    case 5: st<5><<<grid, 256>>>(out, iters, span); break;
                    case 6: st<6><<<grid, 256>>>(out, iters, span); break;
                    case 7: st<7><<<grid, 256>>>(out, iters, span); break;
                    default: st<8><<<grid, 256>>>(out, iters, span); break;
                }
            };
            launch();
            CK(hipDeviceSynchronize());
            float best = 1e9;
            for (int r = 0; r < 5; r++) {
                CK(hipEventRecord(e0));
                launch();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            const double winst = (double)grid * 4 * iters * insts_per[s];  // wave store instructions
            const double ns_per = best * 1e6 / (winst / cus);
            std::printf("wg/CU %d %-32s %8.4f ms  %6.1f ns per wave-store per CU (%5.1f cyc @2.4GHz)  %7.0f GB/s\n", wpc,
                        names[s], best, ns_per, ns_per * 2.4, (double)grid * 4 * iters * bytes_per[s] / (best * 1e6));
            std::fflush(stdout);
        }
    }
    return 0;
}
