// Micro-benchmark: read bandwidth of "stage a contiguous tile into LDS" loops
// (the decode kernel's input pattern) under different structures.
//   mode 0: glds (LDS-DMA) single buffer, synchronous (issue, wait, barrier, touch)
//   mode 1: glds double buffer (issue next before touching current)
//   mode 2: register staging (dwordx4 to VGPRs, then ds_write_b128), single buffer
//   mode 3: plain streaming read to registers, no LDS (reference ceiling)
// Tiles are TILE bytes; grid = wgs_per_cu * 256 persistent workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define GAS __attribute__((address_space(1)))
#define LAS __attribute__((address_space(3)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(256) stage(const uint8_t* __restrict__ src, uint64_t ntiles, uint32_t tile,
                                             unsigned long long* sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const GAS uint8_t* g0 = (const GAS uint8_t*)src;
    uint32_t acc = 0;
    const uint64_t G = gridDim.x;
    if (MODE == 0 || MODE == 1) {
        uint32_t i = 0;
        uint64_t t = blockIdx.x;
        if (MODE == 1 && t < ntiles) {
            for (uint32_t c = wave; c * 1024 < tile; c += 4)
                __builtin_amdgcn_global_load_lds((const GAS void*)(g0 + t * tile + c * 1024 + lane * 16),
                                                 (LAS void*)(lds + c * 1024), 16, 0, 0);
        }
        for (; t < ntiles; t += G, i++) {
            uint8_t* buf = lds + (MODE == 1 ? (i & 1) * tile : 0);
            if (MODE == 0) {
                for (uint32_t c = wave; c * 1024 < tile; c += 4)
                    __builtin_amdgcn_global_load_lds((const GAS void*)(g0 + t * tile + c * 1024 + lane * 16),
                                                     (LAS void*)(buf + c * 1024), 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (MODE == 1 && t + G < ntiles) {
                uint8_t* nb = lds + ((i + 1) & 1) * tile;
                for (uint32_t c = wave; c * 1024 < tile; c += 4)
                    __builtin_amdgcn_global_load_lds((const GAS void*)(g0 + (t + G) * tile + c * 1024 + lane * 16),
                                                     (LAS void*)(nb + c * 1024), 16, 0, 0);
            }
            for (uint32_t k = tid; k < tile / 4; k += 256) acc += reinterpret_cast<const uint32_t*>(buf)[k];
            __syncthreads();
        }
    } else if (MODE == 2) {
        for (uint64_t t = blockIdx.x; t < ntiles; t += G) {
            u32x4 r[8];
            const uint32_t n16 = tile / 16;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t c = j * 256 + tid;
                if (c < n16) r[j] = *(const GAS u32x4*)(g0 + t * tile + c * 16);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t c = j * 256 + tid;
                if (c < n16) reinterpret_cast<u32x4*>(lds)[c] = r[j];
            }
            __syncthreads();
            for (uint32_t k = tid; k < tile / 4; k += 256) acc += reinterpret_cast<const uint32_t*>(lds)[k];
            __syncthreads();
        }
    } else {
        for (uint64_t t = blockIdx.x; t < ntiles; t += G) {
            u32x4 r[8];
            const uint32_t n16 = tile / 16;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t c = j * 256 + tid;
                if (c < n16) r[j] = *(const GAS u32x4*)(g0 + t * tile + c * 16);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t c = j * 256 + tid;
                if (c < n16) acc += r[j].x ^ r[j].y ^ r[j].z ^ r[j].w;
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keep the loads alive
}

template <int MODE>
float run(const uint8_t* d, uint64_t bytes, uint32_t tile, int wgs_per_cu, unsigned long long* sink) {
    const uint64_t ntiles = bytes / tile;
    const uint32_t lds = MODE == 1 ? 2 * tile : (MODE == 3 ? 0 : tile);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = 256 * wgs_per_cu;
    hipLaunchKernelGGL(stage<MODE>, dim3(grid), dim3(256), lds, 0, d, ntiles, tile, sink);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(stage<MODE>, dim3(grid), dim3(256), lds, 0, d, ntiles, tile, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return (float)(bytes * reps / (ms * 1e-3) / 1e12);
}

int main() {
    const uint64_t bytes = 2ull << 30;
    uint8_t* d;
    unsigned long long* sink;
    if (hipMalloc(&d, bytes + 65536) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    hipMemset(d, 1, bytes);
    for (uint32_t tile : {4096u, 8192u, 16384u, 32768u}) {
        for (int w : {1, 2, 3, 4, 6, 8}) {
            const uint32_t lds1 = tile, lds2 = 2 * tile;
            printf("tile %6u wg/cu %d | glds1 %s%.2f | glds2 %s%.2f | reg %s%.2f | noLDS %.2f TB/s\n", tile, w,
                   (uint64_t)w * lds1 > 160 * 1024 ? "*" : " ", run<0>(d, bytes, tile, w, sink),
                   (uint64_t)w * lds2 > 160 * 1024 ? "*" : " ", run<1>(d, bytes, tile, w, sink),
                   (uint64_t)w * lds1 > 160 * 1024 ? "*" : " ", tile <= 32768 ? run<2>(d, bytes, tile, w, sink) : 0.f,
                   run<3>(d, bytes, tile, w, sink));
        }
    }
    return 0;
}
