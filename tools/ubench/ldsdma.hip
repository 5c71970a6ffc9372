// Probe: what one 1 KiB wave-instruction of loads costs the CU's memory
// pipeline (TA/TD) by form -- LDS-DMA (global_load_lds_dwordx4, the decode
// loader's form), a dwordx4 load into VGPRs followed by ds_write_b128 (register
// staging), and a dwordx4 load into VGPRs alone -- from an L2-resident window
// (pipeline cost) and streamed from HBM (bandwidth), with W waves per CU each
// keeping K instructions in flight.  Round 6: DESIGN.md §7 priced an LDS-DMA
// load at ~110 cycles per KiB without a measurement behind it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 ldsdma.hip -o ldsdma
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
#define LAS __attribute__((address_space(3)))
#define GAS __attribute__((address_space(1)))
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void glds16(const GAS void* src, LAS void* dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst))
                 : "memory");
}

// FORM 0: LDS-DMA; 1: VGPR load + ds_write_b128; 2: VGPR load only.
// K instructions issued per group, then waited for.  `span`: bytes the
// workgroup's waves sweep (L2 window), or the whole buffer (stream).
template <int FORM, int K>
__global__ void __launch_bounds__(256) ld(const uint8_t* __restrict__ buf, uint64_t span, uint32_t iters,
                                          uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * K * 1024];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t nw = (uint64_t)gridDim.x * 4, w = (uint64_t)blockIdx.x * 4 + wave;
    uint32_t acc = 0;
    LAS uint8_t* mine = (LAS uint8_t*)lds + wave * K * 1024;
    for (uint32_t it = 0; it < iters; it++) {
        // piece index: waves interleaved so consecutive waves read consecutive KiB
        const uint64_t base = ((uint64_t)it * nw * K + w * K) * 1024 % span;
        if constexpr (FORM == 0) {
#pragma unroll
            for (int k = 0; k < K; k++)
                glds16((const GAS uint8_t*)buf + (base + k * 1024) % span + lane * 16, mine + k * 1024);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            u32x4 v[K];
#pragma unroll
            for (int k = 0; k < K; k++) v[k] = *(const GAS u32x4*)(buf + (base + k * 1024) % span + lane * 16);
#pragma unroll
            for (int k = 0; k < K; k++) {
                if constexpr (FORM == 1) *(LAS u32x4*)(mine + k * 1024 + lane * 16) = v[k];
                else acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
            }
            if constexpr (FORM == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (every iteration's writes kept)
        }
    }
    if constexpr (FORM != 2) {
        __syncthreads();
        acc = ((LAS uint32_t*)lds)[threadIdx.x];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int FORM, int K>
void run(const char* name, const uint8_t* buf, uint64_t span, int wgs_per_cu, uint32_t iters, uint32_t* out,
         bool stream) {
    const int cus = 256;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 g(cus * wgs_per_cu);
    ld<FORM, K><<<g, 256>>>(buf, span, iters, out);  // warm
    CK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; r++) ld<FORM, K><<<g, 256>>>(buf, span, iters, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double instr = (double)g.x * 4 * iters * K;  // wave-instructions of 1 KiB
    const double per_cu = instr / cus;
    std::printf("%-26s %s W/CU %2d K %d: %.4f ms  %6.1f cycles per KiB-instr per CU @2.4GHz  %7.0f GB/s\n", name,
                stream ? "stream" : "L2    ", 4 * wgs_per_cu, K, ms, ms * 1e-3 * 2.4e9 / per_cu, instr * 1024 / (ms * 1e-3) / 1e9);
    std::fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main() {
    const uint64_t big = 2ull << 30;  // streamed: 2 GiB
    uint8_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, big));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 1, big));
    const uint64_t l2 = 1u << 20;  // L2 window (each XCD's L2 holds it)
    for (int wpc : {1, 2, 4}) {
        run<0, 4>("lds-dma", buf, l2, wpc, 512, out, false);
        run<1, 4>("vgpr + ds_write_b128", buf, l2, wpc, 512, out, false);
        run<2, 4>("vgpr only", buf, l2, wpc, 512, out, false);
    }
    // streamed: every byte of 2 GiB once (iters sized to the buffer)
    for (int wpc : {1, 2, 4}) {
        const uint32_t iters = (uint32_t)(big / (256ull * wpc * 4 * 4 * 1024));
        run<0, 4>("lds-dma", buf, big, wpc, iters, out, true);
        run<1, 4>("vgpr + ds_write_b128", buf, big, wpc, iters, out, true);
        run<2, 4>("vgpr only", buf, big, wpc, iters, out, true);
    }
    return 0;
}
