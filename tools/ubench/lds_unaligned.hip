// Unaligned LDS access on gfx950: correctness of ds_read_b32/b64/b128 at any
// byte address, and cost vs aligned reads (ns per wave-instruction, whole chip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4u;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void check(const uint8_t* in, uint32_t* out) {
  __shared__ uint8_t s[8192];
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) ((uint32_t*)s)[i] = ((const uint32_t*)in)[i];
  __syncthreads();
  uint32_t a = threadIdx.x * 7 + blockIdx.x;  // every alignment
  uint32_t* o = out + (blockIdx.x * 256 + threadIdx.x) * 8;
  o[0] = *(const u32u*)(s + a);
  uint64_t v = *(const u64u*)(s + a + 1);
  o[1] = (uint32_t)v;
  o[2] = (uint32_t)(v >> 32);
  u32x4 w = *(const u32x4u*)(s + a + 2);
  o[3] = w.x; o[4] = w.y; o[5] = w.z; o[6] = w.w;
}

// MODE 0: ds_read_b32 at 4-aligned addresses; 1: ds_read_b32 at stride-5
// unaligned addresses; 2: ds_read_u8; 3: ds_read_b64 unaligned; 4: aligned
// ds_read2_b32 + v_alignbyte (the old way to read an unaligned dword)
template <int MODE>
__global__ void __launch_bounds__(256) bw(uint32_t* out, int iters) {
  __shared__ uint8_t s[16384 + 64];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) ((uint32_t*)s)[i] = i * 2654435761u;
  __syncthreads();
  uint32_t a = MODE == 0 ? threadIdx.x * 4 : threadIdx.x * 5 + 1, acc = 0;
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t x = (a + j * 1100) & 8191;
      if (MODE == 0) acc += *(const uint32_t*)(s + (x & ~3u));
      else if (MODE == 1) acc += *(const u32u*)(s + x);
      else if (MODE == 2) acc += s[x];
      else if (MODE == 3) { uint64_t v = *(const u64u*)(s + x); acc += (uint32_t)v ^ (uint32_t)(v >> 32); }
      else {
        const uint32_t* w = (const uint32_t*)(s + (x & ~3u));
        acc += __builtin_amdgcn_alignbyte(w[1], w[0], x & 3);
      }
    }
    a += 4 + (acc & 1);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// unaligned dword stores, lane-contiguous at a 5-byte stride (strings)
__global__ void __launch_bounds__(256) st(uint8_t* out, int iters, int stride) {
  for (int it = 0; it < iters; it++) {
    uint64_t base = ((uint64_t)blockIdx.x * iters + it) * 256 * stride;
    *(u32u*)(out + base + threadIdx.x * stride) = threadIdx.x * 0x01010101u;
  }
}

int main() {
  uint8_t* h = (uint8_t*)malloc(8192);
  for (int i = 0; i < 8192; i++) h[i] = (uint8_t)(i * 131 + 7);
  uint8_t* d; uint32_t* o;
  CK(hipMalloc(&d, 8192)); CK(hipMalloc(&o, 4096 * 256 * 8 * 4));
  CK(hipMemcpy(d, h, 8192, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(check, dim3(64), dim3(256), 0, 0, d, o);
  CK(hipGetLastError());
  uint32_t* ho = (uint32_t*)malloc(64 * 256 * 8 * 4);
  CK(hipMemcpy(ho, o, 64 * 256 * 8 * 4, hipMemcpyDeviceToHost));
  long bad = 0;
  for (int b = 0; b < 64; b++) for (int t = 0; t < 256; t++) {
    uint32_t a = t * 7 + b; const uint32_t* r = ho + (b * 256 + t) * 8;
    uint32_t e0, e1, e2, e3[4];
    memcpy(&e0, h + a, 4); memcpy(&e1, h + a + 1, 4); memcpy(&e2, h + a + 5, 4); memcpy(e3, h + a + 2, 16);
    if (r[0] != e0 || r[1] != e1 || r[2] != e2 || r[3] != e3[0] || r[4] != e3[1] || r[5] != e3[2] || r[6] != e3[3]) bad++;
  }
  printf("unaligned LDS read mismatches: %ld of %d\n", bad, 64 * 256);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int grid = 4096, iters = 2000;
  const char* names[] = {"ds_read_b32 aligned", "ds_read_b32 unaligned", "ds_read_u8", "ds_read_b64 unaligned",
                         "read2 + alignbyte"};
#define RUN(M) { hipLaunchKernelGGL((bw<M>), dim3(grid), dim3(256), 0, 0, o, 10); CK(hipDeviceSynchronize()); \
    CK(hipEventRecord(e0)); hipLaunchKernelGGL((bw<M>), dim3(grid), dim3(256), 0, 0, o, iters); CK(hipEventRecord(e1)); \
    CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); \
    double wi = (double)grid * 4 * iters * 8; \
    printf("%-24s %.3f ms  %.1f wave-instr/ns chip  %.2f cyc/instr/CU@2.4GHz\n", names[M], ms, wi / (ms * 1e6), \
           (ms * 1e-3 * 2.4e9 * 256) / wi); }
  RUN(0) RUN(1) RUN(2) RUN(3) RUN(4)
  uint8_t* big; CK(hipMalloc(&big, (size_t)2048 * 400 * 256 * 8 + 64));
  for (int stride : {4, 5, 8}) {
    hipLaunchKernelGGL(st, dim3(2048), dim3(256), 0, 0, big, 400, stride); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); hipLaunchKernelGGL(st, dim3(2048), dim3(256), 0, 0, big, 400, stride); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double bytes = 2048.0 * 400 * 256 * 4;
    printf("global_store_dword stride %d: %.3f ms  %.0f GB/s (4 B per lane)\n", stride, ms, bytes / (ms * 1e6));
  }
  return bad != 0;
}
