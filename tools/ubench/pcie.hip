// Host link probe (round 4): pinned hipMemcpyAsync rates H2D and D2H alone,
// and both directions at once on two streams, per transfer size -- the
// ceiling of the streaming host decode (murr_hstream).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 pcie.hip -o pcie
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

// a kernel that copies device memory into pinned host memory (or host to
// device) with 16-B coalesced accesses: zero-copy over PCIe, no DMA engine
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void kcopy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main() {
    const size_t maxb = 64ull << 20;
    void *h1, *h2, *d1, *d2;
    CK(hipHostMalloc(&h1, maxb, hipHostMallocDefault));
    CK(hipHostMalloc(&h2, maxb, hipHostMallocDefault));
    CK(hipMalloc(&d1, maxb));
    CK(hipMalloc(&d2, maxb));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    hipEvent_t e0, e1, f0, f1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    for (size_t sz : {64ull << 10, 256ull << 10, 1ull << 20, 2730ull << 10, 8ull << 20, 64ull << 20}) {
        const int reps = sz < (4u << 20) ? 200 : 20;
        auto run = [&](bool h2d, bool d2h) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, a));
            CK(hipEventRecord(f0, b));
            for (int r = 0; r < reps; r++) {
                if (h2d) CK(hipMemcpyAsync(d1, h1, sz, hipMemcpyHostToDevice, a));
                if (d2h) CK(hipMemcpyAsync(h2, d2, sz, hipMemcpyDeviceToHost, b));
            }
            CK(hipEventRecord(e1, a));
            CK(hipEventRecord(f1, b));
            CK(hipEventSynchronize(e1));
            CK(hipEventSynchronize(f1));
            float ta = 0, tb = 0;
            CK(hipEventElapsedTime(&ta, e0, e1));
            CK(hipEventElapsedTime(&tb, f0, f1));
            return std::make_pair(h2d ? ta : 0.f, d2h ? tb : 0.f);
        };
        run(true, true);  // warm
        const auto x = run(true, false), y = run(false, true), z = run(true, true);
        const double gb = (double)sz * reps / 1e9;
        std::printf("%8zu KiB: H2D alone %6.1f GB/s  D2H alone %6.1f GB/s  both: H2D %6.1f GB/s D2H %6.1f GB/s  (per copy %.1f / %.1f us)\n",
                    sz >> 10, gb / (x.first * 1e-3), gb / (y.second * 1e-3), gb / (z.first * 1e-3), gb / (z.second * 1e-3),
                    x.first * 1e3 / reps, y.second * 1e3 / reps);
        std::fflush(stdout);
    }
    // kernel copies over PCIe (device -> pinned host, pinned host -> device)
    for (size_t sz : {256ull << 10, 2730ull << 10, 8ull << 20, 64ull << 20}) {
        const size_t n = sz / 16;
        for (int dir = 0; dir < 2; dir++) {
            for (unsigned grid : {64u, 256u, 1024u}) {
                const u32x4* src = (const u32x4*)(dir ? h1 : d1);
                u32x4* dst = (u32x4*)(dir ? d2 : h2);
                kcopy<<<grid, 256, 0, a>>>(src, dst, n);
                CK(hipStreamSynchronize(a));
                const int reps = sz < (4u << 20) ? 100 : 10;
                CK(hipEventRecord(e0, a));
                for (int r = 0; r < reps; r++) kcopy<<<grid, 256, 0, a>>>(src, dst, n);
                CK(hipEventRecord(e1, a));
                CK(hipEventSynchronize(e1));
                float t = 0;
                CK(hipEventElapsedTime(&t, e0, e1));
                std::printf("%8zu KiB kernel copy %s grid %5u: %6.1f GB/s (%.1f us per copy)\n", sz >> 10,
                            dir ? "pinned host -> device" : "device -> pinned host", grid,
                            (double)sz * reps / 1e9 / (t * 1e-3), t * 1e3 / reps);
                std::fflush(stdout);
            }
        }
    }
    // concurrency: a kernel copy in each direction at once (streams a, b), and
    // a kernel copy beside a copy-engine copy the other way
    {
        const size_t sz = 2730ull << 10, n = sz / 16;
        const int reps = 100;
        auto kin = [&](hipStream_t st) { kcopy<<<64, 256, 0, st>>>((const u32x4*)h1, (u32x4*)d1, n); };
        auto kout = [&](hipStream_t st) { kcopy<<<128, 256, 0, st>>>((const u32x4*)d2, (u32x4*)h2, n); };
        auto din = [&](hipStream_t st) { CK(hipMemcpyAsync(d1, h1, sz, hipMemcpyHostToDevice, st)); };
        auto dout = [&](hipStream_t st) { CK(hipMemcpyAsync(h2, d2, sz, hipMemcpyDeviceToHost, st)); };
        auto pair = [&](const char* name, auto fa, auto fb, bool use_b) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, a));
            CK(hipEventRecord(f0, b));
            for (int r = 0; r < reps; r++) {
                fa(a);
                if (use_b) fb(b);
            }
            CK(hipEventRecord(e1, a));
            CK(hipEventRecord(f1, b));
            CK(hipEventSynchronize(e1));
            CK(hipEventSynchronize(f1));
            float ta = 0, tb = 0;
            CK(hipEventElapsedTime(&ta, e0, e1));
            CK(hipEventElapsedTime(&tb, f0, f1));
            const double gb = (double)sz * reps / 1e9;
            std::printf("2730 KiB concurrent %-34s stream a %6.1f GB/s%s", name, gb / (ta * 1e-3), use_b ? "" : "\n");
            if (use_b) std::printf("  stream b %6.1f GB/s\n", gb / (tb * 1e-3));
            std::fflush(stdout);
        };
        pair("kernel H2D alone", kin, kout, false);
        pair("kernel D2H alone", kout, kin, false);
        pair("kernel H2D + kernel D2H", kin, kout, true);
        pair("kernel H2D + kernel H2D", kin, kin, true);
        pair("engine H2D + kernel D2H", din, kout, true);
        pair("kernel H2D + engine D2H", kin, dout, true);
        pair("engine H2D + engine D2H", din, dout, true);
    }
    // round 5: the streaming host decode's own shape without the decode --
    // config B batches with u32 row offsets (2 329 837 B in, 1 451 392 B out
    // per batch, murr_hstream's h2d_bytes / d2h_bytes), four slots each with
    // its own stream: H2D by the copy engine, D2H by a 128-workgroup copy
    // kernel behind it on the slot stream (what murr_hstream issues), or both
    // by engine / both by kernel; batches back to back, slot s + 4 waiting for
    // slot s only through its stream.  batch/s x the Arrow bytes of a batch
    // (1 429 837) is the host-to-host ceiling the stream can reach on this link.
    {
        const size_t in_b = 2329837, out_b = 1451392, arrow_b = 1429837;
        const int depth = 4, batches = 400;
        hipStream_t ss[4];
        for (int k = 0; k < depth; k++) CK(hipStreamCreateWithFlags(&ss[k], hipStreamNonBlocking));
        // 0 engine+kernel, 1 engine+engine, 2 kernel+kernel, 3 engine in two
        // batches per copy (fewer, larger engine copies) + kernel out
        auto stream_shape = [&](const char* name, int mode) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, ss[0]));
            for (int k = 1; k < depth; k++) CK(hipStreamWaitEvent(ss[k], e0, 0));
            if (mode == 3) {
                for (int i = 0; i < batches; i += 2) {
                    hipStream_t st = ss[(i / 2) % depth];
                    uint8_t* din = (uint8_t*)d1 + (size_t)((i / 2) % depth) * (8u << 20);
                    uint8_t* dout = (uint8_t*)d2 + (size_t)((i / 2) % depth) * (8u << 20);
                    uint8_t* hin = (uint8_t*)h1 + (size_t)((i / 2) % depth) * (8u << 20);
                    uint8_t* hout = (uint8_t*)h2 + (size_t)((i / 2) % depth) * (8u << 20);
                    CK(hipMemcpyAsync(din, hin, 2 * in_b, hipMemcpyHostToDevice, st));
                    for (int k = 0; k < 2; k++)
                        kcopy<<<128, 256, 0, st>>>((const u32x4*)(dout + k * (4u << 20)), (u32x4*)(hout + k * (4u << 20)),
                                                   (out_b + 15) / 16);
                }
            }
            for (int i = 0; i < (mode == 3 ? 0 : batches); i++) {
                hipStream_t st = ss[i % depth];
                uint8_t* din = (uint8_t*)d1 + (size_t)(i % depth) * (4u << 20);
                uint8_t* dout = (uint8_t*)d2 + (size_t)(i % depth) * (4u << 20);
                uint8_t* hin = (uint8_t*)h1 + (size_t)(i % depth) * (4u << 20);
                uint8_t* hout = (uint8_t*)h2 + (size_t)(i % depth) * (4u << 20);
                if (mode == 2) kcopy<<<64, 256, 0, st>>>((const u32x4*)hin, (u32x4*)din, (in_b + 15) / 16);
                else CK(hipMemcpyAsync(din, hin, in_b, hipMemcpyHostToDevice, st));
                if (mode == 1) CK(hipMemcpyAsync(hout, dout, out_b, hipMemcpyDeviceToHost, st));
                else kcopy<<<128, 256, 0, st>>>((const u32x4*)dout, (u32x4*)hout, (out_b + 15) / 16);
            }
            for (int k = 0; k < depth; k++) CK(hipStreamSynchronize(ss[k]));
            CK(hipEventRecord(e1, ss[0]));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            const double s = t * 1e-3;
            std::printf("stream shape (B, u32 offsets, depth %d) %-22s %.1f us/batch  in %5.1f GB/s  out %5.1f GB/s  "
                        "ceiling %5.2f GiB/s Arrow host to host\n",
                        depth, name, t * 1e3 / batches, in_b * (double)batches / s / 1e9, out_b * (double)batches / s / 1e9,
                        arrow_b * (double)batches / s / (1024.0 * 1024.0 * 1024.0));
            std::fflush(stdout);
        };
        stream_shape("engine in + kernel out", 0);  // warm
        stream_shape("engine in + kernel out", 0);
        stream_shape("engine in + engine out", 1);
        stream_shape("kernel in + kernel out", 2);
        stream_shape("engine in x2 + kernel out", 3);
    }
    return 0;
}
