// murr_ipc.hip — packs one Arrow IPC record-batch message in HBM.
//
// After a decode, a batch's Arrow buffers sit in separate device allocations.
// The IPC writers of the read path (StreamWriter in the HTTP fetch handler,
// src/api/http/handlers.rs:93-101; FlightDataEncoder in DoGet,
// src/api/flight/mod.rs:85-87) serialise them into one message: metadata, then
// every buffer at an aligned offset with zeroed padding.  This kernel builds
// that message on the device -- job 0 copies the metadata murr_ipc.cpp wrote,
// the others copy one Arrow buffer each and zero its padding -- so the host
// receives a wire-ready message with a single D2H copy.
//
// Pure byte movement, HBM-bound: blockIdx.y picks a job, the x dimension
// strides over it in 16-B units (dwordx4 loads/stores when both sides are
// 16-B aligned, dwordx2 at 8 B, bytes otherwise).
#include "murr_internal.h"

namespace murr {

namespace {

constexpr uint32_t kPackThreads = 256;

__global__ void __launch_bounds__(kPackThreads) ipc_pack(const IpcJob* __restrict__ jobs) {
    const IpcJob j = jobs[blockIdx.y];
    const uint64_t units = (j.padded + 15) / 16;
    const uintptr_t mis = (reinterpret_cast<uintptr_t>(j.src) | reinterpret_cast<uintptr_t>(j.dst));
    const bool a16 = (mis & 15) == 0, a8 = (mis & 7) == 0;
    for (uint64_t u = (uint64_t)blockIdx.x * kPackThreads + threadIdx.x; u < units;
         u += (uint64_t)gridDim.x * kPackThreads) {
        const uint64_t b = u * 16;
        if (b + 16 <= j.len) {
            if (a16) {
                *reinterpret_cast<uint4*>(j.dst + b) = *reinterpret_cast<const uint4*>(j.src + b);
                continue;
            }
            if (a8) {
                const uint2* s = reinterpret_cast<const uint2*>(j.src + b);
                uint2* d = reinterpret_cast<uint2*>(j.dst + b);
                uint2 x = s[0], y = s[1];
                d[0] = x;
                d[1] = y;
                continue;
            }
        }
        const uint64_t end = b + 16 < j.padded ? b + 16 : j.padded;
        for (uint64_t k = b; k < end; k++) j.dst[k] = k < j.len ? j.src[k] : (uint8_t)0;
    }
}

}  // namespace

hipError_t launch_ipc_pack(const IpcJob* jobs, uint32_t njobs, uint64_t max_padded, hipStream_t s) {
    if (!njobs) return hipSuccess;
    uint64_t units = (max_padded + 15) / 16;
    uint64_t gx = (units + kPackThreads * 4 - 1) / (kPackThreads * 4);  // ~4 units per thread
    if (gx < 1) gx = 1;
    if (gx > 2048) gx = 2048;
    hipLaunchKernelGGL(ipc_pack, dim3((uint32_t)gx, njobs), dim3(kPackThreads), 0, s, jobs);
    return hipGetLastError();
}

}  // namespace murr
