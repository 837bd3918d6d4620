// Emulated wire (measurement only): what an R-rank ring all-reduce costs the local GPU,
// without the other R - 1 GPUs.
//
// A ring all-reduce of B bytes (reduce-scatter + all-gather, 2 (R - 1) steps of B / R) reads
// and writes 2 (R - 1) / R * B bytes of the local HBM (chunks sent are read, chunks received
// are written), on the CUs of the collective's workgroups, and cannot finish before the wire
// has carried them: 2 (R - 1) / R * B / busBW (plus a fixed latency).  This kernel reproduces
// those three costs on one GPU so that the exchange step (exchange.cpp) can be measured beside
// an 8-rank wire: `blocks` workgroups read and rewrite 2 (R - 1) / R * B bytes of the buffer in
// place (values unchanged: the result is a one-rank all-reduce's), each workgroup pacing its
// share of the traffic by the device's constant-rate clock so that the whole takes at least
// latency + 2 (R - 1) / R * B / busBW.  Under HBM contention it runs slower than its pace:
// that is what it is for.  Not a collective, not in the product path of any hook.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "common.h"

namespace arctopk {
namespace {

constexpr int kWireThreads = 256;
// 16-B units per thread per slice: a slice is one memory round trip, so a workgroup moves at most
// a slice per round trip.  32 KiB slices (8 units) made the kernel latency-bound beside the
// encode (~90 slices per workgroup at 350 GB/s x ~5 us round trips > its 283 us pace: the
// emulated collective ran 387-642 us); 128 KiB slices keep ~22 round trips per workgroup.
constexpr int kWireUnroll = 32;
constexpr int64_t kWireSlice = (int64_t)kWireThreads * kWireUnroll;  // units per paced slice (128 KiB)

__global__ void __launch_bounds__(kWireThreads) k_wire(float4* __restrict__ buf, int64_t n4, int64_t moves,
                                                       uint64_t ticks) {
    const int64_t per = (moves + gridDim.x - 1) / gridDim.x;
    const int64_t u0 = (int64_t)blockIdx.x * per;
    const int64_t u1 = min(moves, u0 + per);
    const uint64_t t0 = wall_clock64();
    if (u0 < u1) {
        const int64_t span = u1 - u0;
        for (int64_t s = u0; s < u1; s += kWireSlice) {
            const uint64_t due = t0 + (uint64_t)((s - u0) * (int64_t)ticks / span);
            while (wall_clock64() < due) __builtin_amdgcn_s_sleep(4);
            float4 v[kWireUnroll];
            int64_t at[kWireUnroll];
#pragma unroll
            for (int j = 0; j < kWireUnroll; ++j) {
                const int64_t u = s + j * kWireThreads + threadIdx.x;
                at[j] = u < u1 ? u % n4 : -1;
                if (at[j] >= 0) v[j] = buf[at[j]];
            }
#pragma unroll
            for (int j = 0; j < kWireUnroll; ++j)
                if (at[j] >= 0) buf[at[j]] = v[j];
        }
    }
    // the wire's time: nothing of this all-reduce completes before it
    while (wall_clock64() < t0 + ticks) __builtin_amdgcn_s_sleep(8);
}

}  // namespace

// `done` (may be null): completed by the kernel's own completion signal (the communicator's
// serialisation event, exchange.cpp)
int wire_allreduce(const WireParams& w, void* buf, int64_t bytes, hipStream_t st, hipEvent_t done) {
    if (bytes < 0 || (bytes && !buf) || w.ranks < 1 || w.blocks < 1) return ARCTOPK_EINVAL;
    int dev = 0, khz = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    if (e != hipSuccess) return (int)e;
    if (khz <= 0) return ARCTOPK_EINVAL;
    const double frac = 2.0 * (w.ranks - 1) / w.ranks;  // of the buffer, read and written
    const double us = w.latency_us + frac * (double)bytes / (w.busbw_gbs * 1e3);
    const uint64_t ticks = (uint64_t)(us * (double)khz / 1e3);
    const int64_t n4 = bytes / 16;
    const int64_t moves = n4 > 0 ? (int64_t)(frac * (double)n4 + 0.5) : 0;
    if (done)
        hipExtLaunchKernelGGL(k_wire, dim3(w.blocks), dim3(kWireThreads), 0, st, nullptr, done, 0,
                              static_cast<float4*>(buf), n4 > 0 ? n4 : 1, moves, ticks);
    else
        hipLaunchKernelGGL(k_wire, dim3(w.blocks), dim3(kWireThreads), 0, st, static_cast<float4*>(buf),
                           n4 > 0 ? n4 : 1, moves, ticks);
    return (int)hipGetLastError();
}

}  // namespace arctopk
