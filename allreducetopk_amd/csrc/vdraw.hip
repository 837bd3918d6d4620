// Device projections: the standalone draw kernel and the host-side draw table (vdraw.h
// states torch's launch mapping that both follow).
#include "vdraw.h"

#include <algorithm>

using namespace arctopk;

namespace {

template <typename T>
__global__ void __launch_bounds__(256) k_draw_v(const VDraw* __restrict__ segs,
                                                const VChunk* __restrict__ chunks, uint64_t seed,
                                                T* __restrict__ V) {
    draw_v_chunk<T>(segs, chunks[blockIdx.x], seed, V, (int)threadIdx.x, 256);
}

}  // namespace

namespace arctopk {

// host: the draw table of a plan's SKETCH segments (torch's launch geometry on `device`)
int vdraw_table(const arctopk_segment* segs, int nseg, int r, int device, VDraw* out, int* nout,
                uint64_t* advance) {
    int sms = 0, maxthr = 0;
    hipError_t e = hipDeviceGetAttribute(&sms, hipDeviceAttributeMultiprocessorCount, device);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&maxthr, hipDeviceAttributeMaxThreadsPerMultiProcessor, device);
    if (e != hipSuccess) return (int)e;
    const uint64_t grid_cap = (uint64_t)sms * (uint64_t)(maxthr / 256);
    uint64_t off = 0;
    int n = 0;
    for (int i = 0; i < nseg; ++i) {
        if (segs[i].kind != ARCTOPK_SEG_SKETCH) continue;
        const uint64_t numel = (uint64_t)segs[i].m * (uint64_t)r;
        const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((numel + 255) / 256, grid_cap));
        const uint64_t stride = 256 * grid;
        VDraw& d = out[n++];
        d.v_off = segs[i].v_off;
        d.numel = (int64_t)numel;
        d.stride = stride;
        d.offset = off;
        uint64_t inc = ((numel - 1) / (stride * 4) + 1) * 4;
        inc = (inc + 3) / 4 * 4;  // philox_cuda_state rounds the increment to a multiple of 4
        off += inc;
    }
    *nout = n;
    *advance = off;
    return 0;
}

}  // namespace arctopk

extern "C" int arctopk_draw_projections(const arctopk_plan* p, uint64_t seed, void* V, void* stream) {
    if (!p || !V) return ARCTOPK_EINVAL;
    if (p->n_vdraw == 0) return 0;
    const dim3 grid((unsigned)p->n_vchunk);
    hipStream_t st = (hipStream_t)stream;
    if (p->dtype == ARCTOPK_BF16)
        hipLaunchKernelGGL(k_draw_v<bf16_t>, grid, dim3(256), 0, st, p->d_vdraw, p->d_vchunk, seed,
                           static_cast<bf16_t*>(V));
    else
        hipLaunchKernelGGL(k_draw_v<float>, grid, dim3(256), 0, st, p->d_vdraw, p->d_vchunk, seed,
                           static_cast<float*>(V));
    return (int)hipGetLastError();
}

extern "C" int arctopk_plan_philox_advance(const arctopk_plan* p, uint64_t* advance) {
    if (!p || !advance) return ARCTOPK_EINVAL;
    *advance = p->vdraw_advance;
    return 0;
}
