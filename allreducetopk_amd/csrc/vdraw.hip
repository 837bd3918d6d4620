// Device projections: the reference's V draws, on the GPU, bit for bit.
//
// The reference draws V = torch.randn(m, r, device=tensor.device, dtype=tensor.dtype) for
// every 2-D / ND tensor of a bucket, in bucket order, right after torch.manual_seed(seed)
// (comm_hooks/group_topk_hook_no_reshape.py:49, :79, :255).  On a GPU that is torch's
// normal_ kernel: Philox4x32-10 (hiprand / rocrand on ROCm), one state per thread of a
// grid-stride launch -- thread t of a launch with S = 256 * grid threads is initialised with
// (seed, subsequence t, the generator's offset), draws curand_normal4 once per loop
// iteration k, and element t + S * (4k + j) gets component j of iteration k, transformed by
// rand * std + mean (std 1, mean 0) and cast to the tensor's dtype.  After each draw the
// generator's offset advances by ((numel - 1) / (4 S) + 1) * 4.  The grid is
// min(ceil(numel / 256), CUs * maxThreadsPerCU / 256).  This kernel computes every element
// of every tensor's draw independently from that mapping.
//
// Floating-point contraction as in torch's HIP build (hipcc's default, fast): the Box-Muller
// transform inside rocrand is compiled here with the same contraction.
#pragma clang fp contract(fast)
#include <hiprand/hiprand_kernel.h>

#include <algorithm>

#include "common.h"

using namespace arctopk;

namespace {

template <typename T>
__global__ void __launch_bounds__(256) k_draw_v(const VDraw* __restrict__ segs, uint64_t seed,
                                                T* __restrict__ V) {
    const VDraw d = segs[blockIdx.y];
    for (int64_t li = (int64_t)blockIdx.x * 256 + threadIdx.x; li < d.numel;
         li += (int64_t)gridDim.x * 256) {
        const uint64_t t = (uint64_t)li % d.stride, q = (uint64_t)li / d.stride;
        hiprandStatePhilox4_32_10_t st;
        hiprand_init(seed, t, d.offset, &st);
        for (uint64_t k = q >> 2; k > 0; --k) (void)hiprand_normal4(&st);
        const float4 r = hiprand_normal4(&st);
        const int j = (int)(q & 3u);
        const float z = j == 0 ? r.x : (j == 1 ? r.y : (j == 2 ? r.z : r.w));
        const float one = 1.0f, zero = 0.0f;
        V[d.v_off + li] = from_f<T>(z * one + zero);  // normal transform: rand * std + mean
    }
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
    const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(64, (p->vdraw_max + 255) / 256)),
                    (unsigned)p->n_vdraw);
    hipStream_t st = (hipStream_t)stream;
    if (p->dtype == ARCTOPK_BF16)
        hipLaunchKernelGGL(k_draw_v<bf16_t>, grid, dim3(256), 0, st, p->d_vdraw, seed, static_cast<bf16_t*>(V));
    else
        hipLaunchKernelGGL(k_draw_v<float>, grid, dim3(256), 0, st, p->d_vdraw, seed, static_cast<float*>(V));
    return (int)hipGetLastError();
}

extern "C" int arctopk_plan_philox_advance(const arctopk_plan* p, uint64_t* advance) {
    if (!p || !advance) return ARCTOPK_EINVAL;
    *advance = p->vdraw_advance;
    return 0;
}
