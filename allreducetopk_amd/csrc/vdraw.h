// Device projections: the reference's V draws, on the GPU, bit for bit (device side).
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
// min(ceil(numel / 256), CUs * maxThreadsPerCU / 256) (vdraw_table, vdraw.hip).  Every
// element is computed independently from that mapping, so any block can draw any range:
// draw_v_chunk serves both the standalone draw kernel and the trailing blocks of the select
// launch that draw the NEXT call's projections (arctopk_select_draw).
//
// Include this header before anything else that includes rocrand: its Box-Muller transform
// is compiled with fast floating-point contraction, as in torch's HIP build (hipcc's
// default); the rest of the translation unit keeps -ffp-contract=off.
#pragma once

#include "common.h"

#pragma clang fp contract(fast)
#include <hiprand/hiprand_kernel.h>

namespace arctopk {

template <typename T>
__device__ __forceinline__ void draw_v_chunk(const VDraw* __restrict__ segs, const VChunk c,
                                             uint64_t seed, T* __restrict__ V, int tid, int nt) {
    const VDraw d = segs[c.entry];
    const uint32_t S = (uint32_t)d.stride;  // numel < 2^31 (plan checks m * r)
    for (uint32_t li = c.lo + (uint32_t)tid; li < c.hi; li += (uint32_t)nt) {
        uint32_t t = li, q = 0;  // element li = thread t's component q % 4 of draw q / 4
        if (li >= S) {
            q = li / S;
            t = li - q * S;
        }
        hiprandStatePhilox4_32_10_t st;
        hiprand_init(seed, t, d.offset, &st);
        for (uint32_t k = q >> 2; k > 0; --k) (void)rocrand4(&st);
        // curand_normal4 = (box_muller(x, y), box_muller(z, w)): only the needed pair
        const uint4 u = rocrand4(&st);
        const uint32_t j = q & 3u;
        const float2 bm = j < 2 ? rocrand_device::detail::box_muller(u.x, u.y)
                                : rocrand_device::detail::box_muller(u.z, u.w);
        const float z = (j & 1u) ? bm.y : bm.x;
        const float one = 1.0f, zero = 0.0f;
        V[d.v_off + li] = from_f<T>(z * one + zero);  // normal transform: rand * std + mean
    }
}

// the trailing `job.n` blocks of a launch draw one chunk each; true for those blocks
template <typename T>
__device__ __forceinline__ bool maybe_draw_v(const VDrawJob& job, int nt) {
    const int b = (int)blockIdx.x - ((int)gridDim.x - job.n);
    if (b < 0) return false;
    draw_v_chunk<T>(job.segs, job.chunks[b], job.seed, static_cast<T*>(job.V), (int)threadIdx.x, nt);
    return true;
}

}  // namespace arctopk

#pragma clang fp contract(off)
