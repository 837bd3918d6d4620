// TopK / RandK baseline kernels (comm_hooks/sparse_hook.py) for MI355X (gfx950).
//
// TopK: exact element top-k of |x| per tensor.  Multi-block MSB-first radix select
// (4 digit passes over the tensor, block-local LDS histograms merged with one global
// atomic per bin), then an index-ordered compaction: per-block counts, a scan over
// blocks, and per-block ballot compaction -- so the selected indices come out
// ascending and ties at the threshold resolve to the lowest indices.
// All tensors of a bucket (up to ARCTOPK_SPARSE_MAX_BATCH per launch) go into the
// same launches via blockIdx.y.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"

namespace {

constexpr int kB = ARCTOPK_SPARSE_MAX_BATCH;
constexpr int kHistBlocks = 512;  // blocks per tensor in histogram passes
constexpr int kCmpBlocks = 256;   // fixed range partition per tensor for compaction

struct SparseBatch {
    int64_t off[kB];
    int64_t n[kB];
    int64_t k[kB];
    int64_t koff[kB];
    int32_t nt;
};

struct SelState {      // per tensor
    uint32_t prefix, mask;
    int64_t kk;        // keys still to take among those matching prefix
};

struct Workspace {
    uint32_t hist[kB][256];
    SelState st[kB];
    int64_t cnt_gt[kB][kCmpBlocks];
    int64_t cnt_eq[kB][kCmpBlocks];
    int64_t take_eq[kB][kCmpBlocks];
    int64_t sel_before[kB][kCmpBlocks];
};

__device__ __forceinline__ uint32_t abs_key(float v) { return __float_as_uint(v) & 0x7FFFFFFFu; }

__global__ void k_topk_init(SparseBatch b, Workspace* ws) {
    const int t = blockIdx.x;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) ws->hist[t][i] = 0;
    if (threadIdx.x == 0) {
        ws->st[t].prefix = 0;
        ws->st[t].mask = 0;
        ws->st[t].kk = b.k[t];
    }
}

__global__ void __launch_bounds__(256) k_topk_hist(SparseBatch b, const float* __restrict__ x,
                                                   Workspace* ws, int shift) {
    __shared__ uint32_t h[256];
    const int t = blockIdx.y;
    const int64_t n = b.n[t];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t prefix = ws->st[t].prefix, mask = ws->st[t].mask;
    const float* xs = x + b.off[t];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint32_t k = abs_key(xs[i]);
        if ((k & mask) == prefix) atomicAdd(&h[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    const uint32_t c = h[threadIdx.x];
    if (c) atomicAdd(&ws->hist[t][threadIdx.x], c);
}

// one wave per tensor: pick the digit holding the kk-th largest key, clear the histogram
__global__ void k_topk_digit(SparseBatch b, Workspace* ws, int shift) {
    const int t = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t kk = ws->st[t].kk;
    uint32_t c[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        c[q] = ws->hist[t][255 - 4 * lane - q];
        sum += c[q];
    }
    uint64_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const uint64_t excl = incl - sum;
    if (excl < (uint64_t)kk && incl >= (uint64_t)kk) {
        uint64_t acc = excl;
        int q = 0;
        for (; q < 3; ++q) {
            if (acc + c[q] >= (uint64_t)kk) break;
            acc += c[q];
        }
        const uint32_t d = 255 - 4 * lane - q;
        ws->st[t].prefix |= d << shift;
        ws->st[t].mask |= 255u << shift;
        ws->st[t].kk = kk - (int64_t)acc;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) ws->hist[t][4 * lane + q] = 0;
}

__global__ void __launch_bounds__(256) k_topk_count(SparseBatch b, const float* __restrict__ x,
                                                    Workspace* ws) {
    __shared__ int64_t s_gt[4], s_eq[4];
    const int t = blockIdx.y;
    const int64_t n = b.n[t];
    const int64_t per = (n + kCmpBlocks - 1) / kCmpBlocks;
    const int64_t r0 = min<int64_t>(n, blockIdx.x * per), r1 = min<int64_t>(n, r0 + per);
    const uint32_t T = ws->st[t].prefix;
    const float* xs = x + b.off[t];
    int64_t gt = 0, eq = 0;
    for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) {
        const uint32_t k = abs_key(xs[i]);
        gt += k > T;
        eq += k == T;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        gt += __shfl_xor(gt, o, 64);
        eq += __shfl_xor(eq, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        s_gt[threadIdx.x >> 6] = gt;
        s_eq[threadIdx.x >> 6] = eq;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ws->cnt_gt[t][blockIdx.x] = s_gt[0] + s_gt[1] + s_gt[2] + s_gt[3];
        ws->cnt_eq[t][blockIdx.x] = s_eq[0] + s_eq[1] + s_eq[2] + s_eq[3];
    }
}

// one block (kCmpBlocks threads) per tensor: allowances of threshold-equal keys per
// range (lowest ranges first) and the output offset of every range
__global__ void __launch_bounds__(kCmpBlocks) k_topk_offsets(SparseBatch b, Workspace* ws) {
    __shared__ int64_t buf[kCmpBlocks];
    const int t = blockIdx.x;
    const int i = threadIdx.x;
    const int64_t eq = ws->cnt_eq[t][i];
    buf[i] = eq;
    __syncthreads();
    for (int o = 1; o < kCmpBlocks; o <<= 1) {  // inclusive Hillis-Steele scan
        const int64_t y = i >= o ? buf[i - o] : 0;
        __syncthreads();
        buf[i] += y;
        __syncthreads();
    }
    const int64_t eq_before = buf[i] - eq;
    const int64_t need = ws->st[t].kk;
    int64_t take = need - eq_before;
    take = take < 0 ? 0 : (take > eq ? eq : take);
    ws->take_eq[t][i] = take;
    const int64_t sel = ws->cnt_gt[t][i] + take;
    __syncthreads();
    buf[i] = sel;
    __syncthreads();
    for (int o = 1; o < kCmpBlocks; o <<= 1) {
        const int64_t y = i >= o ? buf[i - o] : 0;
        __syncthreads();
        buf[i] += y;
        __syncthreads();
    }
    ws->sel_before[t][i] = buf[i] - sel;
}

__global__ void __launch_bounds__(256) k_topk_write(SparseBatch b, const float* __restrict__ x,
                                                    Workspace* ws, int32_t* __restrict__ idx,
                                                    float* __restrict__ vals) {
    __shared__ uint32_t s_sel[4], s_eq[4];
    const int t = blockIdx.y;
    const int64_t n = b.n[t];
    const int64_t per = (n + kCmpBlocks - 1) / kCmpBlocks;
    const int64_t r0 = min<int64_t>(n, blockIdx.x * per), r1 = min<int64_t>(n, r0 + per);
    const uint32_t T = ws->st[t].prefix;
    const int64_t take_eq = ws->take_eq[t][blockIdx.x];
    int64_t slot = ws->sel_before[t][blockIdx.x];
    int64_t eq_seen = 0;
    const float* xs = x + b.off[t];
    int32_t* oi = idx + b.koff[t];
    float* ov = vals + b.koff[t];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int64_t base = r0; base < r1; base += 256) {
        const int64_t i = base + threadIdx.x;
        float v = 0.f;
        uint32_t k = 0;
        const bool in = i < r1;
        if (in) {
            v = xs[i];
            k = abs_key(v);
        }
        const bool gt = in && k > T;
        const bool eq = in && k == T;
        // rank of this eq among the tile's eqs (index order)
        const uint64_t beq = __ballot(eq);
        if (lane == 0) s_eq[wave] = __popcll(beq);
        __syncthreads();
        uint32_t eq_rank = __popcll(beq & lt);
        for (int w = 0; w < wave; ++w) eq_rank += s_eq[w];
        const uint32_t eq_tile = s_eq[0] + s_eq[1] + s_eq[2] + s_eq[3];
        const bool sel = gt || (eq && (eq_seen + eq_rank) < take_eq);
        const uint64_t bsel = __ballot(sel);
        if (lane == 0) s_sel[wave] = __popcll(bsel);
        __syncthreads();
        uint32_t sel_rank = __popcll(bsel & lt);
        for (int w = 0; w < wave; ++w) sel_rank += s_sel[w];
        const uint32_t sel_tile = s_sel[0] + s_sel[1] + s_sel[2] + s_sel[3];
        if (sel) {
            oi[slot + sel_rank] = (int32_t)i;
            ov[slot + sel_rank] = v;
        }
        slot += sel_tile;
        eq_seen += eq_tile;
        __syncthreads();
    }
}

// ---- RandK index source: keyed Feistel permutation of [0, 2^bits), cycle-walked to [0, n)
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du;
    x ^= x >> 15; x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t feistel(uint32_t v, int half, uint32_t hmask, uint64_t key) {
    uint32_t L = v >> half, R = v & hmask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t f = mix32(R ^ (uint32_t)(key >> (r * 8)) ^ (uint32_t)(key >> 32) * (r + 1)) & hmask;
        const uint32_t nl = R;
        R = L ^ f;
        L = nl;
    }
    return (L << half) | R;
}

__global__ void __launch_bounds__(256) k_randk(SparseBatch b, uint64_t seed, int32_t* __restrict__ idx) {
    const int t = blockIdx.y;
    const int64_t n = b.n[t], k = b.k[t];
    int bits = 2;
    while ((1ll << bits) < n) ++bits;
    if (bits & 1) ++bits;  // balanced halves
    const int half = bits / 2;
    const uint32_t hmask = (1u << half) - 1u;
    const uint64_t key = seed * 0x9E3779B97F4A7C15ull + (uint64_t)(t + 1) * 0xD1B54A32D192ED03ull;
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
        uint32_t v = (uint32_t)j;
        // cycle walking: the orbit of j returns below n; bounded for safety
        for (int it = 0; it < 4096; ++it) {
            v = feistel(v, half, hmask, key);
            if (v < (uint32_t)n) break;
        }
        idx[b.koff[t] + j] = (int32_t)v;
    }
}

__global__ void __launch_bounds__(256) k_gather(SparseBatch b, const float* __restrict__ x,
                                                const int32_t* __restrict__ idx,
                                                float* __restrict__ vals) {
    const int t = blockIdx.y;
    const int64_t k = b.k[t];
    const float* xs = x + b.off[t];
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256)
        vals[b.koff[t] + j] = xs[idx[b.koff[t] + j]];
}

template <int EF>
__global__ void __launch_bounds__(256) k_residual(SparseBatch b, float* __restrict__ E,
                                                  const int32_t* __restrict__ idx,
                                                  const float* __restrict__ vals) {
    const int t = blockIdx.y;
    const int64_t k = b.k[t];
    float* es = E + b.off[t];
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
        const int32_t i = idx[b.koff[t] + j];
        if constexpr (EF == ARCTOPK_EF14) es[i] = 0.f;
        else es[i] = es[i] + vals[b.koff[t] + j];
    }
}

// rank-ordered decode: one launch per rank keeps the sum order of the reference
template <bool ACC>
__global__ void __launch_bounds__(256) k_scatter(SparseBatch b, float* __restrict__ out,
                                                 const int32_t* __restrict__ idx,
                                                 const float* __restrict__ vals, float wsf) {
    const int t = blockIdx.y;
    const int64_t k = b.k[t];
    float* os = out + b.off[t];
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
        const int32_t i = idx[b.koff[t] + j];
        const float v = vals[b.koff[t] + j];
        if constexpr (ACC) os[i] = os[i] + v;          // indices unique within one payload
        else os[i] = __fdiv_rn(v, wsf);
    }
}

__global__ void __launch_bounds__(256) k_div_gE(float* __restrict__ out, float* __restrict__ gE,
                                                int64_t n, float wsf, int do_div) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float v = out[i];
        if (do_div) v = __fdiv_rn(v, wsf);
        if (gE) {
            v = gE[i] + v;
            gE[i] = v;
        }
        out[i] = v;
    }
}

int fill_batch(SparseBatch& b, int32_t first, int32_t count, const int64_t* offsets,
               const int64_t* numels, const int64_t* ks, const int64_t* k_off, int64_t& maxn,
               int64_t& maxk) {
    b.nt = count;
    maxn = maxk = 0;
    for (int i = 0; i < count; ++i) {
        b.off[i] = offsets ? offsets[first + i] : 0;
        b.n[i] = numels ? numels[first + i] : 0;
        b.k[i] = ks[first + i];
        b.koff[i] = k_off[first + i];
        if (numels && (b.n[i] < 1 || b.n[i] >= (1ll << 31))) return ARCTOPK_EINVAL;
        if (numels && (b.k[i] < 1 || b.k[i] > b.n[i])) return ARCTOPK_EINVAL;
        maxn = std::max(maxn, b.n[i]);
        maxk = std::max(maxk, b.k[i]);
    }
    return 0;
}

inline int grid_for(int64_t work, int cap) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(cap, (work + 255) / 256));
}

}  // namespace

extern "C" int64_t arctopk_sparse_workspace_bytes(void) { return (int64_t)sizeof(Workspace); }

extern "C" int arctopk_topk_select(const float* x, int32_t nt, const int64_t* offsets,
                                   const int64_t* numels, const int64_t* ks, const int64_t* k_off,
                                   int32_t* idx, float* vals, void* workspace, void* stream) {
    if (!x || !offsets || !numels || !ks || !k_off || !idx || !vals || !workspace || nt < 1)
        return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    Workspace* ws = (Workspace*)workspace;
    for (int32_t first = 0; first < nt; first += kB) {
        SparseBatch b;
        int64_t maxn, maxk;
        const int cnt = std::min<int32_t>(kB, nt - first);
        int e = fill_batch(b, first, cnt, offsets, numels, ks, k_off, maxn, maxk);
        if (e) return e;
        hipLaunchKernelGGL(k_topk_init, dim3(cnt), dim3(256), 0, st, b, ws);
        const int hb = grid_for(maxn, kHistBlocks);
        for (int shift = 24; shift >= 0; shift -= 8) {
            hipLaunchKernelGGL(k_topk_hist, dim3(hb, cnt), dim3(256), 0, st, b, x, ws, shift);
            hipLaunchKernelGGL(k_topk_digit, dim3(cnt), dim3(64), 0, st, b, ws, shift);
        }
        hipLaunchKernelGGL(k_topk_count, dim3(kCmpBlocks, cnt), dim3(256), 0, st, b, x, ws);
        hipLaunchKernelGGL(k_topk_offsets, dim3(cnt), dim3(kCmpBlocks), 0, st, b, ws);
        hipLaunchKernelGGL(k_topk_write, dim3(kCmpBlocks, cnt), dim3(256), 0, st, b, x, ws, idx, vals);
        e = (int)hipGetLastError();
        if (e) return e;
    }
    return 0;
}

extern "C" int arctopk_randk_indices(int32_t nt, const int64_t* numels, const int64_t* ks,
                                     const int64_t* k_off, uint64_t seed, int32_t* idx, void* stream) {
    if (!numels || !ks || !k_off || !idx || nt < 1) return ARCTOPK_EINVAL;
    for (int32_t first = 0; first < nt; first += kB) {
        SparseBatch b;
        int64_t maxn, maxk;
        const int cnt = std::min<int32_t>(kB, nt - first);
        int e = fill_batch(b, first, cnt, nullptr, numels, ks, k_off, maxn, maxk);
        if (e) return e;
        hipLaunchKernelGGL(k_randk, dim3(grid_for(maxk, 2048), cnt), dim3(256), 0,
                           (hipStream_t)stream, b, seed + (uint64_t)first, idx);
        e = (int)hipGetLastError();
        if (e) return e;
    }
    return 0;
}

extern "C" int arctopk_sparse_gather(const float* x, int32_t nt, const int64_t* offsets,
                                     const int64_t* ks, const int64_t* k_off, const int32_t* idx,
                                     float* vals, void* stream) {
    if (!x || !offsets || !ks || !k_off || !idx || !vals || nt < 1) return ARCTOPK_EINVAL;
    for (int32_t first = 0; first < nt; first += kB) {
        SparseBatch b;
        int64_t maxn, maxk;
        const int cnt = std::min<int32_t>(kB, nt - first);
        int e = fill_batch(b, first, cnt, offsets, nullptr, ks, k_off, maxn, maxk);
        if (e) return e;
        hipLaunchKernelGGL(k_gather, dim3(grid_for(maxk, 2048), cnt), dim3(256), 0,
                           (hipStream_t)stream, b, x, idx, vals);
        e = (int)hipGetLastError();
        if (e) return e;
    }
    return 0;
}

extern "C" int arctopk_sparse_residual(float* E, int32_t nt, const int64_t* offsets,
                                       const int64_t* ks, const int64_t* k_off, const int32_t* idx,
                                       const float* vals, int32_t ef, void* stream) {
    if (ef == ARCTOPK_EF_NONE) return 0;
    if (!E || !offsets || !ks || !k_off || !idx || nt < 1) return ARCTOPK_EINVAL;
    if (ef == ARCTOPK_EF21 && !vals) return ARCTOPK_EINVAL;
    for (int32_t first = 0; first < nt; first += kB) {
        SparseBatch b;
        int64_t maxn, maxk;
        const int cnt = std::min<int32_t>(kB, nt - first);
        int e = fill_batch(b, first, cnt, offsets, nullptr, ks, k_off, maxn, maxk);
        if (e) return e;
        dim3 grid(grid_for(maxk, 2048), cnt);
        if (ef == ARCTOPK_EF14)
            hipLaunchKernelGGL(k_residual<ARCTOPK_EF14>, grid, dim3(256), 0, (hipStream_t)stream, b, E, idx, vals);
        else if (ef == ARCTOPK_EF21)
            hipLaunchKernelGGL(k_residual<ARCTOPK_EF21>, grid, dim3(256), 0, (hipStream_t)stream, b, E, idx, vals);
        else
            return ARCTOPK_EINVAL;
        e = (int)hipGetLastError();
        if (e) return e;
    }
    return 0;
}

extern "C" int arctopk_sparse_decode(float* out, int64_t numel, int32_t nt, const int64_t* offsets,
                                     const int64_t* ks, const int64_t* k_off, int64_t packed_len,
                                     const int32_t* idx, const float* vals, int32_t nranks,
                                     int32_t world_size, int32_t accumulate, float* gerr,
                                     void* stream) {
    if (!out || !offsets || !ks || !k_off || !idx || !vals || nt < 1 || nranks < 1 ||
        world_size < 1 || numel < 0)
        return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    hipError_t he = hipMemsetAsync(out, 0, (size_t)numel * sizeof(float), st);
    if (he != hipSuccess) return (int)he;
    const float wsf = (float)world_size;
    const int nr = accumulate ? nranks : 1;
    for (int q = 0; q < nr; ++q) {
        for (int32_t first = 0; first < nt; first += kB) {
            SparseBatch b;
            int64_t maxn, maxk;
            const int cnt = std::min<int32_t>(kB, nt - first);
            int e = fill_batch(b, first, cnt, offsets, nullptr, ks, k_off, maxn, maxk);
            if (e) return e;
            dim3 grid(grid_for(maxk, 2048), cnt);
            const int32_t* iq = idx + (int64_t)q * packed_len;
            const float* vq = vals + (int64_t)q * packed_len;
            if (accumulate)
                hipLaunchKernelGGL(k_scatter<true>, grid, dim3(256), 0, st, b, out, iq, vq, wsf);
            else
                hipLaunchKernelGGL(k_scatter<false>, grid, dim3(256), 0, st, b, out, iq, vq, wsf);
        }
    }
    if (accumulate || gerr) {
        hipLaunchKernelGGL(k_div_gE, dim3(grid_for(numel, 8192)), dim3(256), 0, st, out, gerr,
                           numel, wsf, accumulate);
    }
    return (int)hipGetLastError();
}
