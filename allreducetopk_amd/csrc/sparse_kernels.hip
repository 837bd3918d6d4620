// TopK / RandK baseline kernels (comm_hooks/sparse_hook.py) for MI355X (gfx950).
//
// TopK: exact element top-k of |x| per tensor.  Multi-block MSB-first radix select
// (4 digit passes over the tensor, block-local LDS histograms merged with one global
// atomic per bin), then an index-ordered compaction: per-block counts, a scan over
// blocks, and per-block ballot compaction -- so the selected indices come out
// ascending and ties at the threshold resolve to the lowest indices.
// All tensors of a bucket (up to ARCTOPK_SPARSE_MAX_BATCH per launch) go into the
// same launches via blockIdx.y.  fp32 and bf16 buckets: values, residuals and the decoded
// bucket stay in the bucket dtype, every add / divide rounded to it as the reference's
// torch ops on a bf16 tensor do (sparse_hook.py:16-34, :103-141, :257-297).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "common.h"
#include "mselect.h"

namespace {

constexpr int kB = ARCTOPK_SPARSE_MAX_BATCH;

struct SparseBatch {
    int64_t off[kB];
    int64_t n[kB];
    int64_t k[kB];
    int64_t koff[kB];
    int32_t nt;
};



template <typename T>
__global__ void __launch_bounds__(256) k_gather(SparseBatch b, const T* __restrict__ x,
                                                const int32_t* __restrict__ idx,
                                                T* __restrict__ vals) {
    const int t = blockIdx.y;
    const int64_t k = b.k[t];
    const T* xs = x + b.off[t];
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256)
        vals[b.koff[t] + j] = xs[idx[b.koff[t] + j]];
}

// EF21: E[i] = E[i] + decay * v, one rounding (torch's add_(C, alpha) on CPU: a fused
// multiply-add per element, sparse_hook.py:265; decay = 1 gives E[i] + v exactly)
template <typename T, int EF>
__global__ void __launch_bounds__(256) k_residual(SparseBatch b, T* __restrict__ E,
                                                  const int32_t* __restrict__ idx,
                                                  const T* __restrict__ vals, float decay) {
    const int t = blockIdx.y;
    const int64_t k = b.k[t];
    T* es = E + b.off[t];
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
        const int32_t i = idx[b.koff[t] + j];
        if constexpr (EF == ARCTOPK_EF14) es[i] = arctopk::from_f<T>(0.f);
        else
            es[i] = arctopk::from_f<T>(__fmaf_rn(decay, arctopk::to_f(vals[b.koff[t] + j]), arctopk::to_f(es[i])));
    }
}

// rank-ordered decode: one launch per rank keeps the sum order of the reference
// MODE 0: out[i] = v / ws (RandK); 1: out[i] += v (TopK, ranks after the first);
// 2: out[i] = 0 + v (TopK's first rank into the zeroed bucket: no read, -0 still becomes +0)
template <typename T, int MODE>
__global__ void __launch_bounds__(256) k_scatter(SparseBatch b, T* __restrict__ out,
                                                 const int32_t* __restrict__ idx,
                                                 const T* __restrict__ vals, float wsf) {
    using arctopk::from_f;
    using arctopk::to_f;
    const int t = blockIdx.y;
    const int64_t k = b.k[t];
    T* os = out + b.off[t];
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
        const int32_t i = idx[b.koff[t] + j];
        const float v = to_f(vals[b.koff[t] + j]);
        if constexpr (MODE == 1) os[i] = from_f<T>(to_f(os[i]) + v);  // indices unique within one payload
        else if constexpr (MODE == 2) os[i] = from_f<T>(0.f + v);
        else os[i] = from_f<T>(__fdiv_rn(v, wsf));
    }
}

// TopK's first payload (rank 0) -- or RandK's all-reduced payload (DIV: v / ws) -- into the
// bucket, zero fill included: each block composes a 4096-element chunk of one tensor in LDS
// (zeros, then the values at the payload's indices that fall in the chunk) and writes it whole.
// The payload's indices are ascending per tensor (arctopk_topk_select, arctopk_randk_select), so
// the chunk's slice of them is found by two 64-way searches.  Replaces the bucket memset + a
// scattered pass.
constexpr int kDecChunk = 4096;

// first position in a[lo, hi) with a[p] >= target (a ascending), one wave
__device__ __forceinline__ int64_t wave_lower_bound(const int32_t* __restrict__ a, int64_t lo, int64_t hi,
                                                    int32_t target) {
    const int lane = threadIdx.x & 63;
    while (hi - lo > 64) {
        const int64_t step = (hi - lo + 63) / 64;
        const int64_t p = lo + (int64_t)lane * step;
        const bool pred = p < hi && a[p] < target;
        const int c = __popcll(__ballot(pred));
        if (c == 0) return lo;
        const int64_t nlo = lo + (int64_t)(c - 1) * step + 1;
        const int64_t phi = lo + (int64_t)c * step;
        hi = phi < hi ? phi : hi;
        lo = nlo;
    }
    const int64_t p = lo + lane;
    return lo + __popcll(__ballot(p < hi && a[p] < target));
}

template <typename T, bool DIV>
__global__ void __launch_bounds__(256) k_scatter_first(SparseBatch b, T* __restrict__ out,
                                                       const int32_t* __restrict__ idx,
                                                       const T* __restrict__ vals, float wsf) {
    using arctopk::from_f;
    using arctopk::to_f;
    __shared__ T chunk[kDecChunk];
    __shared__ int64_t s_lb[2];
    const int t = blockIdx.y;
    const int64_t n = b.n[t];
    const int64_t c0 = (int64_t)blockIdx.x * kDecChunk;
    if (c0 >= n) return;
    const int64_t c1 = min<int64_t>(n, c0 + kDecChunk);
    const int32_t* it = idx + b.koff[t];
    const T* vt = vals + b.koff[t];
    const int wave = threadIdx.x >> 6;
    if (wave < 2) {
        const int64_t lb = wave_lower_bound(it, 0, b.k[t], (int32_t)(wave == 0 ? c0 : c1));
        if ((threadIdx.x & 63) == 0) s_lb[wave] = lb;
    }
    for (int e = threadIdx.x; e < kDecChunk; e += 256) chunk[e] = from_f<T>(0.f);
    __syncthreads();
    for (int64_t j = s_lb[0] + threadIdx.x; j < s_lb[1]; j += 256)  // TopK: 0 + v; RandK: v / ws
        chunk[it[j] - c0] = DIV ? from_f<T>(__fdiv_rn(to_f(vt[j]), wsf)) : from_f<T>(0.f + to_f(vt[j]));
    __syncthreads();
    T* o = out + b.off[t] + c0;
    for (int64_t e = threadIdx.x; e < c1 - c0; e += 256) o[e] = chunk[e];
}

// TopK's out /= ws; EF21: gE = gE + decay * out (one rounding, as torch's add_ with alpha,
// sparse_hook.py:296), out = gE
template <typename T>
__global__ void __launch_bounds__(256) k_div_gE(T* __restrict__ out, T* __restrict__ gE,
                                                int64_t n, float wsf, int do_div, float decay) {
    using arctopk::from_f;
    using arctopk::to_f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float v = to_f(out[i]);
        if (do_div) v = to_f(from_f<T>(__fdiv_rn(v, wsf)));
        if (gE) {
            v = to_f(from_f<T>(__fmaf_rn(decay, v, to_f(gE[i]))));
            gE[i] = from_f<T>(v);
        }
        out[i] = from_f<T>(v);
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

// Tensors of at most kMSmallSel elements take the single-block select (ms_select_small), the rest
// the multi-block one, in batches of kMB in tensor order within each group
static void split_small(int32_t nt, const int64_t* numels, std::vector<int32_t>* small, std::vector<int32_t>* large) {
    for (int32_t j = 0; j < nt; ++j) (numels[j] <= arctopk::kMSmallSel ? small : large)->push_back(j);
}

// candidate slots the multi-block select needs: the largest per-batch sum of its items' capacities
static int64_t topk_cap_total(int32_t nt, const int64_t* numels) {
    std::vector<int32_t> small, large;
    split_small(nt, numels, &small, &large);
    int64_t best = 0;
    for (size_t a = 0; a < large.size(); a += arctopk::kMB) {
        int64_t cap = 0;
        for (size_t q = a; q < std::min(large.size(), a + (size_t)arctopk::kMB); ++q) {
            arctopk::MItem it{};
            it.n = std::max<int64_t>(1, numels[large[q]]);
            arctopk::ms_item_geometry(it);
            cap += it.cand_cap;
        }
        best = std::max(best, cap);
    }
    return best;
}

// the TopK / RandK select over every tensor: key_off = offsets[j] (0 without x), out_off = k_off[j];
// hashed: RandK keys of tensor j's seed; zero_x / fold / fold_g as ms_select's
static int sparse_select(const void* x, int x_bf16, int32_t nt, const int64_t* offsets, const int64_t* numels,
                         const int64_t* ks, const int64_t* k_off, bool hashed, uint64_t seed, int32_t* idx,
                         void* vals, arctopk::MWorkspace* ws, void* zero_x, int fold, const void* fold_g,
                         hipStream_t st);

extern "C" int64_t arctopk_sparse_workspace_bytes(int32_t nt, const int64_t* numels) {
    if (nt < 1 || !numels) return -(int64_t)ARCTOPK_EINVAL;
    for (int32_t j = 0; j < nt; ++j)
        if (numels[j] < 1 || numels[j] >= (1ll << 31)) return -(int64_t)ARCTOPK_EINVAL;
    return arctopk::ms_workspace_bytes(topk_cap_total(nt, numels));
}

extern "C" int arctopk_topk_select(const void* x, int32_t nt, const int64_t* offsets,
                                   const int64_t* numels, const int64_t* ks, const int64_t* k_off,
                                   int32_t* idx, void* vals, void* workspace, int32_t dtype,
                                   int32_t zero_selected, void* stream) {
    if (!x || !offsets || !numels || !ks || !k_off || !idx || !vals || !workspace || nt < 1)
        return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EINVAL;
    for (int32_t j = 0; j < nt; ++j)
        if (numels[j] < 1 || numels[j] >= (1ll << 31) || ks[j] < 1 || ks[j] > numels[j])
            return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    return sparse_select(x, dtype == ARCTOPK_BF16, nt, offsets, numels, ks, k_off, false, 0, idx, vals,
                         (arctopk::MWorkspace*)workspace, zero_selected ? const_cast<void*>(x) : nullptr, 0, nullptr, st);
}

// RandK's per-tensor key seed: splitmix64 of the call's seed and the tensor's place in the bucket
static uint32_t rk_tensor_seed(uint64_t seed, int32_t t) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(t + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)(z ^ (z >> 31));
}

static int sparse_select(const void* x, int x_bf16, int32_t nt, const int64_t* offsets, const int64_t* numels,
                         const int64_t* ks, const int64_t* k_off, bool hashed, uint64_t seed, int32_t* idx,
                         void* vals, arctopk::MWorkspace* ws, void* zero_x, int fold, const void* fold_g,
                         hipStream_t st) {
    std::vector<int32_t> small, large;
    split_small(nt, numels, &small, &large);
    const int64_t cap_total = topk_cap_total(nt, numels);
    for (int pass = 0; pass < 2; ++pass) {
        const std::vector<int32_t>& list = pass == 0 ? small : large;
        for (size_t a = 0; a < list.size(); a += arctopk::kMB) {
            arctopk::MBatch b;
            b.cnt = (int32_t)std::min(list.size() - a, (size_t)arctopk::kMB);
            int64_t maxn = 0, cap = 0;
            for (int i = 0; i < b.cnt; ++i) {
                const int j = list[a + i];
                arctopk::MItem& it = b.it[i];
                it.key_off = x ? offsets[j] : 0;
                it.n = numels[j];
                it.k = ks[j];
                it.out_off = k_off[j];
                it.slot_off = 0;
                arctopk::ms_item_geometry(it);
                it.hseed = hashed ? rk_tensor_seed(seed, j) : 0u;
                it.cand_off = cap;
                cap += it.cand_cap;
                maxn = std::max(maxn, numels[j]);
            }
            const int e = pass == 0
                ? arctopk::ms_select_small(b, x, x_bf16, idx, vals, zero_x, st, hashed, fold, fold_g)
                : arctopk::ms_select(b, maxn, nullptr, x, x_bf16, false, ws, cap_total, idx, vals, nullptr, zero_x, st,
                                     hashed, fold, fold_g);
            if (e) return e;
        }
    }
    return 0;
}

extern "C" int arctopk_randk_select(const void* x, int32_t nt, const int64_t* offsets, const int64_t* numels,
                                    const int64_t* ks, const int64_t* k_off, uint64_t seed, int32_t* idx,
                                    void* vals, void* workspace, int32_t dtype, int32_t zero_selected,
                                    void* stream) {
    if (!numels || !ks || !k_off || !idx || !workspace || nt < 1) return ARCTOPK_EINVAL;
    if (x ? (!offsets || !vals) : (vals != nullptr || zero_selected)) return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EINVAL;
    for (int32_t j = 0; j < nt; ++j)
        if (numels[j] < 1 || numels[j] >= (1ll << 31) || ks[j] < 1 || ks[j] > numels[j])
            return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    return sparse_select(x, dtype == ARCTOPK_BF16, nt, offsets, numels, ks, k_off, true, seed, idx, vals,
                         (arctopk::MWorkspace*)workspace, zero_selected ? const_cast<void*>(x) : nullptr, 0, nullptr, st);
}

extern "C" int arctopk_topk_select_ef14(const void* g, void* E, int32_t err_in, int32_t nt, const int64_t* offsets,
                                        const int64_t* numels, const int64_t* ks, const int64_t* k_off, int32_t* idx,
                                        void* vals, void* workspace, int32_t dtype, void* stream) {
    if (!g || !E || !offsets || !numels || !ks || !k_off || !idx || !vals || !workspace || nt < 1)
        return ARCTOPK_EINVAL;
    // the fold streams 16-B quads: fp32, every tensor 16-B aligned in both buffers and n % 4 == 0
    // (ARCTOPK_EINVAL otherwise: the caller folds first and calls arctopk_topk_select)
    if (dtype != ARCTOPK_F32 || (((uintptr_t)g | (uintptr_t)E) & 15)) return ARCTOPK_EINVAL;
    for (int32_t j = 0; j < nt; ++j)
        if (numels[j] < 1 || numels[j] >= (1ll << 31) || ks[j] < 1 || ks[j] > numels[j] || (numels[j] & 3) ||
            (offsets[j] & 3))
            return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    return sparse_select(E, 0, nt, offsets, numels, ks, k_off, false, 0, idx, vals, (arctopk::MWorkspace*)workspace,
                         E, err_in ? 1 : 2, g, st);
}

extern "C" int arctopk_randk_select_ef14(const void* g, void* E, int32_t err_in, int32_t nt, const int64_t* offsets,
                                         const int64_t* numels, const int64_t* ks, const int64_t* k_off,
                                         uint64_t seed, int32_t* idx, void* vals, void* workspace, int32_t dtype,
                                         void* stream) {
    if (!g || !E || !offsets || !numels || !ks || !k_off || !idx || !vals || !workspace || nt < 1)
        return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EINVAL;
    for (int32_t j = 0; j < nt; ++j)
        if (numels[j] < 1 || numels[j] >= (1ll << 31) || ks[j] < 1 || ks[j] > numels[j])
            return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    return sparse_select(g, dtype == ARCTOPK_BF16, nt, offsets, numels, ks, k_off, true, seed, idx, vals,
                         (arctopk::MWorkspace*)workspace, E, err_in ? 1 : 2, g, st);
}

extern "C" int arctopk_sparse_gather(const void* x, int32_t nt, const int64_t* offsets,
                                     const int64_t* ks, const int64_t* k_off, const int32_t* idx,
                                     void* vals, int32_t dtype, void* stream) {
    if (!x || !offsets || !ks || !k_off || !idx || !vals || nt < 1) return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EINVAL;
    for (int32_t first = 0; first < nt; first += kB) {
        SparseBatch b;
        int64_t maxn, maxk;
        const int cnt = std::min<int32_t>(kB, nt - first);
        int e = fill_batch(b, first, cnt, offsets, nullptr, ks, k_off, maxn, maxk);
        if (e) return e;
        if (dtype == ARCTOPK_BF16)
            hipLaunchKernelGGL(k_gather<arctopk::bf16_t>, dim3(grid_for(maxk, 2048), cnt), dim3(256), 0,
                               (hipStream_t)stream, b, static_cast<const arctopk::bf16_t*>(x), idx,
                               static_cast<arctopk::bf16_t*>(vals));
        else
            hipLaunchKernelGGL(k_gather<float>, dim3(grid_for(maxk, 2048), cnt), dim3(256), 0,
                               (hipStream_t)stream, b, static_cast<const float*>(x), idx, static_cast<float*>(vals));
        e = (int)hipGetLastError();
        if (e) return e;
    }
    return 0;
}

extern "C" int arctopk_sparse_residual(void* E, int32_t nt, const int64_t* offsets,
                                       const int64_t* ks, const int64_t* k_off, const int32_t* idx,
                                       const void* vals, int32_t ef, float decay, int32_t dtype,
                                       void* stream) {
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EINVAL;
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
        hipStream_t st = (hipStream_t)stream;
        using arctopk::bf16_t;
        if (dtype == ARCTOPK_BF16) {
            bf16_t* Eb = static_cast<bf16_t*>(E);
            const bf16_t* vb = static_cast<const bf16_t*>(vals);
            if (ef == ARCTOPK_EF14)
                hipLaunchKernelGGL((k_residual<bf16_t, ARCTOPK_EF14>), grid, dim3(256), 0, st, b, Eb, idx, vb, decay);
            else if (ef == ARCTOPK_EF21)
                hipLaunchKernelGGL((k_residual<bf16_t, ARCTOPK_EF21>), grid, dim3(256), 0, st, b, Eb, idx, vb, decay);
            else
                return ARCTOPK_EINVAL;
        } else {
            float* Ef = static_cast<float*>(E);
            const float* vf = static_cast<const float*>(vals);
            if (ef == ARCTOPK_EF14)
                hipLaunchKernelGGL((k_residual<float, ARCTOPK_EF14>), grid, dim3(256), 0, st, b, Ef, idx, vf, decay);
            else if (ef == ARCTOPK_EF21)
                hipLaunchKernelGGL((k_residual<float, ARCTOPK_EF21>), grid, dim3(256), 0, st, b, Ef, idx, vf, decay);
            else
                return ARCTOPK_EINVAL;
        }
        e = (int)hipGetLastError();
        if (e) return e;
    }
    return 0;
}

namespace {
template <typename T>
int sparse_decode_t(T* out, int64_t numel, int32_t nt, const int64_t* offsets, const int64_t* ks,
                    const int64_t* k_off, int64_t packed_len, const int32_t* idx, const T* vals,
                    int32_t nranks, int32_t world_size, int32_t accumulate, T* gerr, float decay,
                    hipStream_t st) {
    // TopK (accumulate 1) and RandK with ascending indices (accumulate 2): the first payload
    // writes the whole bucket, zeros included (k_scatter_first); the tensors tile the bucket in order
    bool tiled = accumulate != 0;
    for (int32_t i = 0; tiled && i < nt; ++i) {
        const int64_t end = i + 1 < nt ? offsets[i + 1] : numel;
        if (offsets[i] < 0 || end <= offsets[i] || end - offsets[i] >= (1ll << 31) || (i == 0 && offsets[0] != 0))
            tiled = false;
    }
    if (!tiled) {
        hipError_t he = hipMemsetAsync(out, 0, (size_t)numel * sizeof(T), st);
        if (he != hipSuccess) return (int)he;
    } else {
        std::vector<int64_t> numels(nt);
        for (int32_t i = 0; i < nt; ++i) numels[i] = (i + 1 < nt ? offsets[i + 1] : numel) - offsets[i];
        for (int32_t first = 0; first < nt; first += kB) {
            SparseBatch b;
            int64_t maxn, maxk;
            const int cnt = std::min<int32_t>(kB, nt - first);
            int e = fill_batch(b, first, cnt, offsets, numels.data(), ks, k_off, maxn, maxk);
            if (e) return e;
            const dim3 grid((unsigned)((maxn + kDecChunk - 1) / kDecChunk), cnt);
            if (accumulate == 2)
                hipLaunchKernelGGL((k_scatter_first<T, true>), grid, dim3(256), 0, st, b, out, idx, vals,
                                   (float)world_size);
            else
                hipLaunchKernelGGL((k_scatter_first<T, false>), grid, dim3(256), 0, st, b, out, idx, vals, 1.0f);
        }
    }
    const float wsf = (float)world_size;
    const int nr = accumulate == 1 ? nranks : 1;
    for (int q = tiled ? 1 : 0; q < nr; ++q) {
        for (int32_t first = 0; first < nt; first += kB) {
            SparseBatch b;
            int64_t maxn, maxk;
            const int cnt = std::min<int32_t>(kB, nt - first);
            int e = fill_batch(b, first, cnt, offsets, nullptr, ks, k_off, maxn, maxk);
            if (e) return e;
            dim3 grid(grid_for(maxk, 2048), cnt);
            const int32_t* iq = idx + (int64_t)q * packed_len;
            const T* vq = vals + (int64_t)q * packed_len;
            if (accumulate == 1 && q > 0)
                hipLaunchKernelGGL((k_scatter<T, 1>), grid, dim3(256), 0, st, b, out, iq, vq, wsf);
            else if (accumulate == 1)
                hipLaunchKernelGGL((k_scatter<T, 2>), grid, dim3(256), 0, st, b, out, iq, vq, wsf);
            else
                hipLaunchKernelGGL((k_scatter<T, 0>), grid, dim3(256), 0, st, b, out, iq, vq, wsf);
        }
    }
    // TopK's out /= ws (sparse_hook.py:293) is the identity at ws = 1 (x / 1 == x for every x)
    const bool div = accumulate == 1 && world_size > 1;
    if (div || gerr) {
        hipLaunchKernelGGL(k_div_gE<T>, dim3(grid_for(numel, 8192)), dim3(256), 0, st, out, gerr,
                           numel, wsf, div ? 1 : 0, decay);
    }
    return (int)hipGetLastError();
}
}  // namespace

extern "C" int arctopk_sparse_decode(void* out, int64_t numel, int32_t nt, const int64_t* offsets,
                                     const int64_t* ks, const int64_t* k_off, int64_t packed_len,
                                     const int32_t* idx, const void* vals, int32_t nranks,
                                     int32_t world_size, int32_t accumulate, void* gerr,
                                     float decay, int32_t dtype, void* stream) {
    if (!out || !offsets || !ks || !k_off || !idx || !vals || nt < 1 || nranks < 1 ||
        world_size < 1 || numel < 0 || accumulate < 0 || accumulate > 2)
        return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    using arctopk::bf16_t;
    if (dtype == ARCTOPK_BF16)
        return sparse_decode_t<bf16_t>(static_cast<bf16_t*>(out), numel, nt, offsets, ks, k_off, packed_len, idx,
                                       static_cast<const bf16_t*>(vals), nranks, world_size, accumulate,
                                       static_cast<bf16_t*>(gerr), decay, st);
    return sparse_decode_t<float>(static_cast<float*>(out), numel, nt, offsets, ks, k_off, packed_len, idx,
                                  static_cast<const float*>(vals), nranks, world_size, accumulate,
                                  static_cast<float*>(gerr), decay, st);
}
