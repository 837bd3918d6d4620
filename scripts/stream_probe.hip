// Encode-pattern ceiling probe (MI355X): EF14 encode reads G and E and writes E over a
// 16 x [2048, 2048] fp32 bucket, right after a decode-like full write of G (as in the hook's
// steady state).  Compares flat streaming (no sketch) with and without nontemporal hints
// against the library's k_encode, so the cost of the sketch structure is visible.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o scripts/stream_probe scripts/stream_probe.hip \
//         -Lallreducetopk_amd/lib -larctopk -Wl,-rpath,'$ORIGIN/../allreducetopk_amd/lib'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "arctopk.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4f ld(const v4f* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v4f* p, v4f v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// flat grid-stride: E := G + E (the encode's bytes without the sketch)
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_r2w1(const v4f* __restrict__ g, v4f* __restrict__ e, size_t n4) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
        v4f a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = min(base + (size_t)u * 256, n4 - 1);
            a[u] = ld<NTL>(g + i);
            b[u] = ld<NTL>(e + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n4) st<NTS>(e + i, a[u] + b[u]);
        }
    }
}

// contiguous chunk per block (row-tile-like ownership), E := G + E
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_r2w1_chunk(const v4f* __restrict__ g, v4f* __restrict__ e, size_t n4,
                                                    size_t per_block) {
    const size_t b0 = (size_t)blockIdx.x * per_block;
    const size_t b1 = min(n4, b0 + per_block);
    for (size_t base = b0 + threadIdx.x; base < b1; base += 256 * U) {
        v4f a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = min(base + (size_t)u * 256, b1 - 1);
            a[u] = ld<NTL>(g + i);
            b[u] = ld<NTL>(e + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < b1) st<NTS>(e + i, a[u] + b[u]);
        }
    }
}

// flat grid-stride: E := G + E and G := 0 (EF14 encode that also clears the bucket)
template <int U>
__global__ void __launch_bounds__(256) k_r2w2(v4f* __restrict__ g, v4f* __restrict__ e, size_t n4) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
        v4f a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = min(base + (size_t)u * 256, n4 - 1);
            a[u] = ld<true>(g + i);
            b[u] = ld<true>(e + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n4) {
                st<true>(e + i, a[u] + b[u]);
                st<true>(g + i, v4f{0.f, 0.f, 0.f, 0.f});
            }
        }
    }
}

template <bool NT>
__global__ void __launch_bounds__(256) k_zero(v4f* __restrict__ x, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        st<NT>(x + i, v4f{0.f, 0.f, 0.f, 0.f});
}

__global__ void __launch_bounds__(256) k_fill(v4f* __restrict__ x, size_t n4, float v) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        x[i] = v4f{v, v, v, v};
}

__global__ void __launch_bounds__(256) k_read(const v4f* __restrict__ x, size_t n4, float* out) {
    v4f acc = {0, 0, 0, 0};
    const size_t stride = (size_t)gridDim.x * 256 * 8;
    for (size_t base = (size_t)blockIdx.x * 256 * 8 + threadIdx.x; base < n4; base += stride) {
        v4f a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = x[min(base + (size_t)u * 256, n4 - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += a[u];
    }
    if (acc.x == 1234.5f) out[0] = acc.y;
}

int main() {
    const int T = 16, n = 2048, m = 2048;
    const size_t N = (size_t)T * n * m, n4 = N / 4;
    float *G, *E, *V, *S, *big, *out;
    CK(hipMalloc(&G, N * 4));
    CK(hipMalloc(&E, N * 4));
    CK(hipMalloc(&V, (size_t)T * m * 4 * 4));
    CK(hipMalloc(&S, (size_t)T * n * 4 * 4));
    CK(hipMalloc(&out, 64));
    const size_t nbig = 256ull << 20;  // 1 GiB, to evict the 256 MiB infinity cache
    CK(hipMalloc(&big, nbig * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (v4f*)G, n4, 0.5f);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (v4f*)E, n4, 0.25f);
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, (v4f*)V, (size_t)T * m, 0.01f);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (v4f*)big, nbig / 4, 0.f);
    CK(hipDeviceSynchronize());
    std::vector<int64_t> dims;
    std::vector<int32_t> nd(T, 2);
    for (int i = 0; i < T; ++i) { dims.push_back(n); dims.push_back(m); }
    arctopk_plan* plan = nullptr;
    int st_ = arctopk_plan_create(dims.data(), nd.data(), T, 4, 0.2, ARCTOPK_F32, 0, &plan);
    if (st_) { printf("plan_create %d\n", st_); return 1; }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // prelude: "decode" rewrite of G (as in the hook) or a 1 GiB flush
    auto timed = [&](const char* name, int prelude, auto launch, double bytes) {
        std::vector<float> ts;
        for (int r = 0; r < 15; ++r) {
            if (prelude == 1) hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (v4f*)G, n4, 0.5f);
            if (prelude == 2) hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (v4f*)big, nbig / 4, 0.f);
            (void)hipEventRecord(e0);
            launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r >= 3) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const float ms = ts[ts.size() / 2];
        printf("%-44s prelude %-6s %8.1f us  %7.0f GB/s\n", name, prelude == 0 ? "none" : prelude == 1 ? "G-fill" : "flush",
               ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    };
    const double enc_bytes = 12.0 * N;
    for (int pre = 0; pre < 3; ++pre) {
        timed("read G only (U8, 8/CU)", pre, [&] { hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, 0, (const v4f*)G, n4, out); }, 4.0 * N);
        for (int bpc : {4, 8, 16}) {
            char nm[96];
            snprintf(nm, sizeof nm, "flat R2W1 U4 %d/CU", bpc);
            timed(nm, pre, [&] { hipLaunchKernelGGL((k_r2w1<4, false, false>), dim3(256 * bpc), dim3(256), 0, 0, (const v4f*)G, (v4f*)E, n4); }, enc_bytes);
            snprintf(nm, sizeof nm, "flat R2W1 U4 %d/CU nt-load", bpc);
            timed(nm, pre, [&] { hipLaunchKernelGGL((k_r2w1<4, true, false>), dim3(256 * bpc), dim3(256), 0, 0, (const v4f*)G, (v4f*)E, n4); }, enc_bytes);
            snprintf(nm, sizeof nm, "flat R2W1 U4 %d/CU nt-store", bpc);
            timed(nm, pre, [&] { hipLaunchKernelGGL((k_r2w1<4, false, true>), dim3(256 * bpc), dim3(256), 0, 0, (const v4f*)G, (v4f*)E, n4); }, enc_bytes);
            snprintf(nm, sizeof nm, "flat R2W1 U4 %d/CU nt both", bpc);
            timed(nm, pre, [&] { hipLaunchKernelGGL((k_r2w1<4, true, true>), dim3(256 * bpc), dim3(256), 0, 0, (const v4f*)G, (v4f*)E, n4); }, enc_bytes);
        }
        for (size_t per : {16384ul, 65536ul}) {
            char nm[96];
            const int grid = (int)((n4 + per - 1) / per);
            snprintf(nm, sizeof nm, "chunk R2W1 U4 %zu f4/blk (grid %d)", per, grid);
            timed(nm, pre, [&] { hipLaunchKernelGGL((k_r2w1_chunk<4, false, false>), dim3(grid), dim3(256), 0, 0, (const v4f*)G, (v4f*)E, n4, per); }, enc_bytes);
            snprintf(nm, sizeof nm, "chunk R2W1 U4 %zu f4/blk nt both", per);
            timed(nm, pre, [&] { hipLaunchKernelGGL((k_r2w1_chunk<4, true, true>), dim3(grid), dim3(256), 0, 0, (const v4f*)G, (v4f*)E, n4, per); }, enc_bytes);
        }
        for (int bpc : {4, 8}) {
            char nm[96];
            snprintf(nm, sizeof nm, "flat R2W2 (E=G+E, G=0) nt %d/CU", bpc);
            timed(nm, pre, [&] { hipLaunchKernelGGL((k_r2w2<4>), dim3(256 * bpc), dim3(256), 0, 0, (v4f*)G, (v4f*)E, n4); }, 16.0 * N);
        }
        timed("zero G (decode-like) plain", pre, [&] { hipLaunchKernelGGL(k_zero<false>, dim3(2048), dim3(256), 0, 0, (v4f*)G, n4); }, 4.0 * N);
        timed("zero G (decode-like) nt", pre, [&] { hipLaunchKernelGGL(k_zero<true>, dim3(2048), dim3(256), 0, 0, (v4f*)G, n4); }, 4.0 * N);
        timed("library k_encode EF14", pre, [&] { arctopk_encode(plan, G, E, ARCTOPK_EF14, 1, V, S, 0); }, enc_bytes);
        timed("library k_encode noef (read G)", pre, [&] { arctopk_encode(plan, G, E, ARCTOPK_EF_NONE, 0, V, S, 0); }, 4.0 * N);
        timed("library k_encode EF21 (read G, E)", pre, [&] { arctopk_encode(plan, G, E, ARCTOPK_EF21, 1, V, S, 0); }, 8.0 * N);
    }
    arctopk_plan_destroy(plan);
    return 0;
}
