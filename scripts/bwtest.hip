// Standalone HBM bandwidth probe for MI355X: which streaming shapes reach what GB/s.
// hipcc --offload-arch=gfx950 -O3 -o bwtest scripts/bwtest.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// grid-stride read, U independent float4 loads per iteration
template <int U>
__global__ void __launch_bounds__(256) k_read(const float4* __restrict__ x, size_t n4, float* out) {
    float acc = 0.f;
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            v[u] = i < n4 ? x[i] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 12345.f) out[0] = acc;
}

// contiguous chunk per block (no grid stride): chunk = 256*U*iters float4
template <int U>
__global__ void __launch_bounds__(256) k_read_chunk(const float4* __restrict__ x, size_t n4, int iters, float* out) {
    float acc = 0.f;
    size_t base = (size_t)blockIdx.x * 256 * U * iters + threadIdx.x;
    for (int it = 0; it < iters; ++it, base += 256 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            v[u] = i < n4 ? x[i] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 12345.f) out[0] = acc;
}

template <int U>
__global__ void __launch_bounds__(256) k_add(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
        float4 va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < n4) { va[u] = a[i]; vb[u] = b[i]; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < n4) { float4 r = va[u]; r.x += vb[u].x; r.y += vb[u].y; r.z += vb[u].z; r.w += vb[u].w; b[i] = r; }
        }
    }
}

template <int U>
__global__ void __launch_bounds__(256) k_write(float4* __restrict__ b, size_t n4) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            if (i < n4) b[i] = make_float4(0, 0, 0, 0);
        }
    }
}

// nontemporal read (global_load ... nt)
template <int U>
__global__ void __launch_bounds__(256) k_read_nt(const float4* __restrict__ x, size_t n4, float* out) {
    float acc = 0.f;
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * 256;
            typedef float v4f __attribute__((ext_vector_type(4)));
            if (i < n4) {
                v4f t = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(x) + i);
                v[u] = make_float4(t.x, t.y, t.z, t.w);
            } else {
                v[u] = make_float4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 12345.f) out[0] = acc;
}

template <typename F>
float timeit(F f, hipEvent_t e0, hipEvent_t e1) {
    std::vector<float> ts;
    for (int r = 0; r < 12; ++r) {
        hipEventRecord(e0);
        f();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const size_t n = 64ull << 20;  // 64M floats = 256 MiB
    const size_t n4 = n / 4;
    float4 *a, *b, *c;
    float* out;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&c, n * 4));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 0, n * 4));
    CK(hipMemset(b, 0, n * 4));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double GB = 1e9;
    for (int bpc : {1, 2, 4, 8, 16}) {
        int grid = 256 * bpc;
        float t1 = timeit([&] { hipLaunchKernelGGL(k_read<1>, dim3(grid), dim3(256), 0, 0, a, n4, out); }, e0, e1);
        float t4 = timeit([&] { hipLaunchKernelGGL(k_read<4>, dim3(grid), dim3(256), 0, 0, a, n4, out); }, e0, e1);
        float t8 = timeit([&] { hipLaunchKernelGGL(k_read<8>, dim3(grid), dim3(256), 0, 0, a, n4, out); }, e0, e1);
        float tn = timeit([&] { hipLaunchKernelGGL(k_read_nt<8>, dim3(grid), dim3(256), 0, 0, a, n4, out); }, e0, e1);
        float ta = timeit([&] { hipLaunchKernelGGL(k_add<4>, dim3(grid), dim3(256), 0, 0, a, b, n4); }, e0, e1);
        float tw = timeit([&] { hipLaunchKernelGGL(k_write<4>, dim3(grid), dim3(256), 0, 0, b, n4); }, e0, e1);
        printf("blocks/CU %2d: read U1 %6.0f  U4 %6.0f  U8 %6.0f  U8nt %6.0f | add(R2W1) %6.0f | write %6.0f GB/s\n", bpc,
               n * 4 / (t1 * 1e-3) / GB, n * 4 / (t4 * 1e-3) / GB, n * 4 / (t8 * 1e-3) / GB, n * 4 / (tn * 1e-3) / GB,
               n * 12 / (ta * 1e-3) / GB, n * 4 / (tw * 1e-3) / GB);
    }
    for (int iters : {1, 2, 4, 8, 16, 32}) {
        size_t per_block = 256ull * 8 * iters;
        int grid = (int)((n4 + per_block - 1) / per_block);
        float t = timeit([&] { hipLaunchKernelGGL(k_read_chunk<8>, dim3(grid), dim3(256), 0, 0, a, n4, iters, out); }, e0, e1);
        printf("read chunk U8 iters %2d (grid %6d): %6.0f GB/s\n", iters, grid, n * 4 / (t * 1e-3) / GB);
    }
    // 1 GiB read to defeat the 256 MiB infinity cache
    float4* big;
    const size_t nb = 256ull << 20;
    CK(hipMalloc(&big, nb * 4));
    CK(hipMemset(big, 0, nb * 4));
    for (int bpc : {2, 4, 8}) {
        float t = timeit([&] { hipLaunchKernelGGL(k_read<8>, dim3(256 * bpc), dim3(256), 0, 0, big, nb / 4, out); }, e0, e1);
        printf("1 GiB read U8 blocks/CU %d: %6.0f GB/s\n", bpc, nb * 4 / (t * 1e-3) / GB);
    }
    return 0;
}
