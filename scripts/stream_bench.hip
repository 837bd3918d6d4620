// HBM stream calibration on one MI355X: what a plain streaming kernel reaches for the
// read/write mixes of the codec's phases (encode EF14: read G, E, write E in place).
//   hipcc --offload-arch=gfx950 -O3 scripts/stream_bench.hip -o scripts/stream_bench
//   ./scripts/stream_bench [MiB per array]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

template <int U>
__global__ void __launch_bounds__(256) k_read(const float4* __restrict__ a, size_t n4, float* out) {
    float acc = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = (i + u * 256 < n4) ? a[i + u * 256] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 12345.678f) out[0] = acc;
}

template <int U>
__global__ void __launch_bounds__(256) k_copy(const float4* __restrict__ a, float4* __restrict__ c, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + u * 256 < n4) v[u] = a[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + u * 256 < n4) c[i + u * 256] = v[u];
    }
}

// b = a + b (in place: EF14's E := G + E)
template <int U>
__global__ void __launch_bounds__(256) k_addip(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256 * U) {
        float4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) {
                x[u] = a[i + u * 256];
                y[u] = b[i + u * 256];
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4)
                b[i + u * 256] = make_float4(x[u].x + y[u].x, x[u].y + y[u].y, x[u].z + y[u].z, x[u].w + y[u].w);
    }
}

// b = a + b with nontemporal stores
template <int U>
__global__ void __launch_bounds__(256) k_addip_nt(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256 * U) {
        float4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) {
                x[u] = a[i + u * 256];
                y[u] = b[i + u * 256];
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) {
                float4 r = make_float4(x[u].x + y[u].x, x[u].y + y[u].y, x[u].z + y[u].z, x[u].w + y[u].w);
                __builtin_nontemporal_store(r.x, &b[i + u * 256].x);
                __builtin_nontemporal_store(r.y, &b[i + u * 256].y);
                __builtin_nontemporal_store(r.z, &b[i + u * 256].z);
                __builtin_nontemporal_store(r.w, &b[i + u * 256].w);
            }
    }
}

template <typename F>
float time_it(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / reps;
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? (size_t)std::atoll(argv[1]) : 256;
    const size_t n = mib << 18;  // floats
    const size_t n4 = n / 4;
    float *a, *b, *c, *out;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&c, n * 4));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(a, 0, n * 4));
    CK(hipMemset(b, 0, n * 4));
    CK(hipMemset(c, 0, n * 4));
    const double bytes = (double)n * 4;
    const int grids[] = {1024, 2048, 4096, 8192, 16384, 0};
    for (int gi = 0; gi < 6; ++gi) {
        const unsigned g4 = grids[gi] ? grids[gi] : (unsigned)((n4 + 1023) / 1024);
        const unsigned g1 = grids[gi] ? grids[gi] : (unsigned)((n4 + 255) / 256);
        const float tr4 = time_it([&] { hipLaunchKernelGGL(k_read<4>, dim3(g4), dim3(256), 0, 0, (const float4*)a, n4, out); }, 20);
        const float tc4 = time_it([&] { hipLaunchKernelGGL(k_copy<4>, dim3(g4), dim3(256), 0, 0, (const float4*)a, (float4*)c, n4); }, 20);
        const float ta1 = time_it([&] { hipLaunchKernelGGL(k_addip<1>, dim3(g1), dim3(256), 0, 0, (const float4*)a, (float4*)b, n4); }, 20);
        const float ta2 = time_it([&] { hipLaunchKernelGGL(k_addip<2>, dim3(g4), dim3(256), 0, 0, (const float4*)a, (float4*)b, n4); }, 20);
        const float ta4 = time_it([&] { hipLaunchKernelGGL(k_addip<4>, dim3(g4), dim3(256), 0, 0, (const float4*)a, (float4*)b, n4); }, 20);
        const float tn4 = time_it([&] { hipLaunchKernelGGL(k_addip_nt<4>, dim3(g4), dim3(256), 0, 0, (const float4*)a, (float4*)b, n4); }, 20);
        std::printf("grid %6u: read %.0f GB/s  copy %.0f  addip(U1) %.0f  addip(U2) %.0f  addip(U4) %.0f  addip_nt(U4) %.0f"
                    "   [addip U4 %.1f us for %zu MiB x3]\n",
                    g4, bytes / tr4 / 1e6, 2 * bytes / tc4 / 1e6, 3 * bytes / ta1 / 1e6, 3 * bytes / ta2 / 1e6,
                    3 * bytes / ta4 / 1e6, 3 * bytes / tn4 / 1e6, ta4 * 1e3, mib);
    }
    return 0;
}
