// HBM stream calibration on one MI355X: what a plain streaming kernel reaches for the
// read/write mixes of the codec's phases (encode EF14: read G, E, write E in place).
//   hipcc --offload-arch=gfx950 -O3 scripts/stream_bench.hip -o scripts/stream_bench
//   ./scripts/stream_bench [MiB per array] [sets]
//
// Two regimes per kernel: "warm" repeats the kernel on ONE set of arrays (what earlier rounds
// quoted: 2-3 x 256 MiB fit the 256 MB Infinity Cache (MALL) in part, so repeats find some of
// their lines there), and "cold" cycles over `sets` (default 4) disjoint sets of arrays, as the
// bench's four buckets do, so no kernel finds its data in the MALL.  The row-wave kernels stream
// the in-place add in the encode's own shape: 16 tensors of 2048 rows of 8 KiB, one wave per row
// step (64 lanes x 4 x 16 B), tiles of rows interleaved across blocks as the encode plan lays
// them out (k_encode's ENC_ROW_VEC walk without the sketch).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_nt(const float4* p) {
    const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(float4* p, float4 v) {
    __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(p));
}

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

// b = a + b in place (EF14's E := G + E), nontemporal loads and stores, flat grid-stride
template <int U>
__global__ void __launch_bounds__(256) k_addip_nt(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256 * U) {
        float4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + u * 256 < n4 ? i + u * 256 : n4 - 1;
            x[u] = ld_nt(a + j);
            y[u] = ld_nt(b + j);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4)
                st_nt(b + i + u * 256, make_float4(x[u].x + y[u].x, x[u].y + y[u].y, x[u].z + y[u].z, x[u].w + y[u].w));
    }
}

// the encode's shape: T tensors of R rows x 2048 floats; block = one tile (interleaved rows
// ti, ti + ntiles, ... of one tensor), wave q takes the tile's rows q, q + 4, ...; a row is 2
// steps of 64 lanes x U units of 16 B; the next step's loads issue before the current's stores
template <int U>
__global__ void __launch_bounds__(256) k_rows(const float4* __restrict__ a, float4* __restrict__ b, int rows,
                                             int ntiles) {
    constexpr int MU = 512;  // 16-B units per row (2048 floats)
    const int t = blockIdx.x / ntiles, ti = blockIdx.x % ntiles;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nr = (rows - ti + ntiles - 1) / ntiles;
    const size_t base = (size_t)t * rows * MU;
    for (int q = wave; q < nr; q += 4) {
        const size_t row = base + (size_t)(ti + q * ntiles) * MU;
        for (int st = 0; st < MU / (64 * U); ++st) {
            float4 x[U], y[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t j = row + st * 64 * U + u * 64 + lane;
                x[u] = ld_nt(a + j);
                y[u] = ld_nt(b + j);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t j = row + st * 64 * U + u * 64 + lane;
                st_nt(b + j, make_float4(x[u].x + y[u].x, x[u].y + y[u].y, x[u].z + y[u].z, x[u].w + y[u].w));
            }
        }
    }
}

// rows in sweep order: wave w of the grid takes rows w, w + W, w + 2 W, ... (W = all waves of
// the grid), so the waves in flight walk one contiguous window of rows, as the flat kernel does
template <int U>
__global__ void __launch_bounds__(256) k_rows_sweep(const float4* __restrict__ a, float4* __restrict__ b,
                                                   int total_rows) {
    constexpr int MU = 512;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int W = gridDim.x * 4;
    for (int r = blockIdx.x * 4 + wave; r < total_rows; r += W) {
        const size_t row = (size_t)r * MU;
        for (int st = 0; st < MU / (64 * U); ++st) {
            float4 x[U], y[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t j = row + st * 64 * U + u * 64 + lane;
                x[u] = ld_nt(a + j);
                y[u] = ld_nt(b + j);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t j = row + st * 64 * U + u * 64 + lane;
                st_nt(b + j, make_float4(x[u].x + y[u].x, x[u].y + y[u].y, x[u].z + y[u].z, x[u].w + y[u].w));
            }
        }
    }
}

// the same sweep with each wave's U loads of a step spread over the row (unit u of lane l at
// quad u * MU / U + st * 64 + l: 1 KiB pieces 2 KiB apart) instead of one contiguous 4 KiB
// piece -- the flat kernel's per-wave pattern (its waves' pieces are 4 KiB apart)
template <int U>
__global__ void __launch_bounds__(256) k_rows_sweep_il(const float4* __restrict__ a, float4* __restrict__ b,
                                                      int total_rows) {
    constexpr int MU = 512;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int W = gridDim.x * 4;
    for (int r = blockIdx.x * 4 + wave; r < total_rows; r += W) {
        const size_t row = (size_t)r * MU;
        for (int st = 0; st < MU / (64 * U); ++st) {
            float4 x[U], y[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t j = row + u * (MU / U) + st * 64 + lane;
                x[u] = ld_nt(a + j);
                y[u] = ld_nt(b + j);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t j = row + u * (MU / U) + st * 64 + lane;
                st_nt(b + j, make_float4(x[u].x + y[u].x, x[u].y + y[u].y, x[u].z + y[u].z, x[u].w + y[u].w));
            }
        }
    }
}

template <typename F>
float time_it(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f(0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) f(i);
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
    const int sets = argc > 2 ? std::atoi(argv[2]) : 4;
    const size_t n = mib << 18;  // floats per array
    const size_t n4 = n / 4;
    std::vector<float*> A(sets), B(sets);
    for (int s = 0; s < sets; ++s) {
        CK(hipMalloc(&A[s], n * 4));
        CK(hipMalloc(&B[s], n * 4));
        CK(hipMemset(A[s], 0, n * 4));
        CK(hipMemset(B[s], 0, n * 4));
    }
    float* out;
    CK(hipMalloc(&out, 4));
    const double bytes = (double)n * 4;
    const int reps = 24;
    std::printf("%zu MiB per array, %d sets (cold: every launch on the next set)\n", mib, sets);
    for (int cold = 0; cold < 2; ++cold) {
        auto pick = [&](int i) { return cold ? i % sets : 0; };
        for (unsigned g : {1024u, 2048u, 4096u, 8192u, 16384u}) {
            const float tr = time_it([&](int i) {
                hipLaunchKernelGGL(k_read<4>, dim3(g), dim3(256), 0, 0, (const float4*)A[pick(i)], n4, out); }, reps);
            const float ta = time_it([&](int i) {
                hipLaunchKernelGGL(k_addip_nt<4>, dim3(g), dim3(256), 0, 0, (const float4*)A[pick(i)],
                                   (float4*)B[pick(i)], n4); }, reps);
            std::printf("%s grid %6u: read %5.0f GB/s   in-place add (nt) %5.0f GB/s  %6.1f us\n",
                        cold ? "cold" : "warm", g, bytes / tr / 1e6, 3 * bytes / ta / 1e6, ta * 1e3);
        }
        if (mib == 256) {  // the encode's row shape: 16 x 2048 rows of 8 KiB
            for (int g : {1280, 2048, 2560, 4096, 8192}) {
                const float tw = time_it([&](int i) {
                    hipLaunchKernelGGL(k_rows_sweep<4>, dim3(g), dim3(256), 0, 0, (const float4*)A[pick(i)],
                                       (float4*)B[pick(i)], 16 * 2048); }, reps);
                std::printf("%s rows in sweep order, %5d blocks: in-place add (nt) %5.0f GB/s  %6.1f us\n",
                            cold ? "cold" : "warm", g, 3 * bytes / tw / 1e6, tw * 1e3);
                const float ti = time_it([&](int i) {
                    hipLaunchKernelGGL(k_rows_sweep_il<4>, dim3(g), dim3(256), 0, 0, (const float4*)A[pick(i)],
                                       (float4*)B[pick(i)], 16 * 2048); }, reps);
                std::printf("%s rows in sweep order, spread units, %5d blocks: in-place add (nt) %5.0f GB/s  %6.1f us\n",
                            cold ? "cold" : "warm", g, 3 * bytes / ti / 1e6, ti * 1e3);
            }
            for (int ntiles : {64, 80, 128, 160, 256, 512}) {
                const float tw = time_it([&](int i) {
                    hipLaunchKernelGGL(k_rows<4>, dim3(16 * ntiles), dim3(256), 0, 0, (const float4*)A[pick(i)],
                                       (float4*)B[pick(i)], 2048, ntiles); }, reps);
                std::printf("%s rows, %4d tiles per tensor (%5d blocks): in-place add (nt) %5.0f GB/s  %6.1f us\n",
                            cold ? "cold" : "warm", ntiles, 16 * ntiles, 3 * bytes / tw / 1e6, tw * 1e3);
            }
        }
    }
    return 0;
}
