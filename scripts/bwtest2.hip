// Row-per-wave streaming probe: which part of the encode structure costs bandwidth.
// hipcc --offload-arch=gfx950 -O3 -o bwtest2 scripts/bwtest2.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int M = 2048, M4 = M / 4;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// MODE 0: loads + plain sum;  1: + 4 FMAs chains with register V + wave reduce
// 2: + V^T from LDS (staged per block);  3: mode 2 with 2 rows in flight per wave
template <int MODE, int ROWS_PER_BLOCK>
__global__ void __launch_bounds__(256) k_rows(const float* __restrict__ G, const float* __restrict__ V,
                                              float* __restrict__ out, int nrows) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row0 = blockIdx.x * ROWS_PER_BLOCK;
    if constexpr (MODE >= 2) {
        const float4* v4 = reinterpret_cast<const float4*>(V);
        for (int c = threadIdx.x; c < M; c += 256) {
            const float4 v = v4[c];
            lds[c] = v.x; lds[M + c] = v.y; lds[2 * M + c] = v.z; lds[3 * M + c] = v.w;
        }
        __syncthreads();
    }
    const float4* vt4 = reinterpret_cast<const float4*>(lds);
    float vr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) vr[i] = 0.001f * (i + lane);
    constexpr int RS = (MODE == 3) ? 2 : 1;
    for (int r = row0 + wave * RS; r < row0 + ROWS_PER_BLOCK && r < nrows; r += 4 * RS) {
        float4 x[RS][8];
#pragma unroll
        for (int q = 0; q < RS; ++q) {
            const float4* g4 = reinterpret_cast<const float4*>(G + (size_t)(r + q) * M);
#pragma unroll
            for (int u = 0; u < 8; ++u) x[q][u] = g4[u * 64 + lane];
        }
#pragma unroll
        for (int q = 0; q < RS; ++q) {
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int c = u * 64 + lane;
                if constexpr (MODE == 0) {
                    acc[0] += x[q][u].x + x[q][u].y + x[q][u].z + x[q][u].w;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        float4 v;
                        if constexpr (MODE == 1) v = make_float4(vr[4 * j], vr[4 * j + 1], vr[4 * j + 2], vr[4 * j + 3]);
                        else v = vt4[j * M4 + c];
                        acc[j] = fmaf(x[q][u].x, v.x, acc[j]);
                        acc[j] = fmaf(x[q][u].y, v.y, acc[j]);
                        acc[j] = fmaf(x[q][u].z, v.z, acc[j]);
                        acc[j] = fmaf(x[q][u].w, v.w, acc[j]);
                    }
                }
            }
            if constexpr (MODE == 0) {
                if (acc[0] == 1234.5f) out[r + q] = acc[0];
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = wave_sum(acc[j]);
                if (lane < 4) out[(size_t)(r + q) * 4 + lane] = lane == 0 ? acc[0] : lane == 1 ? acc[1] : lane == 2 ? acc[2] : acc[3];
            }
        }
    }
}

template <typename F>
float timeit(F f, hipEvent_t e0, hipEvent_t e1) {
    std::vector<float> ts;
    for (int r = 0; r < 12; ++r) {
        (void)hipEventRecord(e0);
        f();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

template <int MODE, int RPB>
void run(const char* name, const float* G, const float* V, float* out, int nrows, hipEvent_t e0, hipEvent_t e1) {
    const int grid = (nrows + RPB - 1) / RPB;
    const size_t lds = MODE >= 2 ? M * 4 * 4 : 0;
    float t = timeit([&] { hipLaunchKernelGGL((k_rows<MODE, RPB>), dim3(grid), dim3(256), lds, 0, G, V, out, nrows); }, e0, e1);
    printf("%-28s rows/block %3d grid %5d: %7.1f us  %6.0f GB/s\n", name, RPB, grid, t * 1e3,
           (double)nrows * M * 4 / (t * 1e-3) / 1e9);
}

int main() {
    const int nrows = 32768;  // 256 MiB
    float *G, *V, *out;
    CK(hipMalloc(&G, (size_t)nrows * M * 4));
    CK(hipMalloc(&V, M * 4 * 4));
    CK(hipMalloc(&out, (size_t)nrows * 16));
    std::vector<float> h((size_t)nrows * M);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.001f - 0.5f;
    CK(hipMemcpy(G, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(V, h.data(), M * 16, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    run<0, 32>("plain sum", G, V, out, nrows, e0, e1);
    run<0, 8>("plain sum", G, V, out, nrows, e0, e1);
    run<1, 32>("fma regV + reduce", G, V, out, nrows, e0, e1);
    run<1, 8>("fma regV + reduce", G, V, out, nrows, e0, e1);
    run<2, 32>("fma ldsV + reduce", G, V, out, nrows, e0, e1);
    run<2, 64>("fma ldsV + reduce", G, V, out, nrows, e0, e1);
    run<2, 128>("fma ldsV + reduce", G, V, out, nrows, e0, e1);
    run<3, 32>("ldsV, 2 rows in flight", G, V, out, nrows, e0, e1);
    run<3, 64>("ldsV, 2 rows in flight", G, V, out, nrows, e0, e1);
    run<3, 128>("ldsV, 2 rows in flight", G, V, out, nrows, e0, e1);
    return 0;
}
