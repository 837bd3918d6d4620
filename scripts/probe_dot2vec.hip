// probe (compile-only, `hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S`): bit_cast of ext_vector elements
// to __bf16 x2 feeding fdot2 -- k_elem loads one dword and feeds it to all four dot2 (ROCm 7.2 clang);
// k_scalar, the words through scalars, is lowered correctly
#include <hip/hip_runtime.h>
#include <cstdint>
typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u4_t __attribute__((ext_vector_type(4)));
__global__ void k_elem(const u4_t* a, const u4_t* b, float* out) {
    const u4_t x = a[threadIdx.x], v = b[threadIdx.x];
    float acc = 0.f;
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, x.x), __builtin_bit_cast(bf2_t, v.x), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, x.y), __builtin_bit_cast(bf2_t, v.y), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, x.z), __builtin_bit_cast(bf2_t, v.z), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, x.w), __builtin_bit_cast(bf2_t, v.w), acc, false);
    out[threadIdx.x] = acc;
}
__device__ __forceinline__ bf2_t word_bf2(u4_t q, int i) {
    const uint32_t w = i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w;
    return __builtin_bit_cast(bf2_t, w);
}
__global__ void k_scalar(const u4_t* a, const u4_t* b, float* out) {
    const u4_t x = a[threadIdx.x], v = b[threadIdx.x];
    uint32_t xw[4] = {x.x, x.y, x.z, x.w}, vw[4] = {v.x, v.y, v.z, v.w};
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, xw[i]), __builtin_bit_cast(bf2_t, vw[i]), acc, false);
    out[threadIdx.x] = acc;
}
