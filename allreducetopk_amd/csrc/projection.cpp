// Host-side projections: the exact values of the reference's per-tensor
// torch.randn(m, r, dtype=...) on CPU (group_topk_hook_no_reshape.py:49, :79) after
// torch.manual_seed(seed) (:255), one native call per bucket (outside the GIL) instead
// of one torch call per tensor.
//
// After manual_seed torch's CPU generator is mt19937 (init_genrand, low 32 bits of the
// seed) with no cached normal sample.  torch.randn of n values, per tensor:
//  * n >= 16 (contiguous): normal_fill -- one uniform per element (float: (x & 0xFFFFFF)
//    * 2^-24; bf16: (x & 0xFF) / 256), then per block of 16 and j < 8, with
//    u1 = 1 - u[j], u2 = u[j + 8]: radius = sqrt(-2 * log(u1)), theta = 2*pi*u2 (formed in
//    double, narrowed), out[j] = radius * cos(theta), out[j + 8] = radius * sin(theta); if
//    n % 16 != 0 the last 16 values are recomputed from 16 fresh uniforms.
//    float: torch's AVX2 kernel (Cephes log / sincos polynomials in float, theta = float(2 pi)
//    * u2; restated below); projections.py checks this routine against the running torch
//    once per process before using it.  bf16: the scalar kernel, every BFloat16 operation
//    computed in float (libm) and rounded to bf16 (RNE); with 8-bit uniforms each output
//    is a function of (u[j], u[j+8]) only: two 256 x 256 tables.  Both end in
//    "* std + mean" with std 1, mean 0, which turns -0 into +0.
//  * n < 16: at::normal_distribution<double> per element -- Box-Muller on two 53-bit
//    uniforms (random64 = first draw << 32 | second), r = sqrt(-2 log1p(-u2)),
//    theta = 2 pi u1; returns r cos(theta) and caches r sin(theta) in the generator for
//    the next such element (also across tensors); narrowed to the dtype (bf16 via float).
// Pinned bit for bit against torch by tests/test_host_logic.py.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include <immintrin.h>

#include <hip/hip_runtime.h>

#include "arctopk.h"

namespace {

uint16_t bf16_bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7FFFFFFFu) > 0x7F800000u) return 0x7FC0u;
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
float bf16_val(uint16_t b) {
    const uint32_t u = (uint32_t)b << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
float rb(float f) { return bf16_val(bf16_bits(f)); }  // round to bf16

constexpr double kPi = 3.14159265358979323846;

uint16_t g_cos[256 * 256], g_sin[256 * 256];
std::once_flag g_once;

void build_tables() {
    float radius[256], c[256], s[256];
    for (int k = 0; k < 256; ++k) {
        const float u = rb((float)k / 256.0f);
        const float u1 = rb(1.0f - u);
        const float lg = rb(std::log(u1));
        radius[k] = rb(std::sqrt(rb(-2.0f * lg)));
        const float theta = rb((float)(2.0 * kPi * (double)u));
        c[k] = rb(std::cos(theta));
        s[k] = rb(std::sin(theta));
    }
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b) {
            g_cos[a * 256 + b] = bf16_bits(rb(radius[a] * c[b]) + 0.0f);  // "* std + mean"
            g_sin[a * 256 + b] = bf16_bits(rb(radius[a] * s[b]) + 0.0f);
        }
}

// std::mt19937 as torch's CPU generator (seeded by init_genrand with the low 32 bits)
struct MT {
    uint32_t st[624];
    int i = 624;
    explicit MT(uint32_t seed) {
        st[0] = seed;
        for (int k = 1; k < 624; ++k) st[k] = 1812433253u * (st[k - 1] ^ (st[k - 1] >> 30)) + (uint32_t)k;
    }
    static uint32_t mix(uint32_t a, uint32_t b, uint32_t c) {
        const uint32_t y = (a & 0x80000000u) | (b & 0x7FFFFFFFu);
        return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
    }
    void twist() {
        int k = 0;
        for (; k < 624 - 397; ++k) st[k] = mix(st[k], st[k + 1], st[k + 397]);
        for (; k < 623; ++k) st[k] = mix(st[k], st[k + 1], st[k + 397 - 624]);
        st[623] = mix(st[623], st[0], st[396]);
        i = 0;
    }
    uint32_t next() {
        if (i >= 624) twist();
        uint32_t y = st[i++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9D2C5680u;
        y ^= (y << 15) & 0xEFC60000u;
        y ^= y >> 18;
        return y;
    }
};

// torch's CPUGeneratorImpl stream right after manual_seed
struct Gen {
    MT mt;
    bool has_dn = false;  // cached second Box-Muller value of normal_distribution<double>
    double dn = 0.0;
    explicit Gen(uint64_t seed) : mt((uint32_t)(seed & 0xFFFFFFFFu)) {}
    uint64_t random64() {
        const uint64_t hi = mt.next();
        const uint64_t lo = mt.next();
        return (hi << 32) | lo;
    }
    float uniform_f() { return (float)(mt.next() & 0xFFFFFFu) * (1.0f / 16777216.0f); }
    double normal_d() {
        if (has_dn) {
            has_dn = false;
            return dn * 1.0 + 0.0;  // transformation::normal(x, mean 0, std 1)
        }
        const double u1 = (double)(random64() & ((1ull << 53) - 1)) * (1.0 / 9007199254740992.0);
        const double u2 = (double)(random64() & ((1ull << 53) - 1)) * (1.0 / 9007199254740992.0);
        const double r = std::sqrt(-2.0 * std::log1p(-u2));
        const double theta = 2.0 * kPi * u1;
        dn = r * std::sin(theta);
        has_dn = true;
        return r * std::cos(theta) * 1.0 + 0.0;
    }
};

// torch's AVX2 normal_fill (the kernel its CPU dispatch runs for float, also on AVX512
// hosts) transforms with the Cephes-derived vector routines log256_ps / sincos256_ps of
// ATen/native/cpu/avx_mathfun.h, op for op in float -- including the multiply-adds the
// compiler fuses from those intrinsics (-mfma, default contraction): each mul whose only
// use is an add, in statement order.  Scalar restatements of the two (bit-identical on 4 M
// draws, tests/test_host_logic.py).
float bits_f(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
uint32_t f_bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

__attribute__((target("fma"))) float cephes_log(float x) {  // x in (0, 1]
    x = std::fmax(x, bits_f(0x00800000u));
    int32_t imm0 = (int32_t)(f_bits(x) >> 23);
    x = bits_f((f_bits(x) & ~0x7f800000u) | f_bits(0.5f));
    imm0 -= 0x7f;
    float e = (float)imm0;
    e = e + 1.0f;
    const bool mask = x < (float)0.707106781186547524;
    const float tmp0 = mask ? x : 0.0f;
    x = x - 1.0f;
    e = e - (mask ? 1.0f : 0.0f);
    x = x + tmp0;
    const float z = x * x;
    float y = (float)7.0376836292E-2;
    y = __builtin_fmaf(y, x, (float)-1.1514610310E-1);
    y = __builtin_fmaf(y, x, (float)1.1676998740E-1);
    y = __builtin_fmaf(y, x, (float)-1.2420140846E-1);
    y = __builtin_fmaf(y, x, (float)1.4249322787E-1);
    y = __builtin_fmaf(y, x, (float)-1.6668057665E-1);
    y = __builtin_fmaf(y, x, (float)2.0000714765E-1);
    y = __builtin_fmaf(y, x, (float)-2.4999993993E-1);
    y = __builtin_fmaf(y, x, (float)3.3333331174E-1);
    y = y * x;
    y = __builtin_fmaf(y, z, e * (float)-2.12194440e-4);
    y = __builtin_fmaf(-z, 0.5f, y);
    x = x + y;
    x = __builtin_fmaf(e, (float)0.693359375, x);
    return x;
}

__attribute__((target("fma"))) void cephes_sincos(float x, float* s, float* c) {  // x >= 0
    uint32_t sign_sin = f_bits(x) & 0x80000000u;
    x = bits_f(f_bits(x) & 0x7FFFFFFFu);
    float y = x * (float)1.27323954473516;
    int32_t j = (int32_t)y;  // truncation (cvttps)
    j = (j + 1) & ~1;
    y = (float)j;
    const uint32_t swap_sin = ((uint32_t)j & 4u) << 29;
    const bool poly = (j & 2) == 0;
    x = __builtin_fmaf(y, -0.78515625f, x);
    x = __builtin_fmaf(y, -2.4187564849853515625e-4f, x);
    x = __builtin_fmaf(y, (float)-3.77489497744594108e-8, x);
    const uint32_t sign_cos = (~(uint32_t)(j - 2) & 4u) << 29;
    sign_sin ^= swap_sin;
    const float z = x * x;
    float yc = (float)2.443315711809948E-005;
    yc = __builtin_fmaf(yc, z, (float)-1.388731625493765E-003);
    yc = __builtin_fmaf(yc, z, (float)4.166664568298827E-002);
    yc = yc * z;
    yc = __builtin_fmaf(yc, z, -(z * 0.5f));
    yc = yc + 1.0f;
    float ys = (float)-1.9515295891E-4;
    ys = __builtin_fmaf(ys, z, (float)8.3321608736E-3);
    ys = __builtin_fmaf(ys, z, (float)-1.6666654611E-1);
    ys = ys * z;
    ys = __builtin_fmaf(ys, x, x);
    const float ysin2 = poly ? ys : 0.0f;
    const float ysin1 = poly ? 0.0f : yc;
    ys = ys - ysin2;
    yc = yc - ysin1;
    *s = bits_f(f_bits(ysin1 + ysin2) ^ sign_sin);
    *c = bits_f(f_bits(yc + ys) ^ sign_cos);
}

__attribute__((target("fma"))) void f32_block16(float* d) {
    const float two_pi = (float)(2.0 * kPi);
    for (int j = 0; j < 8; ++j) {
        const float u1 = 1.0f - d[j];
        const float u2 = d[j + 8];
        const float radius = std::sqrt(-2.0f * cephes_log(u1));
        float sn, cs;
        cephes_sincos(two_pi * u2, &sn, &cs);
        d[j] = radius * cs + 0.0f;  // fmadd(n, std = 1, mean = 0): -0 becomes +0
        d[j + 8] = radius * sn + 0.0f;
    }
}

// The same block on 8 lanes at once (AVX2 + FMA hosts): torch's operation sequence with
// the fused multiply-adds written out.
__attribute__((target("avx2,fma"))) void f32_block16_avx2(float* d) {
    const __m256 one = _mm256_set1_ps(1.0f);
    const __m256 u1 = _mm256_sub_ps(one, _mm256_loadu_ps(d));
    const __m256 u2 = _mm256_loadu_ps(d + 8);
    // log(u1)
    __m256 x = _mm256_max_ps(u1, _mm256_castsi256_ps(_mm256_set1_epi32(0x00800000)));
    __m256i imm0 = _mm256_srli_epi32(_mm256_castps_si256(x), 23);
    x = _mm256_and_ps(x, _mm256_castsi256_ps(_mm256_set1_epi32(~0x7f800000)));
    x = _mm256_or_ps(x, _mm256_set1_ps(0.5f));
    imm0 = _mm256_sub_epi32(imm0, _mm256_set1_epi32(0x7f));
    __m256 e = _mm256_add_ps(_mm256_cvtepi32_ps(imm0), one);
    const __m256 mask = _mm256_cmp_ps(x, _mm256_set1_ps((float)0.707106781186547524), _CMP_LT_OS);
    const __m256 tmp = _mm256_and_ps(x, mask);
    x = _mm256_sub_ps(x, one);
    e = _mm256_sub_ps(e, _mm256_and_ps(one, mask));
    x = _mm256_add_ps(x, tmp);
    const __m256 z = _mm256_mul_ps(x, x);
    __m256 y = _mm256_set1_ps((float)7.0376836292E-2);
    y = _mm256_fmadd_ps(y, x, _mm256_set1_ps((float)-1.1514610310E-1));
    y = _mm256_fmadd_ps(y, x, _mm256_set1_ps((float)1.1676998740E-1));
    y = _mm256_fmadd_ps(y, x, _mm256_set1_ps((float)-1.2420140846E-1));
    y = _mm256_fmadd_ps(y, x, _mm256_set1_ps((float)1.4249322787E-1));
    y = _mm256_fmadd_ps(y, x, _mm256_set1_ps((float)-1.6668057665E-1));
    y = _mm256_fmadd_ps(y, x, _mm256_set1_ps((float)2.0000714765E-1));
    y = _mm256_fmadd_ps(y, x, _mm256_set1_ps((float)-2.4999993993E-1));
    y = _mm256_fmadd_ps(y, x, _mm256_set1_ps((float)3.3333331174E-1));
    y = _mm256_mul_ps(y, x);
    y = _mm256_fmadd_ps(y, z, _mm256_mul_ps(e, _mm256_set1_ps((float)-2.12194440e-4)));
    y = _mm256_fnmadd_ps(z, _mm256_set1_ps(0.5f), y);
    x = _mm256_add_ps(x, y);
    x = _mm256_fmadd_ps(e, _mm256_set1_ps((float)0.693359375), x);
    const __m256 radius = _mm256_sqrt_ps(_mm256_mul_ps(_mm256_set1_ps(-2.0f), x));
    // sincos(2 pi u2), argument >= 0
    const __m256 th = _mm256_mul_ps(_mm256_set1_ps((float)(2.0 * kPi)), u2);
    const __m256 sign_mask = _mm256_castsi256_ps(_mm256_set1_epi32((int)0x80000000));
    __m256 xs = _mm256_andnot_ps(sign_mask, th);
    __m256 sign_sin = _mm256_and_ps(th, sign_mask);
    __m256 ys = _mm256_mul_ps(xs, _mm256_set1_ps((float)1.27323954473516));
    __m256i j = _mm256_cvttps_epi32(ys);
    j = _mm256_and_si256(_mm256_add_epi32(j, _mm256_set1_epi32(1)), _mm256_set1_epi32(~1));
    ys = _mm256_cvtepi32_ps(j);
    const __m256 swap_sin = _mm256_castsi256_ps(_mm256_slli_epi32(_mm256_and_si256(j, _mm256_set1_epi32(4)), 29));
    const __m256 poly = _mm256_castsi256_ps(
        _mm256_cmpeq_epi32(_mm256_and_si256(j, _mm256_set1_epi32(2)), _mm256_setzero_si256()));
    xs = _mm256_fmadd_ps(ys, _mm256_set1_ps(-0.78515625f), xs);
    xs = _mm256_fmadd_ps(ys, _mm256_set1_ps(-2.4187564849853515625e-4f), xs);
    xs = _mm256_fmadd_ps(ys, _mm256_set1_ps((float)-3.77489497744594108e-8), xs);
    const __m256 sign_cos = _mm256_castsi256_ps(_mm256_slli_epi32(
        _mm256_andnot_si256(_mm256_sub_epi32(j, _mm256_set1_epi32(2)), _mm256_set1_epi32(4)), 29));
    sign_sin = _mm256_xor_ps(sign_sin, swap_sin);
    const __m256 zz = _mm256_mul_ps(xs, xs);
    __m256 yc = _mm256_set1_ps((float)2.443315711809948E-005);
    yc = _mm256_fmadd_ps(yc, zz, _mm256_set1_ps((float)-1.388731625493765E-003));
    yc = _mm256_fmadd_ps(yc, zz, _mm256_set1_ps((float)4.166664568298827E-002));
    yc = _mm256_mul_ps(yc, zz);
    yc = _mm256_fmsub_ps(yc, zz, _mm256_mul_ps(zz, _mm256_set1_ps(0.5f)));
    yc = _mm256_add_ps(yc, one);
    __m256 y2 = _mm256_set1_ps((float)-1.9515295891E-4);
    y2 = _mm256_fmadd_ps(y2, zz, _mm256_set1_ps((float)8.3321608736E-3));
    y2 = _mm256_fmadd_ps(y2, zz, _mm256_set1_ps((float)-1.6666654611E-1));
    y2 = _mm256_mul_ps(y2, zz);
    y2 = _mm256_fmadd_ps(y2, xs, xs);
    const __m256 ysin2 = _mm256_and_ps(poly, y2);
    const __m256 ysin1 = _mm256_andnot_ps(poly, yc);
    y2 = _mm256_sub_ps(y2, ysin2);
    yc = _mm256_sub_ps(yc, ysin1);
    const __m256 sn = _mm256_xor_ps(_mm256_add_ps(ysin1, ysin2), sign_sin);
    const __m256 cs = _mm256_xor_ps(_mm256_add_ps(yc, y2), sign_cos);
    const __m256 zero = _mm256_setzero_ps();
    _mm256_storeu_ps(d, _mm256_fmadd_ps(_mm256_mul_ps(radius, cs), one, zero));
    _mm256_storeu_ps(d + 8, _mm256_fmadd_ps(_mm256_mul_ps(radius, sn), one, zero));
}

bool have_avx2_fma() {
    static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
    return ok;
}

__attribute__((target("fma"))) void draw_f32(Gen& g, int64_t n, float* d) {
    if (n < 16) {
        for (int64_t i = 0; i < n; ++i) d[i] = (float)g.normal_d();
        return;
    }
    void (*block)(float*) = have_avx2_fma() ? f32_block16_avx2 : f32_block16;
    for (int64_t i = 0; i < n; ++i) d[i] = g.uniform_f();
    for (int64_t i = 0; i + 16 <= n; i += 16) block(d + i);
    if (n % 16) {  // recompute the last 16 values from fresh uniforms
        float* t = d + n - 16;
        for (int j = 0; j < 16; ++j) t[j] = g.uniform_f();
        block(t);
    }
}

void bf16_block16(Gen& g, uint16_t* d) {
    uint8_t u[16];
    for (int j = 0; j < 16; ++j) u[j] = (uint8_t)(g.mt.next() & 0xFFu);
    for (int j = 0; j < 8; ++j) {
        const int cell = ((int)u[j] << 8) | u[j + 8];
        d[j] = g_cos[cell];
        d[j + 8] = g_sin[cell];
    }
}

void draw_bf16(Gen& g, int64_t n, uint16_t* d) {
    if (n < 16) {
        for (int64_t i = 0; i < n; ++i) d[i] = bf16_bits((float)g.normal_d());
        return;
    }
    std::call_once(g_once, build_tables);
    // all n uniforms precede every transform, and whole blocks consume them in order
    const int64_t whole = n / 16 * 16;
    for (int64_t i = 0; i < whole; i += 16) bf16_block16(g, d + i);
    if (n % 16) {
        for (int64_t i = whole; i < n; ++i) (void)g.mt.next();  // the partial block's uniforms
        bf16_block16(g, d + n - 16);                           // last 16 from fresh ones
    }
}

}  // namespace

extern "C" int arctopk_draw_normal(uint64_t seed, int32_t dtype, int32_t ntensors,
                                   const int64_t* sizes, void* out) {
    if (ntensors < 0 || (ntensors > 0 && (!sizes || !out))) return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EINVAL;
    for (int32_t t = 0; t < ntensors; ++t)
        if (sizes[t] < 0) return ARCTOPK_EINVAL;
    Gen g(seed);
    int64_t off = 0;
    for (int32_t t = 0; t < ntensors; ++t) {
        if (dtype == ARCTOPK_F32)
            draw_f32(g, sizes[t], static_cast<float*>(out) + off);
        else
            draw_bf16(g, sizes[t], static_cast<uint16_t*>(out) + off);
        off += sizes[t];
    }
    return 0;
}

extern "C" int arctopk_draw_bf16_normal(uint64_t seed, int64_t total, uint16_t* out) {
    if (!out || total < 0 || total % 16 != 0) return ARCTOPK_EINVAL;
    // whole 16-blocks only: one fill of the concatenation equals the per-tensor fills
    Gen g(seed);
    if (total) draw_bf16(g, total, out);
    return 0;
}

// ---- background draws -------------------------------------------------------------------
// The projections of the next calls are drawn ahead on native threads: no Python thread
// holds or waits for the GIL while the hook's thread enqueues kernels.
namespace {

struct DrawTask {
    int64_t ticket;
    uint64_t seed;
    int32_t dtype;
    std::vector<int64_t> sizes;
    void* out;
};

struct DrawPool {
    std::mutex mu;
    std::condition_variable cv_task, cv_done;
    std::deque<DrawTask> queue;
    std::unordered_map<int64_t, int> done;  // ticket -> status, until waited / polled
    std::vector<std::thread> threads;
    int64_t next_ticket = 1;
    bool stop = false;

    void run() {
        for (;;) {
            DrawTask t;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_task.wait(lk, [&] { return stop || !queue.empty(); });
                if (stop) return;  // queued draws are dropped: their buffers are the caller's
                t = std::move(queue.front());
                queue.pop_front();
            }
            const int rc = arctopk_draw_normal(t.seed, t.dtype, (int32_t)t.sizes.size(), t.sizes.data(), t.out);
            {
                std::lock_guard<std::mutex> lk(mu);
                done[t.ticket] = rc;
            }
            cv_done.notify_all();
        }
    }
};

}  // namespace

extern "C" int arctopk_draw_pool_create(int32_t nthreads, void** pool) {
    if (!pool || nthreads < 1 || nthreads > 64) return ARCTOPK_EINVAL;
    DrawPool* p = new DrawPool;
    for (int i = 0; i < nthreads; ++i) p->threads.emplace_back([p] { p->run(); });
    *pool = p;
    return 0;
}

extern "C" int arctopk_draw_pool_destroy(void* pool) {
    if (!pool) return 0;
    DrawPool* p = static_cast<DrawPool*>(pool);
    {
        std::lock_guard<std::mutex> lk(p->mu);
        p->stop = true;
        p->queue.clear();
    }
    p->cv_task.notify_all();
    for (std::thread& t : p->threads) t.join();  // running draws finish first
    delete p;
    return 0;
}

extern "C" int64_t arctopk_draw_submit(void* pool, uint64_t seed, int32_t dtype, int32_t ntensors,
                                       const int64_t* sizes, void* out) {
    if (!pool || ntensors < 0 || (ntensors > 0 && (!sizes || !out))) return -ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return -ARCTOPK_EINVAL;
    DrawPool* p = static_cast<DrawPool*>(pool);
    DrawTask t{0, seed, dtype, std::vector<int64_t>(sizes, sizes + ntensors), out};
    int64_t ticket;
    {
        std::lock_guard<std::mutex> lk(p->mu);
        ticket = t.ticket = p->next_ticket++;
        p->queue.push_back(std::move(t));
    }
    p->cv_task.notify_one();
    return ticket;
}

// Block until the draw of `ticket` is complete; returns its status and forgets the ticket.
extern "C" int arctopk_draw_wait(void* pool, int64_t ticket) {
    if (!pool || ticket < 1) return ARCTOPK_EINVAL;
    DrawPool* p = static_cast<DrawPool*>(pool);
    std::unique_lock<std::mutex> lk(p->mu);
    p->cv_done.wait(lk, [&] { return p->done.count(ticket) != 0; });
    const int rc = p->done[ticket];
    p->done.erase(ticket);
    return rc;
}

// Non-blocking: 1 if the draw is complete, -status if it failed (the ticket is forgotten
// either way), 0 if not yet.
extern "C" int arctopk_draw_poll(void* pool, int64_t ticket) {
    if (!pool || ticket < 1) return -ARCTOPK_EINVAL;
    DrawPool* p = static_cast<DrawPool*>(pool);
    std::lock_guard<std::mutex> lk(p->mu);
    auto it = p->done.find(ticket);
    if (it == p->done.end()) return 0;
    const int rc = it->second;
    p->done.erase(it);
    return rc ? -rc : 1;
}

// Stream-ordered host -> device copy (hipMemcpyAsync) without a torch dispatch.
extern "C" int arctopk_memcpy_h2d_async(void* dst, const void* src, int64_t bytes, void* stream) {
    if (!dst || !src || bytes < 0) return ARCTOPK_EINVAL;
    if (bytes == 0) return 0;
    return (int)hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, (hipStream_t)stream);
}
