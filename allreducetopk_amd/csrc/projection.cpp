// Host-side bf16 projections: the exact values of the reference's
// torch.randn(m, r, dtype=torch.bfloat16) on CPU (group_topk_hook_no_reshape.py:49, :79) after
// torch.manual_seed(seed) (:255), without torch's scalar per-element loop.
//
// torch's CPU normal_ on a bf16 tensor of >= 16 elements runs normal_fill in BFloat16
// arithmetic: one mt19937 draw per element, u = (x & 0xFF) / 256 (an 8-bit uniform, exact
// in bf16), then per block of 16 and j < 8, with u1 = 1 - u[j] and u2 = u[j + 8]:
//   radius = sqrt(-2 * log(u1)), theta = 2*pi*u2,
//   out[j] = radius * cos(theta), out[j + 8] = radius * sin(theta),
// every BFloat16 operation computed in float (libm logf / sqrtf / cosf / sinf) and rounded
// to bf16 (round-to-nearest-even), theta formed in double then narrowed to float and bf16.
// With 8-bit uniforms each output is a function of (u[j], u[j+8]) only: two 256 x 256 tables.
// Pinned bit for bit against torch by tests/test_host_logic.py.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>

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

uint16_t g_cos[256 * 256], g_sin[256 * 256];
std::once_flag g_once;

void build_tables() {
    float radius[256], c[256], s[256];
    for (int k = 0; k < 256; ++k) {
        const float u = rb((float)k / 256.0f);
        const float u1 = rb(1.0f - u);
        const float lg = rb(std::log(u1));
        radius[k] = rb(std::sqrt(rb(-2.0f * lg)));
        const float theta = rb((float)(2.0 * 3.14159265358979323846 * (double)u));
        c[k] = rb(std::cos(theta));
        s[k] = rb(std::sin(theta));
    }
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b) {
            g_cos[a * 256 + b] = bf16_bits(radius[a] * c[b]);
            g_sin[a * 256 + b] = bf16_bits(radius[a] * s[b]);
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
    void twist() {
        for (int k = 0; k < 624; ++k) {
            const uint32_t y = (st[k] & 0x80000000u) | (st[(k + 1) % 624] & 0x7FFFFFFFu);
            st[k] = st[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
        }
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

}  // namespace

extern "C" int arctopk_draw_bf16_normal(uint64_t seed, int64_t total, uint16_t* out) {
    if (!out || total < 0 || total % 16 != 0) return ARCTOPK_EINVAL;
    std::call_once(g_once, build_tables);
    MT mt((uint32_t)(seed & 0xFFFFFFFFu));
    uint8_t u[16];
    for (int64_t b = 0; b < total; b += 16) {
        for (int j = 0; j < 16; ++j) u[j] = (uint8_t)(mt.next() & 0xFFu);
        for (int j = 0; j < 8; ++j) {
            const int cell = ((int)u[j] << 8) | u[j + 8];
            out[b + j] = g_cos[cell];
            out[b + j + 8] = g_sin[cell];
        }
    }
    return 0;
}
