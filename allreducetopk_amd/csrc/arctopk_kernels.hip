// ARC-TopK per-bucket codec kernels for MI355X (gfx950, wave64).
//
//   K1 encode : EF pre-apply + rank-r sketch, one HBM pass over the bucket
//   K2 select : mean sketch -> row energy -> exact top-k rows by LDS radix select
//   K3 pack   : gather selected rows into the packed buffer + residual update
//   K4 decode : one full-bucket write of the mean of the selected rows (+ EF21 gE)
//
// All kernels are HBM-streaming except K2 (latency-bound, a few KiB per segment).
// Reference: comm_hooks/group_topk_hook_no_reshape.py (see include/arctopk.h).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>

#include "common.h"
#include "mselect.h"
#include "mselect_dev.h"
#include "vdraw.h"  // (fast contraction inside, for rocrand only)

using namespace arctopk;

namespace {
// a kernel launch whose argument list is checked against the kernel's parameter types
template <typename... P, typename... A>
void launch_job_kernel(void (*f)(P...), dim3 grid, dim3 block, size_t shm, hipStream_t st, A... a) {
    static_assert(sizeof...(P) == sizeof...(A), "argument count");
    hipLaunchKernelGGL(f, grid, block, shm, st, static_cast<P>(a)...);
}
}  // namespace

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int EF, bool ERR_IN>
__device__ __forceinline__ float4 ef_apply4(const float4* __restrict__ g4, float4* __restrict__ e4,
                                            int64_t i) {
    float4 x = g4[i];
    if constexpr (EF == ARCTOPK_EF14) {
        if constexpr (ERR_IN) {
            const float4 e = e4[i];
            x.x += e.x; x.y += e.y; x.z += e.z; x.w += e.w;
        }
    } else if constexpr (EF == ARCTOPK_EF21) {
        const float4 e = e4[i];
        x.x -= e.x; x.y -= e.y; x.z -= e.z; x.w -= e.w;
    }
    return x;
}

// X = G (+|-) E of one element, rounded to T as the reference's in-place add_ on a T bucket
template <typename T, int EF, bool ERR_IN>
__device__ __forceinline__ float ef_apply1(const T* __restrict__ g, const T* __restrict__ e,
                                           int64_t i) {
    float x = ld1<T, true>(g + i);
    if constexpr (EF == ARCTOPK_EF14) {
        if constexpr (ERR_IN) x = rnd<T>(x + ld1<T, true>(e + i));
    } else if constexpr (EF == ARCTOPK_EF21) {
        x = rnd<T>(x - ld1<T, true>(e + i));
    }
    return x;
}

// the same on a quad (x = g (+|-) e, rounded to T)
template <typename T, int EF, bool ERR_IN>
__device__ __forceinline__ float4 ef_combine4(float4 x, float4 e) {
    if constexpr (EF == ARCTOPK_EF14 && ERR_IN) {
        x.x += e.x; x.y += e.y; x.z += e.z; x.w += e.w;
        return rnd4<T>(x);
    } else if constexpr (EF == ARCTOPK_EF21) {
        x.x -= e.x; x.y -= e.y; x.z -= e.z; x.w -= e.w;
        return rnd4<T>(x);
    }
    return x;
}

// ---------------------------------------------------------------------------
// K1 encode
// ---------------------------------------------------------------------------
// One block (256 threads = 4 waves) per tile.
//  ENC_ROW_VEC    : wave per row, float4 columns, V^T staged in LDS ([R][m]) -- the
//                   [2048,2048] fast path; every lane keeps 8 x 16 B loads in flight.
//  ENC_ROW_SCALAR : same, scalar columns (misaligned rows / m % 4 != 0).
//  ENC_TILE       : m < 64 (ND convs, m = 2*t^2): the tile's rows are loaded coalesced
//                   into LDS, then one thread per row forms its R dot products.
//  ENC_RAW        : 1-D tensors: the sketch is the (EF-applied) values themselves.
// Order key: energies are >= +0 or NaN; as uint32 the non-negative floats are
// ordered, and every NaN (either sign) maps above +inf, as torch.topk ranks NaN largest.
__device__ __forceinline__ uint32_t energy_key(float e) {
    uint32_t u = __float_as_uint(e);
    if (e != e) u = 0x7FFFFFFFu;  // NaN largest (above +inf 0x7F800000; bit 31 stays clear)
    return u & 0x7FFFFFFFu ? u : 0u;  // -0 cannot occur; keep +0 = 0
}

// The energy of a row from its R fp32 sketch sums in registers, exactly as row_energy forms it
// from the stored sketch at world size 1: each sum rounded to T as it is stored, divided by 1
// (exact), squared and summed in order (keys mode of the encode).
template <typename T, int R>
__device__ __forceinline__ float energy_regs(const float (&acc)[R]) {
    const float a = rnd<T>(acc[0]);
    float s = rnd<T>(__fmul_rn(a, a));
#pragma unroll
    for (int j = 1; j < R; ++j) {
        const float b = rnd<T>(acc[j]);
        s = __fadd_rn(s, rnd<T>(__fmul_rn(b, b)));
    }
    return rnd<T>(s);
}

template <typename T, int R, int EF, bool ERR_IN, bool ROWS = true>
__device__ __forceinline__ void encode_tile(const SegDev* __restrict__ segs, const EncTile t,
                                            const T* __restrict__ G, T* __restrict__ E,
                                            const T* __restrict__ V, T* __restrict__ sketch,
                                            float* __restrict__ part_buf, uint32_t* __restrict__ keys,
                                            float* __restrict__ lds) {
    const SegDev s = segs[t.seg];
    // keys mode (world size 1, multi-block select items): the row's energy key instead of its
    // sketch -- the key the select's key pass would form from the sketch (k_arc_keys)
    uint32_t* const kout = (keys && s.keyed) ? keys + s.row_off : nullptr;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    constexpr bool WRITE_E = (EF == ARCTOPK_EF14);

    if (t.mode == ENC_RAW) {
        const int64_t base = s.offset + t.row0;
        T* out = sketch + s.sketch_off + t.row0;
        int64_t done = 0;
        if constexpr (sizeof(T) == 4) {
            if ((base & 3) == 0 && ((s.sketch_off + t.row0) & 3) == 0) {
                // 16-B quads, all of a thread's loads issued before its stores (the scalar loop
                // below is one dependent round trip per element: a store to E may not move above
                // the next load from E)
                constexpr int Q = 4;
                constexpr bool LOAD_E = (EF == ARCTOPK_EF21) || (EF == ARCTOPK_EF14 && ERR_IN);
                const int cnt4 = (int)(t.nrows >> 2);
                for (int q0 = tid; q0 < cnt4; q0 += 256 * Q) {
                    float4 gv[Q], ev[Q];
#pragma unroll
                    for (int u = 0; u < Q; ++u) {
                        const int q = min(q0 + u * 256, cnt4 - 1);
                        gv[u] = ldq<T, true>(G + base, q);
                        if constexpr (LOAD_E) ev[u] = ldq<T, true>(E + base, q);
                    }
#pragma unroll
                    for (int u = 0; u < Q; ++u) {
                        const int q = q0 + u * 256;
                        if (q < cnt4) {
                            const float4 x = ef_combine4<T, EF, ERR_IN>(gv[u], ev[u]);
                            if constexpr (WRITE_E) stq<T, true>(E + base, q, x);
                            stq<T, false>(out, q, x);
                        }
                    }
                }
                done = (int64_t)cnt4 << 2;
            }
        }
        for (int64_t i = done + tid; i < t.nrows; i += 256) {
            const float x = ef_apply1<T, EF, ERR_IN>(G + base, E + base, i);
            if constexpr (WRITE_E) st1<T, true>(E + base + i, x);
            st1<T>(out + i, x);
        }
        return;
    }

    const int m = (int)s.m;
    const T* __restrict__ Vs = V + s.v_off;  // [m][R]

    if (t.mode == ENC_TILE) {
        // LDS: V [m][R] (padded to 16 B), then the tile [nrows*m]
        float* vl = lds;
        float* tile = lds + ((m * R + 3) & ~3);
        for (int i = tid; i < m * R; i += 256) vl[i] = to_f(Vs[i]);
        const int64_t base = s.offset + t.row0 * m;
        const int cnt = (int)t.nrows * m;
        int done = 0;
        if ((base & 3) == 0) {
            // 16-B streams, all of a thread's loads issued before its stores (a store to E
            // may not be reordered above a later load from E by the compiler)
            constexpr int Q = 4;
            constexpr bool LOAD_E = (EF == ARCTOPK_EF21) || (EF == ARCTOPK_EF14 && ERR_IN);
            const int cnt4 = cnt >> 2;
            const T* gp = G + base;
            T* ep = E + base;
            float4* t4 = reinterpret_cast<float4*>(tile);
            for (int q0 = tid; q0 < cnt4; q0 += 256 * Q) {
                float4 gv[Q], ev[Q];
#pragma unroll
                for (int u = 0; u < Q; ++u) {
                    const int q = min(q0 + u * 256, cnt4 - 1);
                    gv[u] = ldq<T, true>(gp, q);
                    if constexpr (LOAD_E) ev[u] = ldq<T, true>(ep, q);
                }
#pragma unroll
                for (int u = 0; u < Q; ++u) {
                    const int q = q0 + u * 256;
                    if (q < cnt4) {
                        const float4 x = ef_combine4<T, EF, ERR_IN>(gv[u], ev[u]);
                        if constexpr (WRITE_E) stq<T, true>(ep, q, x);
                        t4[q] = x;
                    }
                }
            }
            done = cnt4 << 2;
        }
        for (int i = done + tid; i < cnt; i += 256) {
            const float x = ef_apply1<T, EF, ERR_IN>(G + base, E + base, i);
            if constexpr (WRITE_E) st1<T, true>(E + base + i, x);
            tile[i] = x;
        }
        __syncthreads();
        // thread per row (tiles of up to a few thousand rows for the smallest m)
        const bool vec_out = (R == 4) && sizeof(T) == 4 && ((s.sketch_off & 3) == 0);
        for (int rr = tid; rr < t.nrows; rr += 256) {
            float acc[R];
#pragma unroll
            for (int j = 0; j < R; ++j) acc[j] = 0.f;
            const float* row = tile + rr * m;
            for (int c = 0; c < m; ++c) {
                const float x = row[c];
#pragma unroll
                for (int j = 0; j < R; ++j) acc[j] = fmaf(x, vl[c * R + j], acc[j]);
            }
            if (kout) {
                kout[t.row0 + rr] = energy_key(energy_regs<T, R>(acc));
                continue;
            }
            T* out = sketch + s.sketch_off + (t.row0 + rr) * R;
            if constexpr (R == 4 && sizeof(T) == 4) {
                if (vec_out) {
                    *reinterpret_cast<float4*>(out) = make_float4(acc[0], acc[1], acc[2], acc[3]);
                    continue;
                }
            }
#pragma unroll
            for (int j = 0; j < R; ++j) st1<T>(out + j, acc[j]);
        }
        return;
    }
    if constexpr (!ROWS) return;  // k_encode_short: a table without wave-per-row tiles
    else {

    // wave-per-row modes over the tile's columns [c0, c0 + cl): stage that slice of V^T
    // ([R][cl]) in LDS (conflict-free writes: consecutive lanes take consecutive columns
    // of one j).  Column-split tensors write per-part partial sketches, summed in fixed
    // part order by k_sketch_combine.
    const int c0 = t.c0, cl = t.clen;
    // bf16 rows: V^T kept as bf16 pairs, X used as the packed bf16 words it is stored as, and
    // the sketch formed by v_dot2c_f32_bf16 (two products, exact in fp32, per instruction):
    // no unpacking of X and half the VALU instructions of the fp32-FMA form
    constexpr bool kDot2 = sizeof(T) == 2;
    if (kDot2 && t.mode == ENC_ROW_VEC) {
        uint16_t* l16 = reinterpret_cast<uint16_t*>(lds);
#pragma unroll
        for (int j = 0; j < R; ++j)
            for (int c = tid; c < cl; c += 256)
                l16[j * cl + c] = reinterpret_cast<const uint16_t*>(Vs)[(int64_t)(c0 + c) * R + j];
        __syncthreads();
    } else {
        if constexpr (R == 4) {
            for (int c = tid; c < cl; c += 256) {
                const float4 v = ldq<T, false>(Vs, c0 + c);  // V[c0 + c][0..3]
                lds[c] = v.x;
                lds[cl + c] = v.y;
                lds[2 * cl + c] = v.z;
                lds[3 * cl + c] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < R; ++j)
                for (int c = tid; c < cl; c += 256) lds[j * cl + c] = to_f(Vs[(int64_t)(c0 + c) * R + j]);
        }
        __syncthreads();
    }
    // the row's R sums: rounded to T into the sketch, or fp32 partials of a column part
    T* const sk_out = sketch + s.sketch_off;
    float* const pt_out = t.part < 0 ? nullptr : part_buf + s.part_off + (int64_t)t.part * s.n * R;
    auto put = [&](int64_t i, float v) {
        if (pt_out) pt_out[i] = v;
        else st1<T>(sk_out + i, v);
    };
    const int64_t rs = t.rstride;
    if constexpr (kDot2) {
        if (t.mode == ENC_ROW_VEC) {
            constexpr int U = ARCTOPK_ENC_UNITS_BF16;  // 16-B units (8 bf16) per lane per step, two buffers
            constexpr bool LOAD_E = (EF == ARCTOPK_EF21) || (EF == ARCTOPK_EF14 && ERR_IN);
            constexpr bool COMBINE = LOAD_E;  // x = rnd(g +- e); else x = g (already bf16)
            const int mu = cl >> 3;           // units of this tile row (cl is a multiple of 8)
            const int steps = (mu + 64 * U - 1) / (64 * U);
            const u4_t* vp = reinterpret_cast<const u4_t*>(lds);  // [R][mu] units of V^T pairs
            u4_t ga[U], ea[U], gb[U], eb[U];
            float acc[R];
#pragma unroll
            for (int j = 0; j < R; ++j) acc[j] = 0.f;
            auto issue = [&](u4_t (&gx)[U], u4_t (&ex)[U], int64_t r_, int st_) {
                const T* gp = G + s.offset + r_ * m + c0;
                const T* ep = E + s.offset + r_ * m + c0;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int c = min(st_ * 64 * U + u * 64 + lane, mu - 1);
                    gx[u] = ld16raw<T, true>(gp, c);
                    if constexpr (LOAD_E) ex[u] = ld16raw<T, true>(ep, c);
                }
            };
            auto combine = [&](uint32_t g, uint32_t e) -> uint32_t {
                const float gl = __uint_as_float(g << 16), gh = __uint_as_float(g & 0xFFFF0000u);
                const float el = __uint_as_float(e << 16), eh = __uint_as_float(e & 0xFFFF0000u);
                if constexpr (EF == ARCTOPK_EF21) return cvt_pk_bf16(gl - el, gh - eh);
                else return cvt_pk_bf16(gl + el, gh + eh);
            };
            auto consume = [&](u4_t (&gx)[U], u4_t (&ex)[U], int64_t r_, int st_) {
                T* ep = E + s.offset + r_ * m + c0;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int cu = st_ * 64 * U + u * 64 + lane;
                    const bool ok = cu < mu;  // lanes past the row end loaded a clamped copy
                    const int c = ok ? cu : mu - 1;
                    u4_t x = gx[u];
                    if constexpr (COMBINE)
                        x = u4_t{combine(x.x, ex[u].x), combine(x.y, ex[u].y), combine(x.z, ex[u].z),
                                 combine(x.w, ex[u].w)};
                    if constexpr (WRITE_E) {
                        if (ok) __builtin_nontemporal_store(x, reinterpret_cast<u4_t*>(ep) + c);
                    }
                    if (!ok) x = u4_t{0u, 0u, 0u, 0u};
                    // The words go through scalars: ROCm 7.2's clang lowers __builtin_bit_cast of an
                    // ext_vector ELEMENT (x.y, x.z, ...) to element 0 (and loads only that dword;
                    // scripts/probe_dot2vec.hip), which paired every column with the wrong V entry
                    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int j = 0; j < R; ++j) {
                        const u4_t v = vp[j * mu + c];
                        const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
                        float a = acc[j];
#pragma unroll
                        for (int h = 0; h < 4; ++h)
                            a = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, xw[h]),
                                                                __builtin_bit_cast(bf2_t, vw[h]), a, false);
                        acc[j] = a;
                    }
                }
                if (st_ == steps - 1) {
#pragma unroll
                    for (int j = 0; j < R; ++j) acc[j] = wave_sum(acc[j]);
                    if (kout) {
                        if (lane == 0) kout[r_] = energy_key(energy_regs<T, R>(acc));
                    } else if (lane < R) {
                        float v = acc[0];
#pragma unroll
                        for (int j = 1; j < R; ++j)
                            if (lane == j) v = acc[j];
                        put(r_ * R + lane, v);
                    }
#pragma unroll
                    for (int j = 0; j < R; ++j) acc[j] = 0.f;
                }
            };
            const int64_t nq = t.nrows;
            int64_t qa = wave;
            int sa = 0;
            if (qa < nq) issue(ga, ea, t.row0 + qa * rs, sa);
            while (qa < nq) {
                int64_t qb = qa;
                int sb = sa + 1;
                if (sb == steps) { sb = 0; qb += 4; }
                if (qb < nq) issue(gb, eb, t.row0 + qb * rs, sb);
                consume(ga, ea, t.row0 + qa * rs, sa);
                if (qb >= nq) break;
                qa = qb;
                sa = sb + 1;
                if (sa == steps) { sa = 0; qa += 4; }
                if (qa < nq) issue(ga, ea, t.row0 + qa * rs, sa);
                consume(gb, eb, t.row0 + qb * rs, sb);
            }
            return;
        }
    }
    if (t.mode == ENC_ROW_VEC) {
        // Software-pipelined stream: a wave walks its rows in steps of 64*U 16-B units
        // (U per lane; a unit is 4 fp32 or 8 bf16 elements) with two register buffers: the
        // loads of the next step are in flight while the current step forms its dot
        // products, stores E and (at a row end) reduces.  V^T comes from LDS.
        constexpr int PQ = kQuadsPer16<T>;  // quads per 16-B unit
        constexpr bool LOAD_E = (EF == ARCTOPK_EF21) || (EF == ARCTOPK_EF14 && ERR_IN);
        // units per lane per step: a stream of G alone keeps more of them in flight
        constexpr int U = (LOAD_E ? ARCTOPK_ENC_UNITS_GE : ARCTOPK_ENC_UNITS_G_ONLY) / PQ;
        const int m4 = cl >> 2;   // quads of this tile row
        const int mu = m4 / PQ;   // 16-B units (the plan makes m4 a multiple of PQ)
        const int steps = (mu + 64 * U - 1) / (64 * U);
        const float4* vt4 = reinterpret_cast<const float4*>(lds);
        float4 ga[U][PQ], ea[U][PQ], gb[U][PQ], eb[U][PQ];
        float acc[R];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j] = 0.f;
        // packed FMAs (v_pk_fma_f32) on the G-only stream (A/B: noef headline encode 57.7 -> 53.1
        // us; with E loads the EF14 encode measured 140 -> 146 us, so those keep scalar FMAs)
        constexpr bool kPk = !LOAD_E;
        f2_t acc2[R];
#pragma unroll
        for (int j = 0; j < R; ++j) acc2[j] = f2_t{0.f, 0.f};

        auto issue = [&](float4 (&gx)[U][PQ], float4 (&ex)[U][PQ], int64_t r_, int st_) {
            const T* gp = G + s.offset + r_ * m + c0;
            const T* ep = E + s.offset + r_ * m + c0;
#pragma unroll
            for (int u = 0; u < U; ++u) {  // unconditional (clamped) loads: no exec-masked blocks
                const int c = min(st_ * 64 * U + u * 64 + lane, mu - 1);
                ld16<T, kEncNtLoad>(gp, c, gx[u]);
                if constexpr (LOAD_E) ld16<T, kEncNtLoad>(ep, c, ex[u]);
            }
        };
        auto consume = [&](float4 (&gx)[U][PQ], float4 (&ex)[U][PQ], int64_t r_, int st_) {
            T* ep = E + s.offset + r_ * m + c0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int cu = st_ * 64 * U + u * 64 + lane;
                const bool ok = cu < mu;  // lanes past the row end loaded a clamped copy
                const int c = ok ? cu : mu - 1;
                float4 x[PQ];
#pragma unroll
                for (int h = 0; h < PQ; ++h) x[h] = ef_combine4<T, EF, ERR_IN>(gx[u][h], ex[u][h]);
                if constexpr (WRITE_E) {
                    if (ok) st16<T, kEncNtStore>(ep, c, x);
                }
#pragma unroll
                for (int h = 0; h < PQ; ++h)
                    if (!ok) x[h] = make_float4(0.f, 0.f, 0.f, 0.f);
                if constexpr (kPk) {
                    // packed FMA (v_pk_fma_f32): even / odd columns accumulate separately, two
                    // products per instruction; the halves are added at the row end
#pragma unroll
                    for (int j = 0; j < R; ++j) {
                        f2_t a = acc2[j];
#pragma unroll
                        for (int h = 0; h < PQ; ++h) {
                            const float4 v = vt4[j * m4 + c * PQ + h];
                            a = __builtin_elementwise_fma(f2_t{x[h].x, x[h].y}, f2_t{v.x, v.y}, a);
                            a = __builtin_elementwise_fma(f2_t{x[h].z, x[h].w}, f2_t{v.z, v.w}, a);
                        }
                        acc2[j] = a;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < R; ++j) {
                        float a = acc[j];
#pragma unroll
                        for (int h = 0; h < PQ; ++h) {
                            const float4 v = vt4[j * m4 + c * PQ + h];
                            a = fmaf(x[h].x, v.x, a);
                            a = fmaf(x[h].y, v.y, a);
                            a = fmaf(x[h].z, v.z, a);
                            a = fmaf(x[h].w, v.w, a);
                        }
                        acc[j] = a;
                    }
                }
            }
            if (st_ == steps - 1) {
                if constexpr (kPk) {
#pragma unroll
                    for (int j = 0; j < R; ++j) {
                        acc[j] = acc2[j].x + acc2[j].y;
                        acc2[j] = f2_t{0.f, 0.f};
                    }
                }
#pragma unroll
                for (int j = 0; j < R; ++j) acc[j] = wave_sum(acc[j]);
                // every lane holds all R sums; lanes 0..R-1 store one each.  (The compiler
                // makes the pick a dynamically indexed private array, i.e. a few bytes of
                // scratch per row; the alternative, lane 0 storing all R, measured 10 us
                // slower per headline encode, 148 vs 138 us.)
                if (kout) {
                    if (lane == 0) kout[r_] = energy_key(energy_regs<T, R>(acc));
                } else if (lane < R) {
                    float v = acc[0];
#pragma unroll
                    for (int j = 1; j < R; ++j)
                        if (lane == j) v = acc[j];
                    put(r_ * R + lane, v);
                }
#pragma unroll
                for (int j = 0; j < R; ++j) acc[j] = 0.f;
            }
        };
        // cursor over (tile row q, step) pairs of this wave: q = wave, wave + 4, ...
        const int64_t nq = t.nrows;
        int64_t qa = wave;
        int sa = 0;
        if (qa < nq) issue(ga, ea, t.row0 + qa * rs, sa);
        while (qa < nq) {
            int64_t qb = qa;
            int sb = sa + 1;
            if (sb == steps) { sb = 0; qb += 4; }
            if (qb < nq) issue(gb, eb, t.row0 + qb * rs, sb);
            consume(ga, ea, t.row0 + qa * rs, sa);
            if (qb >= nq) break;
            qa = qb;
            sa = sb + 1;
            if (sa == steps) { sa = 0; qa += 4; }
            if (qa < nq) issue(ga, ea, t.row0 + qa * rs, sa);
            consume(gb, eb, t.row0 + qb * rs, sb);
        }
    } else {  // ENC_ROW_SCALAR
        for (int64_t q = wave; q < t.nrows; q += 4) {
            const int64_t row = t.row0 + q * rs;
            const int64_t base = s.offset + row * m + c0;
            float acc[R];
#pragma unroll
            for (int j = 0; j < R; ++j) acc[j] = 0.f;
            for (int c = lane; c < cl; c += 64) {
                const float x = ef_apply1<T, EF, ERR_IN>(G + base, E + base, c);
                if constexpr (WRITE_E) st1<T, true>(E + base + c, x);
#pragma unroll
                for (int j = 0; j < R; ++j) acc[j] = fmaf(x, lds[j * cl + c], acc[j]);
            }
#pragma unroll
            for (int j = 0; j < R; ++j) acc[j] = wave_sum(acc[j]);
            if (lane == 0) {
                if (kout) {
                    kout[row] = energy_key(energy_regs<T, R>(acc));
                } else {
#pragma unroll
                    for (int j = 0; j < R; ++j) put(row * R + j, acc[j]);
                }
            }
        }
    }
    }  // ROWS
}

// The previous bucket's pack riding in this bucket's encode launch (world size 1: nothing waits
// for the packed values before the next call's select, whose launch carries their decode): its
// chunks are the launch's FIRST blocks, so the gathers run beside the encode's stream instead of
// after it.  Same dtype and EF mode as the encode; the buffers are the previous call's.
template <typename T>
struct PackRide {
    const SegDev* segs;
    const Chunk* chunks;
    const T* G;
    T* E;
    const int32_t* rowlist;
    const int32_t* slotmap;
    T* packed;
    int32_t* dfirst;
    int32_t n;  // chunks (blocks); 0: none
};
template <typename T, int EF>
__device__ __forceinline__ void pack_chunk(const SegDev* __restrict__ segs, const Chunk ch,
                                           const T* __restrict__ G, T* __restrict__ E,
                                           const int32_t* __restrict__ rowlist,
                                           const int32_t* __restrict__ slotmap,
                                           T* __restrict__ packed, int32_t* __restrict__ dfirst,
                                           int32_t* __restrict__ rs);

// One tile per block (after the riding pack's chunks).
template <typename T, int R, int EF, bool ERR_IN>
__global__ void __launch_bounds__(256) k_encode(const SegDev* __restrict__ segs,
                                                const EncTile* __restrict__ tiles, int ntiles,
                                                const T* __restrict__ G, T* __restrict__ E,
                                                const T* __restrict__ V,
                                                T* __restrict__ sketch,
                                                float* __restrict__ part_buf,
                                                uint32_t* __restrict__ keys, PackRide<T> pr) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if ((int)blockIdx.x < pr.n) {
        pack_chunk<T, EF>(pr.segs, pr.chunks[blockIdx.x], pr.G, pr.E, pr.rowlist, pr.slotmap, pr.packed,
                          pr.dfirst, reinterpret_cast<int32_t*>(lds));
        return;
    }
    encode_tile<T, R, EF, ERR_IN>(segs, tiles[blockIdx.x - pr.n], G, E, V, sketch, part_buf, keys, lds);
}

// The same for a tile table without wave-per-row tiles (only 1-D tensors and rows of m < 64:
// conv stacks, BatchNorm vectors): the row paths compiled out, so the kernel needs far fewer
// registers than k_encode and more of its short-lived blocks are resident at once.
template <typename T, int R, int EF, bool ERR_IN>
__global__ void __launch_bounds__(256) k_encode_short(const SegDev* __restrict__ segs,
                                                      const EncTile* __restrict__ tiles, int ntiles,
                                                      const T* __restrict__ G, T* __restrict__ E,
                                                      const T* __restrict__ V, T* __restrict__ sketch,
                                                      float* __restrict__ part_buf, uint32_t* __restrict__ keys,
                                                      PackRide<T> pr) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if ((int)blockIdx.x < pr.n) {
        pack_chunk<T, EF>(pr.segs, pr.chunks[blockIdx.x], pr.G, pr.E, pr.rowlist, pr.slotmap, pr.packed,
                          pr.dfirst, reinterpret_cast<int32_t*>(lds));
        return;
    }
    encode_tile<T, R, EF, ERR_IN, false>(segs, tiles[blockIdx.x - pr.n], G, E, V, sketch, part_buf, keys, lds);
}

// A trailing step's encode (arctopk_exchange_trail: a small bucket whose codec rides in the next
// bucket's launches) -- its tile table and buffers; same dtype, r and EF mode as the carrier
template <typename T>
struct EncRide {
    const SegDev* segs;
    const EncTile* tiles;
    const T* G;
    T* E;
    const T* V;
    T* sketch;
    float* part;
    uint32_t* keys;
    int32_t n;  // tiles (blocks); 0: none
};
// k_encode_short (ROWS false) / k_encode with a trailing step's tiles after the riding pack's
// chunks (kernels of their own, so the product encode kernels keep their code)
template <typename T, int R, int EF, bool ERR_IN, bool ROWS>
__global__ void __launch_bounds__(256) k_encode_carry(const SegDev* __restrict__ segs,
                                                            const EncTile* __restrict__ tiles, int ntiles,
                                                            const T* __restrict__ G, T* __restrict__ E,
                                                            const T* __restrict__ V, T* __restrict__ sketch,
                                                            float* __restrict__ part_buf,
                                                            uint32_t* __restrict__ keys, PackRide<T> pr,
                                                            EncRide<T> er) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if ((int)blockIdx.x < pr.n) {
        pack_chunk<T, EF>(pr.segs, pr.chunks[blockIdx.x], pr.G, pr.E, pr.rowlist, pr.slotmap, pr.packed,
                          pr.dfirst, reinterpret_cast<int32_t*>(lds));
        return;
    }
    const int b = (int)blockIdx.x - pr.n;
    if (b < er.n) {
        encode_tile<T, R, EF, ERR_IN, ROWS>(er.segs, er.tiles[b], er.G, er.E, er.V, er.sketch, er.part, er.keys, lds);
        return;
    }
    encode_tile<T, R, EF, ERR_IN, ROWS>(segs, tiles[b - er.n], G, E, V, sketch, part_buf, keys, lds);
}

// ---------------------------------------------------------------------------
// K2 select
// ---------------------------------------------------------------------------
// mean of the all-reduced values: x / ws exactly; for a power-of-two ws the
// reciprocal is exact and x * (1/ws) rounds the same real number as x / ws.
struct Scale {
    float ws, inv;
    int pow2;
    __device__ __forceinline__ float operator()(float x) const {
        return pow2 ? x * inv : __fdiv_rn(x, ws);
    }
    __device__ __forceinline__ float4 operator()(float4 x) const {
        return make_float4((*this)(x.x), (*this)(x.y), (*this)(x.z), (*this)(x.w));
    }
};


// Energy of a row exactly as the reference forms it on the all-reduced sketch:
// p_j = P_j / ws (IEEE division, ref `P /= ws`), q_j = p_j * p_j (`P ** 2`), then
// ((q_0 + q_1) + q_2) + q_3 (torch.sum over dim 1: sequential for fp32 r <= 4; for bf16
// an fp32 accumulation rounded once), each tensor op's result rounded to T.
// __fmul_rn/__fadd_rn keep the compiler from contracting into FMAs.
template <typename T>
__device__ __forceinline__ float energy4(float a, float b, float c, float d, const Scale& sc) {
    a = rnd<T>(sc(a)); b = rnd<T>(sc(b)); c = rnd<T>(sc(c)); d = rnd<T>(sc(d));
    float e = rnd<T>(__fmul_rn(a, a));
    e = __fadd_rn(e, rnd<T>(__fmul_rn(b, b)));
    e = __fadd_rn(e, rnd<T>(__fmul_rn(c, c)));
    e = __fadd_rn(e, rnd<T>(__fmul_rn(d, d)));
    return rnd<T>(e);
}

template <typename T>
__device__ __forceinline__ float row_energy(const T* __restrict__ p, int R, const Scale& sc,
                                           int kind) {
    if (kind == ARCTOPK_SEG_RAW) {
        const float v = rnd<T>(sc(to_f(p[0])));
        return rnd<T>(__fmul_rn(v, v));
    }
    float a = rnd<T>(sc(to_f(p[0])));
    float s = rnd<T>(__fmul_rn(a, a));
    for (int j = 1; j < R; ++j) {
        const float b = rnd<T>(sc(to_f(p[j])));
        s = __fadd_rn(s, rnd<T>(__fmul_rn(b, b)));
    }
    return rnd<T>(s);
}

template <typename T>
__global__ void __launch_bounds__(256) k_energy(const SegDev* __restrict__ segs, int nseg,
                                                const T* __restrict__ sketch, int R, Scale sc,
                                                uint32_t* __restrict__ keys, float* __restrict__ energy) {
    const int si = blockIdx.y;
    const SegDev s = segs[si];
    const int stride = (s.kind == ARCTOPK_SEG_RAW) ? 1 : R;
    for (int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x; row < s.n;
         row += (int64_t)gridDim.x * 256) {
        const float e = row_energy(sketch + s.sketch_off + row * stride, R, sc, s.kind);
        if (keys) keys[s.row_off + row] = energy_key(e);
        if (energy) energy[s.row_off + row] = e;
    }
}

// Small segments (n <= kSmallSelRows): one 256-thread block per segment, keys in LDS.
//  1. energies -> LDS keys; block OR/AND gives the keys' common leading bits, so the
//     first 8-bit digit covers the most significant *varying* bits (energies of one
//     tensor share sign/exponent bits; digits on those would pile every key into one
//     or two histogram bins and serialise the LDS atomics).
//  2. histogram passes on the varying bits until the bin holding the k-th key has at
//     most kCandMax keys (usually after one pass);
//  3. those candidates are ranked exactly by direct comparison -> threshold T and the
//     number of T-equal keys to take;
//  4. index-ordered compaction (ties at T: lowest rows first).
constexpr int kST = 256;
constexpr int kCandMax = 256;

constexpr int kRegB = 8;  // register path: rows per thread (n <= kRegB * threads)

struct SmallSel {
    uint32_t hist[256];
    __attribute__((aligned(16))) uint32_t cand[kCandMax + 4];
    uint32_t ncand;
    uint32_t wor[16], wand[16];  // per wave, up to 1024 threads
    int64_t wsum[16];
    uint32_t digit, dcount, T;
    int64_t kk, need_eq;
    uint32_t tg[kRegB * 16], te[kRegB * 16];  // register path: per (round, wave) counts
};

__device__ __forceinline__ int64_t block_exscan_s(int64_t v, int64_t* wsum) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int64_t before = x - v;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    __syncthreads();
    return before;
}

// register path, wave 0: exclusive prefix sums, in index order (round-major), of the
// per-(round, wave) counts of rows above / equal to the threshold
template <int NW>
__device__ __forceinline__ void table_exscan2(uint32_t* ta, uint32_t* tb) {
    constexpr int NE = kRegB * NW;
    constexpr int PER = (NE + 63) / 64;
    const int lane = threadIdx.x & 63;
    uint32_t a[PER], b[PER], sa = 0, sb = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int i = lane * PER + q;
        a[q] = i < NE ? ta[i] : 0u;
        b[q] = i < NE ? tb[i] : 0u;
        sa += a[q];
        sb += b[q];
    }
    uint32_t ia = sa, ib = sb;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t ya = __shfl_up(ia, o, 64), yb = __shfl_up(ib, o, 64);
        if (lane >= o) {
            ia += ya;
            ib += yb;
        }
    }
    uint32_t ea = ia - sa, eb = ib - sb;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int i = lane * PER + q;
        if (i < NE) {
            ta[i] = ea;
            tb[i] = eb;
        }
        ea += a[q];
        eb += b[q];
    }
}

// Small segments of at most kRegB * NT rows: the same select with every key held in
// registers (row = u * NT + tid, round u < kRegB).  No LDS key array: the histogram passes
// read registers, the threshold-bin candidates are placed by wave ballots (no atomics), and
// the index-ordered compaction is one scan of the per-(round, wave) counts of rows above /
// equal to the threshold: slot(row) = #above before it + min(#equal before it, need_eq).
template <typename T, int NT>
__device__ __forceinline__ void select_small_reg(const SegDev& s, const T* __restrict__ sketch, int R,
                                                 const Scale& sc, int32_t* __restrict__ rowlist,
                                                 int32_t* __restrict__ slotmap, SmallSel& sh) {
    constexpr int B = kRegB, NW = NT / 64;
    const int n = (int)s.n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const T* sk = sketch + s.sketch_off;
    for (int i = tid; i < 256; i += NT) sh.hist[i] = 0;  // first pass's histogram
    uint32_t key[B];
    if (R == 4 && s.kind == ARCTOPK_SEG_SKETCH && (s.sketch_off & 3) == 0) {
        float4 v[B];
#pragma unroll
        for (int u = 0; u < B; ++u)
            if (u * NT < n) v[u] = ldq<T, false>(sk, min(u * NT + tid, n - 1));
#pragma unroll
        for (int u = 0; u < B; ++u)
            key[u] = u * NT < n ? energy_key(energy4<T>(v[u].x, v[u].y, v[u].z, v[u].w, sc)) : 0u;
    } else {
        const int stride = (s.kind == ARCTOPK_SEG_RAW) ? 1 : R;
#pragma unroll
        for (int u = 0; u < B; ++u)
            key[u] = u * NT < n ? energy_key(row_energy(sk + (int64_t)min(u * NT + tid, n - 1) * stride,
                                                        R, sc, s.kind))
                                : 0u;
    }
    uint32_t kor = 0u, kand = ~0u;
#pragma unroll
    for (int u = 0; u < B; ++u)
        if (u * NT + tid < n) {
            kor |= key[u];
            kand &= key[u];
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        kor |= __shfl_xor(kor, o, 64);
        kand &= __shfl_xor(kand, o, 64);
    }
    if (lane == 0) {
        sh.wor[wave] = kor;
        sh.wand[wave] = kand;
    }
    __syncthreads();
    kor = 0u;
    kand = ~0u;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        kor |= sh.wor[w];
        kand &= sh.wand[w];
    }
    const uint32_t diff = kor ^ kand;
    int bit = diff ? 32 - __clz(diff) : 0;
    uint32_t prefix = kand & ~((bit == 32) ? 0xFFFFFFFFu : ((1u << bit) - 1u));
    uint32_t mask = (bit == 32) ? 0u : ~((1u << bit) - 1u);
    int64_t kk = s.k_rows;
    bool ranked = false, first = true;
    while (bit > 0) {
        const int w = bit < 8 ? bit : 8;
        const int shift = bit - w;
        const uint32_t dmask = (1u << w) - 1u;
        if (!first) {
            for (int i = tid; i < 256; i += NT) sh.hist[i] = 0;
            __syncthreads();
        }
        first = false;
#pragma unroll
        for (int u = 0; u < B; ++u)
            if (u * NT + tid < n && (key[u] & mask) == prefix)
                atomicAdd(&sh.hist[(key[u] >> shift) & dmask], 1u);
        __syncthreads();
        if (wave == 0) {  // lane l owns digits 255-4l .. 252-4l (descending)
            uint32_t c[4], sum = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c[q] = sh.hist[255 - 4 * lane - q];
                sum += c[q];
            }
            uint32_t incl = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            const uint32_t excl = incl - sum;
            if ((uint64_t)excl < (uint64_t)kk && (uint64_t)incl >= (uint64_t)kk) {
                uint32_t acc = excl;
                int q = 0;
                for (; q < 3; ++q) {
                    if ((uint64_t)(acc + c[q]) >= (uint64_t)kk) break;
                    acc += c[q];
                }
                sh.digit = 255 - 4 * lane - q;
                sh.dcount = c[q];
                sh.kk = kk - acc;
            }
        }
        __syncthreads();
        prefix |= sh.digit << shift;
        mask |= dmask << shift;
        kk = sh.kk;
        bit = shift;
        const uint32_t dcount = sh.dcount;
        __syncthreads();
        if (bit > 0 && dcount <= (uint32_t)kCandMax) {
            // the threshold bin's keys -> sh.cand, placed by ballots (wave totals, then lanes)
            uint64_t bm[B];
            uint32_t wtot = 0;
#pragma unroll
            for (int u = 0; u < B; ++u) {
                bm[u] = __ballot(u * NT + tid < n && (key[u] & mask) == prefix);
                wtot += (uint32_t)__popcll(bm[u]);
            }
            if (lane == 0) sh.wor[wave] = wtot;
            __syncthreads();
            uint32_t base = 0, nc = 0;
#pragma unroll
            for (int w2 = 0; w2 < NW; ++w2) {
                const uint32_t c = sh.wor[w2];
                base += w2 < wave ? c : 0u;
                nc += c;
            }
#pragma unroll
            for (int u = 0; u < B; ++u) {
                if ((bm[u] >> lane) & 1ull) sh.cand[base + (uint32_t)__popcll(bm[u] & lt)] = key[u];
                base += (uint32_t)__popcll(bm[u]);
            }
            for (int i = (int)nc + tid; i < (int)((nc + 3) & ~3u); i += NT) sh.cand[i] = 0u;  // pad to x4
            __syncthreads();
            const uint4* c4 = reinterpret_cast<const uint4*>(sh.cand);
            for (int t = tid; t < (int)nc; t += NT) {
                const uint32_t v = sh.cand[t];
                int gt = 0, ge = 0;
                const int nq = ((int)nc + 3) >> 2;
#pragma unroll 4
                for (int j = 0; j < nq; ++j) {  // 16-B broadcast reads, 4 candidates each
                    const uint4 c = c4[j];
                    gt += (c.x > v) + (c.y > v) + (c.z > v) + (c.w > v);
                    ge += (c.x >= v) + (c.y >= v) + (c.z >= v) + (c.w >= v);
                }
                if (v == 0u) ge -= (int)((nc + 3) & ~3u) - (int)nc;  // zero padding equals v only when v == 0
                if (gt < kk && kk <= ge) {  // every writer writes the same (T, need)
                    sh.T = v;
                    sh.need_eq = kk - gt;
                }
            }
            __syncthreads();
            ranked = true;
            break;
        }
    }
    uint32_t thr;
    int64_t need_eq;
    if (ranked) {
        thr = sh.T;
        need_eq = sh.need_eq;
    } else {  // every bit fixed: the threshold is the prefix itself
        thr = prefix;
        need_eq = kk;
    }
    uint64_t bg[B], be[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
        const bool ok = u * NT + tid < n;
        bg[u] = __ballot(ok && key[u] > thr);
        be[u] = __ballot(ok && key[u] == thr);
    }
    if (lane == 0) {
#pragma unroll
        for (int u = 0; u < B; ++u) {
            sh.tg[u * NW + wave] = (uint32_t)__popcll(bg[u]);
            sh.te[u * NW + wave] = (uint32_t)__popcll(be[u]);
        }
    }
    __syncthreads();
    if (wave == 0) table_exscan2<NW>(sh.tg, sh.te);
    __syncthreads();
    int32_t* rl = rowlist + s.sel_off;
    int32_t* sm = slotmap + s.row_off;
#pragma unroll
    for (int u = 0; u < B; ++u) {
        const int row = u * NT + tid;
        if (row < n) {
            const bool g = (bg[u] >> lane) & 1ull, e = (be[u] >> lane) & 1ull;
            const int64_t gp = sh.tg[u * NW + wave] + (uint32_t)__popcll(bg[u] & lt);
            const int64_t ep = sh.te[u * NW + wave] + (uint32_t)__popcll(be[u] & lt);
            if (g || (e && ep < need_eq)) {
                const int64_t slot = gp + (ep < need_eq ? ep : need_eq);
                if (slot < s.k_rows) rl[slot] = row;  // bound: never store past the row list
                sm[row] = (int32_t)slot;
            } else {
                sm[row] = -1;
            }
        }
    }
}

template <typename T, int NT>
__device__ __forceinline__ void select_small_seg(const SegDev* __restrict__ segs, int32_t seg_id,
                                                 const T* __restrict__ sketch, int R, Scale sc,
                                                 int32_t* __restrict__ rowlist,
                                                 int32_t* __restrict__ slotmap,
                                                 uint32_t* __restrict__ keys /* LDS, n + 4 */) {
    __shared__ SmallSel sh;
    const SegDev s = segs[seg_id];
    const int n = (int)s.n;
    if (n <= kRegB * NT) {
        select_small_reg<T, NT>(s, sketch, R, sc, rowlist, slotmap, sh);
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int stride = (s.kind == ARCTOPK_SEG_RAW) ? 1 : R;
    const T* sk = sketch + s.sketch_off;
    uint32_t kor = 0u, kand = ~0u;
    if (R == 4 && s.kind == ARCTOPK_SEG_SKETCH && (s.sketch_off & 3) == 0) {
        // one quad per row; 8 rows' loads in flight per thread before any use
        constexpr int B = 8;
        for (int base = 0; base < n; base += NT * B) {
            float4 v[B];
#pragma unroll
            for (int u = 0; u < B; ++u) v[u] = ldq<T, false>(sk, min(base + u * NT + tid, n - 1));
#pragma unroll
            for (int u = 0; u < B; ++u) {
                const int row = base + u * NT + tid;
                const uint32_t key = energy_key(energy4<T>(v[u].x, v[u].y, v[u].z, v[u].w, sc));
                if (row < n) {
                    keys[row] = key;
                    kor |= key;
                    kand &= key;
                }
            }
        }
    } else {
        for (int row = tid; row < n; row += NT) {
            const uint32_t key = energy_key(row_energy(sk + (int64_t)row * stride, R, sc, s.kind));
            keys[row] = key;
            kor |= key;
            kand &= key;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        kor |= __shfl_xor(kor, o, 64);
        kand &= __shfl_xor(kand, o, 64);
    }
    if (lane == 0) {
        sh.wor[wave] = kor;
        sh.wand[wave] = kand;
    }
    __syncthreads();
    kor = 0u;
    kand = ~0u;
#pragma unroll
    for (int w = 0; w < (NT / 64); ++w) {
        kor |= sh.wor[w];
        kand &= sh.wand[w];
    }
    // bits [bit-1 .. 0] still vary among matching keys
    const uint32_t diff = kor ^ kand;
    int bit = diff ? 32 - __clz(diff) : 0;
    uint32_t prefix = kand & ~((bit == 32) ? 0xFFFFFFFFu : ((1u << bit) - 1u));
    uint32_t mask = (bit == 32) ? 0u : ~((1u << bit) - 1u);
    int64_t kk = s.k_rows;
    bool ranked = false;
    while (bit > 0) {
        const int w = bit < 8 ? bit : 8;
        const int shift = bit - w;
        const uint32_t dmask = (1u << w) - 1u;
        for (int i = tid; i < 256; i += NT) sh.hist[i] = 0;
        __syncthreads();
        for (int i = tid; i < n; i += NT) {
            const uint32_t key = keys[i];
            if ((key & mask) == prefix) atomicAdd(&sh.hist[(key >> shift) & dmask], 1u);
        }
        __syncthreads();
        if (wave == 0) {  // lane l owns digits 255-4l .. 252-4l (descending)
            uint32_t c[4], sum = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c[q] = sh.hist[255 - 4 * lane - q];
                sum += c[q];
            }
            uint32_t incl = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            const uint32_t excl = incl - sum;
            if ((uint64_t)excl < (uint64_t)kk && (uint64_t)incl >= (uint64_t)kk) {
                uint32_t acc = excl;
                int q = 0;
                for (; q < 3; ++q) {
                    if ((uint64_t)(acc + c[q]) >= (uint64_t)kk) break;
                    acc += c[q];
                }
                sh.digit = 255 - 4 * lane - q;
                sh.dcount = c[q];
                sh.kk = kk - acc;
            }
        }
        __syncthreads();
        prefix |= sh.digit << shift;
        mask |= dmask << shift;
        kk = sh.kk;
        bit = shift;
        const uint32_t dcount = sh.dcount;
        __syncthreads();
        if (bit > 0 && dcount <= (uint32_t)kCandMax) {
            // rank the few keys of the threshold bin directly
            if (tid == 0) sh.ncand = 0;
            __syncthreads();
            // wave-aggregated append: one LDS atomic per wave and round, not per key
            const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
            for (int b0 = 0; b0 < n; b0 += NT) {
                const int i = b0 + tid;
                const uint32_t key = i < n ? keys[i] : 0u;
                const bool in = i < n && (key & mask) == prefix;
                const uint64_t bm = __ballot(in);
                uint32_t wb = 0;
                if (lane == 0 && bm) wb = atomicAdd(&sh.ncand, (uint32_t)__popcll(bm));
                wb = __shfl(wb, 0, 64);
                if (in) sh.cand[wb + (uint32_t)__popcll(bm & lt)] = key;
            }
            __syncthreads();
            const int nc = (int)sh.ncand;
            for (int i = nc + tid; i < ((nc + 3) & ~3); i += NT) sh.cand[i] = 0u;  // pad to x4
            __syncthreads();
            const uint4* c4 = reinterpret_cast<const uint4*>(sh.cand);
            for (int t = tid; t < nc; t += NT) {
                const uint32_t v = sh.cand[t];
                int gt = 0, ge = 0;
                const int nq = (nc + 3) >> 2;
#pragma unroll 4
                for (int j = 0; j < nq; ++j) {  // 16-B broadcast reads, 4 candidates each
                    const uint4 c = c4[j];
                    gt += (c.x > v) + (c.y > v) + (c.z > v) + (c.w > v);
                    ge += (c.x >= v) + (c.y >= v) + (c.z >= v) + (c.w >= v);
                }
                if (v == 0u) ge -= ((nc + 3) & ~3) - nc;  // zero padding equals v only when v == 0
                if (gt < kk && kk <= ge) {  // every writer writes the same (T, need)
                    sh.T = v;
                    sh.need_eq = kk - gt;
                }
            }
            __syncthreads();
            ranked = true;
            break;
        }
    }
    uint32_t thr;
    int64_t need_eq;
    if (ranked) {
        thr = sh.T;
        need_eq = sh.need_eq;
    } else {  // every bit fixed: the threshold is the prefix itself
        thr = prefix;
        need_eq = kk;
    }
    // index-ordered compaction over contiguous per-thread row ranges (multiples of 4
    // rows, read as 16-B LDS vectors; the key array is padded to a multiple of 4)
    const int per = (((n + NT - 1) / NT) + 3) & ~3;
    const int r0 = min(n, tid * per), r1 = min(n, r0 + per);
    int64_t gt = 0, eq = 0;
    for (int i = r0; i < r1; i += 4) {
        const uint4 q = *reinterpret_cast<const uint4*>(keys + i);
        const uint32_t kv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (i + u < r1) {
                gt += kv[u] > thr;
                eq += kv[u] == thr;
            }
        }
    }
    const int64_t eq_before = block_exscan_s(eq, sh.wsum);
    int64_t take_eq = need_eq - eq_before;
    take_eq = take_eq < 0 ? 0 : (take_eq > eq ? eq : take_eq);
    int64_t slot = block_exscan_s(gt + take_eq, sh.wsum);
    int32_t* rl = rowlist + s.sel_off;
    int32_t* sm = slotmap + s.row_off;
    int64_t eq_seen = 0;
    for (int i = r0; i < r1; i += 4) {
        const uint4 q = *reinterpret_cast<const uint4*>(keys + i);
        const uint32_t kv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (i + u < r1) {
                const uint32_t key = kv[u];
                bool sel = key > thr;
                if (key == thr) {
                    sel = eq_seen < take_eq;
                    ++eq_seen;
                }
                if (sel) {
                    if (slot < s.k_rows) rl[slot] = i + u;  // bound: never store past the row list
                    sm[i + u] = (int32_t)slot;
                    ++slot;
                } else {
                    sm[i + u] = -1;
                }
            }
        }
    }
}

template <typename T, int NT>
__global__ void __launch_bounds__(NT) k_select_small(const SegDev* __restrict__ segs,
                                                      const int32_t* __restrict__ seg_ids,
                                                      const T* __restrict__ sketch, int R,
                                                      Scale sc, int32_t* __restrict__ rowlist,
                                                      int32_t* __restrict__ slotmap, VDrawJob job) {
    if (maybe_draw_v<T>(job, NT)) return;  // trailing blocks: the next call's projections
    extern __shared__ __attribute__((aligned(16))) uint32_t keys[];
    select_small_seg<T, NT>(segs, seg_ids[blockIdx.x], sketch, R, sc, rowlist, slotmap, keys);
}

// exclusive block scan of one uint32 per thread (NW waves); *total = block sum
template <int NW>
__device__ __forceinline__ uint32_t blk_exscan_u32(uint32_t v, uint32_t* lds, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wave] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint32_t v2 = lds[w];
        before += w < wave ? v2 : 0u;
        tot += v2;
    }
    __syncthreads();
    *total = tot;
    return before + x - v;
}

// LDS histogram add, all lanes of the wave (contrib: the lane adds to `bin`).  The lanes
// sharing the first contributing lane's bin add once for all: candidates of a degenerate bin
// (e.g. tied all-zero rows) all hit one word, and one-lane-at-a-time LDS atomics on it
// serialised the radix rounds (~90 us for a Llama embedding with 90 % zero rows).
__device__ __forceinline__ void hist_add_wave(uint32_t* h, uint32_t bin, bool contrib) {
    const uint64_t bm = __ballot(contrib);
    if (!bm) return;
    const int leader = __ffsll((long long)bm) - 1;
    const uint32_t lb = __shfl(bin, leader, 64);
    const uint64_t same = __ballot(contrib && bin == lb);
    if ((int)(threadIdx.x & 63) == leader) atomicAdd(&h[lb], (uint32_t)__popcll(same));
    if (contrib && bin != lb) atomicAdd(&h[bin], 1u);
}

// Decide at once the undecided bits that every candidate shares (kor / kand: OR / AND of the
// candidates, which all match s's prefix): a bin of tied keys (all-zero rows) then needs no
// radix round at all, and s.bit == 0 means every candidate equals the threshold.
__device__ __forceinline__ void decide_common_bits(MState& s, uint32_t kor, uint32_t kand) {
    const uint32_t diff = kor ^ kand;
    const int hb = diff ? 32 - __clz(diff) : 0;
    if (hb < s.bit) {
        const uint32_t above = s.bit >= 32 ? ~0u : ((1u << s.bit) - 1u);
        const uint32_t bits = above & ~((1u << hb) - 1u);  // [hb, s.bit)
        s.prefix |= kand & bits;
        s.mask |= bits;
        s.bit = hb;
    }
}

// two exclusive block scans plus a block-wide OR / AND (kor, kand in place), one pair of
// barriers (lds: 4 * NW words)
template <int NW>
__device__ __forceinline__ void blk_exscan2_or_and(uint32_t a, uint32_t b, uint32_t& kor, uint32_t& kand,
                                                   uint32_t* lds, uint32_t* ea, uint32_t* eb, uint32_t* ta,
                                                   uint32_t* tb) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = a, y = b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t xo = __shfl_up(x, o, 64), yo = __shfl_up(y, o, 64);
        if (lane >= o) {
            x += xo;
            y += yo;
        }
        kor |= __shfl_xor(kor, o, 64);
        kand &= __shfl_xor(kand, o, 64);
    }
    if (lane == 63) {
        lds[wave] = x;
        lds[NW + wave] = y;
        lds[2 * NW + wave] = kor;
        lds[3 * NW + wave] = kand;
    }
    __syncthreads();
    uint32_t bx = 0, by = 0, sx = 0, sy = 0, o_ = 0u, a_ = ~0u;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint32_t vx = lds[w], vy = lds[NW + w];
        bx += w < wave ? vx : 0u;
        by += w < wave ? vy : 0u;
        sx += vx;
        sy += vy;
        o_ |= lds[2 * NW + w];
        a_ &= lds[3 * NW + w];
    }
    __syncthreads();
    *ea = bx + x - a;
    *eb = by + y - b;
    *ta = sx;
    *tb = sy;
    kor = o_;
    kand = a_;
}

// two exclusive block scans with one pair of barriers (lds: 2 * NW words)
template <int NW>
__device__ __forceinline__ void blk_exscan_u32x2(uint32_t a, uint32_t b, uint32_t* lds, uint32_t* ea,
                                                 uint32_t* eb, uint32_t* ta, uint32_t* tb) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = a, y = b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t xo = __shfl_up(x, o, 64), yo = __shfl_up(y, o, 64);
        if (lane >= o) {
            x += xo;
            y += yo;
        }
    }
    if (lane == 63) {
        lds[wave] = x;
        lds[NW + wave] = y;
    }
    __syncthreads();
    uint32_t bx = 0, by = 0, sx = 0, sy = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint32_t vx = lds[w], vy = lds[NW + w];
        bx += w < wave ? vx : 0u;
        by += w < wave ? vy : 0u;
        sx += vx;
        sy += vy;
    }
    __syncthreads();
    *ea = bx + x - a;
    *eb = by + y - b;
    *ta = sx;
    *tb = sy;
}

// ARC refine of one large segment (after ms_arc_compact), one 1024-thread block.  Range r's
// candidates (every key of the first-pass bin in that range, in index order) sit in its
// own region of the candidate list; a block scan of the per-range counts lays them out
// back to back, and they are staged in LDS (read from their regions when they do not fit).
// Two 10-bit LDS histogram rounds fix the remaining bits of the threshold T; each thread
// then counts its range's candidates above / equal to T, and with the keys above the bin
// (compact pass) these become per-range T-equal allowances (lowest ranges first) and
// output offsets for ms_arc_write.  No atomics outside LDS histograms.
constexpr int kRefineThreads = 1024;
#ifndef ARCTOPK_REFINE_PRE
#define ARCTOPK_REFINE_PRE 64  // tuning switch (A/B builds): candidates per range loaded up front, 64 or 128
#endif
constexpr int kRefinePre = ARCTOPK_REFINE_PRE;
#ifndef ARCTOPK_REFINE_UT
#define ARCTOPK_REFINE_UT 4  // tuning switch (A/B builds): tail candidates loaded per thread and round
#endif
static_assert(kRefineThreads == kMMaxRanges, "one range per thread in the offset scan");
__device__ __forceinline__ void arc_refine_item(const MBatch& b, int t, MWorkspace* ws,
                                                const uint32_t* __restrict__ ckey,
                                                uint32_t* __restrict__ stage /* LDS */) {
    constexpr int NT = kRefineThreads, NW = NT / 64, U = 8, W2 = 10;
    __shared__ uint32_t h[1 << W2];
    __shared__ uint32_t roff[kMMaxRanges], rcnt[kMMaxRanges];  // later: per-range (eq, gt) counts
    __shared__ uint32_t toff[kMMaxRanges];  // tail offsets while staging; later: per-range eq counts
    __shared__ uint32_t lds[NW], lds2[4 * NW], s_digit, s_acc;
    constexpr int RB = 16;  // ranges per wave whose first candidates load up front
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const MItem it = b.it[t];
    const uint32_t* src = ckey + it.cand_off;
    // one round trip for everything independent: the state, the per-range counts, and the
    // first 64 candidate slots of each range this wave copies (a range's region is fixed;
    // its count only masks them)
    MState s = ws->st[t];  // the first-pass bin (compact launch / key pass)
    const int nr = it.nranges;
    // loaded for every thread (NT == kMMaxRanges: in bounds) so that they need not wait for
    // `it`; entries past nr are masked below
    const uint32_t gt_raw = ws->cnt_gt[t][tid], cnt_raw = ws->cnt_cand[t][tid];
    const uint32_t or_raw = ws->cand_or[t][tid], and_raw = ws->cand_and[t][tid];
    uint32_t v[RB];  // candidate slots lane and lane + 64 of each range
    [[maybe_unused]] uint32_t v2[RB];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
        const int r = wave + q * NW;
        const int64_t cap = r < nr ? min<int64_t>(kRefinePre, it.n - (int64_t)r * it.range) : 0;  // region bound
        v[q] = lane < cap ? src[(int64_t)r * it.range + lane] : 0u;
        if constexpr (kRefinePre > 64) v2[q] = lane + 64 < cap ? src[(int64_t)r * it.range + 64 + lane] : 0u;
    }
    // every reader of the key pass's histogram (the compact launch) is done: zero it for the
    // next key pass
    for (int i = tid; i < kMBins; i += NT) ws->hist[t][i] = 0u;
    const uint32_t gt_above = tid < nr ? gt_raw : 0u;  // keys above the bin
    const uint32_t my_cnt = tid < nr ? cnt_raw : 0u;
    const uint32_t my_tail = my_cnt > (uint32_t)kRefinePre ? my_cnt - (uint32_t)kRefinePre : 0u;
    uint32_t nc32, ntail, my_off, my_toff;
    uint32_t kor = tid < nr ? or_raw : 0u, kand = tid < nr ? and_raw : ~0u;
    blk_exscan2_or_and<NW>(my_cnt, my_tail, kor, kand, lds2, &my_off, &my_toff, &nc32, &ntail);
    roff[tid] = my_off;
    rcnt[tid] = my_cnt;
    toff[tid] = my_toff;
    __syncthreads();
    decide_common_bits(s, kor, kand);
    const bool all_eq = s.bit == 0;  // every candidate equals the threshold
    const int64_t nc = nc32;
    // last r in [0, nr) with a[r] <= p: the range holding the p-th entry of an exclusive scan
    // (ranges with nothing share their successor's offset; the last of equals holds p)
    auto range_of = [&](const uint32_t* a, uint32_t p) -> int {
        int lo = 0, hi = nr - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (a[mid] <= p) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    // global index of candidate p (p-th in range order)
    auto gidx = [&](uint32_t p) -> int64_t {
        const int lo = range_of(roff, p);
        return (int64_t)lo * it.range + (p - roff[lo]);
    };
    const bool staged = !all_eq && nc <= kRefineLdsCap;
    if (staged) {
        // usual case: wave w copies ranges w, w + NW, ..., lane j candidate j (and j + 64)
        // of each (the first RB ranges' first kRefinePre candidates are already in
        // registers; ranges past NW * RB load here); the tails past kRefinePre follow as one
        // flat list with UT loads in flight per thread (a per-range loop would chain one
        // round trip per range); then everything is read from LDS
        for (int r0 = wave; r0 < nr; r0 += NW * RB) {
            if (r0 != wave) {
#pragma unroll
                for (int q = 0; q < RB; ++q) {
                    const int r = r0 + q * NW;
                    const uint32_t c = r < nr ? rcnt[r] : 0u;
                    v[q] = (uint32_t)lane < c ? src[(int64_t)r * it.range + lane] : 0u;
                    if constexpr (kRefinePre > 64) v2[q] = (uint32_t)lane + 64 < c ? src[(int64_t)r * it.range + 64 + lane] : 0u;
                }
            }
#pragma unroll
            for (int q = 0; q < RB; ++q) {
                const int r = r0 + q * NW;
                if (r < nr) {
                    const uint32_t c = rcnt[r], o = roff[r];
                    if ((uint32_t)lane < c) stage[o + lane] = v[q];
                    if constexpr (kRefinePre > 64) if ((uint32_t)lane + 64 < c) stage[o + 64 + lane] = v2[q];
                }
            }
        }
        constexpr int UT = ARCTOPK_REFINE_UT;
        for (uint32_t p0 = 0; p0 < ntail; p0 += (uint32_t)NT * UT) {
            uint32_t kv[UT], dst[UT];
#pragma unroll
            for (int u = 0; u < UT; ++u) {
                const uint32_t p = p0 + (uint32_t)(u * NT + tid);
                if (p < ntail) {
                    const int r = range_of(toff, p);
                    const uint32_t j = (uint32_t)kRefinePre + (p - toff[r]);
                    kv[u] = src[(int64_t)r * it.range + j];
                    dst[u] = roff[r] + j;
                }
            }
#pragma unroll
            for (int u = 0; u < UT; ++u)
                if (p0 + (uint32_t)(u * NT + tid) < ntail) stage[dst[u]] = kv[u];
        }
        __syncthreads();
    }
    auto key_at = [&](int64_t i) -> uint32_t { return staged ? stage[i] : src[gidx((uint32_t)i)]; };
    while (s.bit > 0) {
        const int w = s.bit < W2 ? s.bit : W2;
        const int shift = s.bit - w;
        const uint32_t dmask = (1u << w) - 1u;
        h[tid] = 0u;  // 1 << W2 == NT bins
        __syncthreads();
        for (int64_t base = 0; base < nc; base += (int64_t)NT * U) {
            uint32_t kv[U];  // all loads of a batch in flight before the LDS atomics
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = base + u * NT + tid;
                kv[u] = i < nc ? key_at(i) : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = base + u * NT + tid;
                hist_add_wave(h, (kv[u] >> shift) & dmask, i < nc && (kv[u] & s.mask) == s.prefix);
            }
        }
        __syncthreads();
        const int nb = 1 << w;
        const uint32_t c = tid < nb ? h[nb - 1 - tid] : 0u;  // descending bins
        uint32_t total;
        const uint32_t excl = blk_exscan_u32<NW>(c, lds, &total);
        if ((uint64_t)excl < (uint64_t)s.kk && (uint64_t)excl + c >= (uint64_t)s.kk) {
            s_digit = (uint32_t)(nb - 1 - tid);
            s_acc = excl;
        }
        __syncthreads();
        s.prefix |= s_digit << shift;
        s.mask |= dmask << shift;
        s.kk -= (int64_t)s_acc;
        s.bit = shift;
        __syncthreads();  // s_digit / s_acc / h are rewritten by the next round
    }
    const uint32_t T = s.prefix;
    const uint32_t* cgt;  // per-range candidates above / equal to T
    const uint32_t* ceq;
    if (all_eq) {
        h[tid] = 0u;
        cgt = h;
        ceq = rcnt;
    } else if (staged) {
        // thread per contiguous run of the staged list (an odd run length keeps the lanes'
        // LDS reads on distinct banks); counts go to LDS per range when the run crosses into
        // the next range (h: gt, toff: eq -- both free now)
        h[tid] = 0u;
        toff[tid] = 0u;
        __syncthreads();
        const uint32_t per = ((nc32 + NT - 1) / NT) | 1u;
        const uint32_t p0 = (uint32_t)tid * per, p1 = min(nc32, p0 + per);
        if (p0 < p1) {
            int r = range_of(roff, p0);
            uint32_t rend = r + 1 < nr ? roff[r + 1] : nc32;
            uint32_t g = 0, e = 0;
            for (uint32_t p = p0; p < p1; ++p) {
                while (p >= rend) {
                    if (g) atomicAdd(&h[r], g);
                    if (e) atomicAdd(&toff[r], e);
                    g = e = 0;
                    ++r;
                    rend = r + 1 < nr ? roff[r + 1] : nc32;
                }
                const uint32_t k = stage[p];
                g += k > T ? 1u : 0u;
                e += k == T ? 1u : 0u;
            }
            if (g) atomicAdd(&h[r], g);
            if (e) atomicAdd(&toff[r], e);
        }
        cgt = h;
        ceq = toff;
    } else {
        // wave per range: its candidates above / equal to T by ballots; the counts replace
        // the range's (count, offset) entries (read first, by the same wave)
        for (int r = wave; r < nr; r += NW) {
            const uint32_t c = rcnt[r];
            uint32_t g = 0, e = 0;
            for (uint32_t j0 = 0; j0 < c; j0 += 64) {
                const uint32_t j = j0 + (uint32_t)lane;
                const uint32_t k = j < c ? src[(int64_t)r * it.range + j] : 0u;
                g += (uint32_t)__popcll(__ballot(j < c && k > T));
                e += (uint32_t)__popcll(__ballot(j < c && k == T));
            }
            if (lane == 0) {
                rcnt[r] = g;
                roff[r] = e;
            }
        }
        cgt = rcnt;
        ceq = roff;
    }
    __syncthreads();
    const int r = tid;
    const uint32_t gt = (tid < nr ? cgt[tid] : 0u) + gt_above;
    const uint32_t eq = tid < nr ? ceq[tid] : 0u;
    uint32_t tot;
    const uint32_t eq_before = blk_exscan_u32<NW>(eq, lds, &tot);
    int64_t take = s.kk - (int64_t)eq_before;
    take = take < 0 ? 0 : (take > (int64_t)eq ? (int64_t)eq : take);
    const uint32_t sel_before = blk_exscan_u32<NW>(gt + (uint32_t)take, lds, &tot);
    if (r < nr) {
        ws->take_eq[t][r] = (uint32_t)take;
        ws->sel_before[t][r] = sel_before;
    }
    if (tid == 0) {
        ws->st[t] = s;  // the write pass reads the threshold (prefix)
    }
}

// The refine of a batch's large segments and, in the same launch, the single-block selects
// of the small segments (blocks b.cnt ..): both are latency-bound and independent, so they
// overlap instead of running back to back.  Trailing blocks may draw the next call's
// projections (VDrawJob).
template <typename T>
__global__ void __launch_bounds__(kRefineThreads) k_arc_refine(const MBatch* __restrict__ bp, int nitems,
                                                               MWorkspace* ws,
                                                               const uint32_t* __restrict__ ckey,
                                                               const SegDev* __restrict__ segs,
                                                               const int32_t* __restrict__ small_ids,
                                                               const T* __restrict__ sketch, int R,
                                                               Scale sc, int32_t* __restrict__ rowlist,
                                                               int32_t* __restrict__ slotmap,
                                                               VDrawJob job) {
    if (maybe_draw_v<T>(job, kRefineThreads)) {
        return;
    }
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
    if ((int)blockIdx.x < nitems) {
        arc_refine_item(*bp, (int)blockIdx.x, ws, ckey, dyn);
    }
    else
        select_small_seg<T, kRefineThreads>(segs, small_ids[blockIdx.x - nitems], sketch, R, sc, rowlist,
                                            slotmap, dyn);
}

// ---- the refine folded into the write pass (items of up to kFuseMaxRows rows) ----
// k_arc_refine is one block per item: a chain of cold round trips (~11 us on ResNet-18's
// 131 K-row items) between the compact and write launches.  For items whose candidate lists
// are a few thousand keys, every write block (one per range, as k_arc_write) re-derives the
// threshold itself instead: it stages the item's candidates in LDS, runs the same two 10-bit
// rounds, counts the candidates of the ranges before its own, and writes its range.  The
// selection is the same exact top-k (same T, same lowest-range-first T-equal allowances).
constexpr int kFuseCap = ARCTOPK_FUSE_CAP;  // staged candidates per block (32 KiB of LDS at 8,192)
constexpr int64_t kFuseMaxRows = ARCTOPK_FUSE_MAX_ROWS;  // host rule: largest item of a fused batch
constexpr int kFuseNT = 256;
constexpr int kFuseMaxBlocks = 512;         // host rule: two blocks per CU (LDS allows three)

// range r of item t, one range per block (spans of several consecutive ranges per block, the
// refine paid once per span, measured slower in rounds 3 and 4 and removed)
__device__ __forceinline__ void arc_write_fused_range(const MItem it, int t, int r,
                                                      const uint32_t* __restrict__ keys,
                                                      MWorkspace* ws, const uint32_t* __restrict__ ckey,
                                                      int32_t* __restrict__ out_idx, int32_t* __restrict__ out_slot,
                                                      uint32_t* __restrict__ stage /* LDS, kFuseCap */) {
    constexpr int NT = kFuseNT, NW = NT / 64, PR = kMMaxRanges / NT, W2 = 10, NB = 1 << W2, PB = NB / NT;
    constexpr int kPer = kMTile / 256;  // keys per lane of a write tile
    __shared__ uint32_t h[NB];
    __shared__ uint32_t roff[kMMaxRanges];
    __shared__ uint32_t lds[4 * NW], s_digit, s_acc, s_eq[NW], s_gt[NW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int nr = it.nranges;
    const uint32_t* src = ckey + it.cand_off;
    const int64_t r0 = (int64_t)r * it.range;
    const int64_t r1 = min<int64_t>(it.n, r0 + it.range);
    // one round trip: the first-pass state, the per-range counts and this range's first tile
    MState s = ws->st[t];
    uint32_t cc[PR], cg[PR], kor = 0u, kand = ~0u;
#pragma unroll
    for (int q = 0; q < PR; ++q) {
        const int rr = tid * PR + q;
        cc[q] = rr < nr ? ws->cnt_cand[t][rr] : 0u;
        cg[q] = rr < r ? ws->cnt_gt[t][rr] : 0u;  // keys above the bin, ranges before r
        kor |= rr < nr ? ws->cand_or[t][rr] : 0u;
        kand &= rr < nr ? ws->cand_and[t][rr] : ~0u;
    }
    const int64_t wb0 = r0 + (int64_t)wave * (kMTile / 4);
    uint32_t kv[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) kv[j] = keys[it.key_off + min<int64_t>(wb0 + j * 64 + lane, r1 - 1)];
    if (r == 0)  // the compact launch was the last reader of the key pass's histogram
        for (int i = tid; i < kMBins; i += NT) ws->hist[t][i] = 0u;
    uint32_t csum = 0, gsum = 0;
#pragma unroll
    for (int q = 0; q < PR; ++q) {
        csum += cc[q];
        gsum += cg[q];
    }
    uint32_t cbase, gdummy, nc32, gabove;
    blk_exscan2_or_and<NW>(csum, gsum, kor, kand, lds, &cbase, &gdummy, &nc32, &gabove);
#pragma unroll
    for (int q = 0; q < PR; ++q) {
        roff[tid * PR + q] = cbase;
        cbase += cc[q];
    }
    __syncthreads();
    decide_common_bits(s, kor, kand);
    const bool all_eq = s.bit == 0;  // every candidate equals the threshold
    const bool staged = !all_eq && nc32 <= (uint32_t)kFuseCap;
    if (staged) {
        constexpr int UT = 8;
        int rr = 0;  // range of the lane's current candidate: positions only grow
        for (uint32_t p0 = 0; p0 < nc32; p0 += (uint32_t)NT * UT) {
            uint32_t v[UT];
#pragma unroll
            for (int u = 0; u < UT; ++u) {
                const uint32_t p = p0 + (uint32_t)(u * NT + tid);
                if (p < nc32) {
                    while (rr + 1 < nr && roff[rr + 1] <= p) ++rr;
                    v[u] = src[(int64_t)rr * it.range + (p - roff[rr])];
                } else {
                    v[u] = 0u;
                }
            }
#pragma unroll
            for (int u = 0; u < UT; ++u) {
                const uint32_t p = p0 + (uint32_t)(u * NT + tid);
                if (p < nc32) stage[p] = v[u];
            }
        }
        __syncthreads();
    }
    // f(p, key) for candidates p < lim: from LDS, or (more than kFuseCap candidates, e.g. a
    // bin of tied zero rows) from their regions with UG loads in flight per thread
    auto sweep = [&](uint32_t lim, auto&& f) {
        if (staged) {
            for (uint32_t p0 = 0; p0 < lim; p0 += (uint32_t)NT * 8) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t p = p0 + (uint32_t)(u * NT + tid);
                    v[u] = p < lim ? stage[p] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t p = p0 + (uint32_t)(u * NT + tid);
                    f(p, v[u], p < lim);  // every lane (f may use wave operations)
                }
            }
        } else {
            constexpr int UG = 32;
            int rr = 0;  // range of the lane's current candidate: positions only grow
            for (uint32_t p0 = 0; p0 < lim; p0 += (uint32_t)NT * UG) {
                uint32_t v[UG];
#pragma unroll
                for (int u = 0; u < UG; ++u) {
                    const uint32_t p = p0 + (uint32_t)(u * NT + tid);
                    if (p < lim) {
                        while (rr + 1 < nr && roff[rr + 1] <= p) ++rr;
                        v[u] = src[(int64_t)rr * it.range + (p - roff[rr])];
                    } else {
                        v[u] = 0u;
                    }
                }
#pragma unroll
                for (int u = 0; u < UG; ++u) {
                    const uint32_t p = p0 + (uint32_t)(u * NT + tid);
                    f(p, v[u], p < lim);
                }
            }
        }
    };
    while (s.bit > 0) {
        const int w = s.bit < W2 ? s.bit : W2;
        const int shift = s.bit - w;
        const uint32_t dmask = (1u << w) - 1u;
#pragma unroll
        for (int q = 0; q < PB; ++q) h[q * NT + tid] = 0u;
        __syncthreads();
        const uint32_t pm = s.mask, pp = s.prefix;
        sweep(nc32, [&](uint32_t, uint32_t k, bool ok) {
            hist_add_wave(h, (k >> shift) & dmask, ok && (k & pm) == pp);
        });
        __syncthreads();
        const int nb = 1 << w;
        const int per = (nb + NT - 1) / NT;  // bins per thread, consecutive from the top
        uint32_t c[PB], sum = 0;
#pragma unroll
        for (int q = 0; q < PB; ++q) {
            const int bin = nb - 1 - (tid * per + q);
            c[q] = (q < per && bin >= 0) ? h[bin] : 0u;
            sum += c[q];
        }
        uint32_t total;
        const uint32_t excl = blk_exscan_u32<NW>(sum, lds, &total);
        if ((uint64_t)excl < (uint64_t)s.kk && (uint64_t)excl + sum >= (uint64_t)s.kk) {
            uint32_t acc = excl;
            int q = 0;
            for (; q < per - 1; ++q) {
                if ((uint64_t)acc + c[q] >= (uint64_t)s.kk) break;
                acc += c[q];
            }
            s_digit = (uint32_t)(nb - 1 - (tid * per + q));
            s_acc = acc;
        }
        __syncthreads();
        s.prefix |= s_digit << shift;
        s.mask |= dmask << shift;
        s.kk -= (int64_t)s_acc;
        s.bit = shift;
        __syncthreads();  // s_digit / s_acc / h are rewritten by the next round
    }
    const uint32_t T = s.prefix;
    // candidates before this range (> T, == T) and this range's == T
    const uint32_t cb = roff[r], ce = r + 1 < nr ? roff[r + 1] : nc32;
    uint32_t gb = 0, eb = 0, eo = 0;
    if (all_eq) {  // no candidate above T; every one ties with it
        if (tid == 0) {
            eb = cb;
            eo = ce - cb;
        }
    } else sweep(ce, [&](uint32_t p, uint32_t k, bool ok) {
        if (!ok) return;
        if (p < cb) {
            gb += k > T ? 1u : 0u;
            eb += k == T ? 1u : 0u;
        } else {
            eo += k == T ? 1u : 0u;
        }
    });
    uint32_t x0, x1, tgb, teb;
    blk_exscan_u32x2<NW>(gb, eb, lds, &x0, &x1, &tgb, &teb);
    uint32_t teo;
    (void)blk_exscan_u32<NW>(eo, lds, &teo);
    const int64_t kk = s.kk;
    int64_t take = kk - (int64_t)teb;
    take = take < 0 ? 0 : (take > (int64_t)teo ? (int64_t)teo : take);
    uint32_t take_left = (uint32_t)take;
    int64_t run = (int64_t)gabove + tgb + min<int64_t>(kk, (int64_t)teb);
    // the write of this range (k_arc_write's body): ballot compaction in index order
    for (int64_t tile = r0; tile < r1; tile += kMTile) {
        const int64_t wb = tile + (int64_t)wave * (kMTile / 4);
        if (tile != r0) {
#pragma unroll
            for (int j = 0; j < kPer; ++j) kv[j] = keys[it.key_off + min<int64_t>(wb + j * 64 + lane, r1 - 1)];
        }
        uint32_t weq = 0, wgt = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const bool valid = wb + j * 64 + lane < r1;
            weq += (uint32_t)__popcll(__ballot(valid && kv[j] == T));
            wgt += (uint32_t)__popcll(__ballot(valid && kv[j] > T));
        }
        if (lane == 0) {
            s_eq[wave] = weq;
            s_gt[wave] = wgt;
        }
        __syncthreads();
        uint32_t eqb = 0, gtb = 0, teq = 0, tgt = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            eqb += w < wave ? s_eq[w] : 0u;
            gtb += w < wave ? s_gt[w] : 0u;
            teq += s_eq[w];
            tgt += s_gt[w];
        }
        __syncthreads();
        uint32_t run_eq = eqb;
        int64_t run_sel = run + gtb + min(eqb, take_left);
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int64_t i = wb + j * 64 + lane;
            const bool valid = i < r1;
            const bool eq = valid && kv[j] == T;
            const bool gt = valid && kv[j] > T;
            const uint64_t beq = __ballot(eq);
            const bool sel = gt || (eq && run_eq + (uint32_t)__popcll(beq & lt) < take_left);
            const uint64_t bsel = __ballot(sel);
            const int64_t my = run_sel + (int64_t)__popcll(bsel & lt);
            if (sel && my < it.k) out_idx[it.out_off + my] = (int32_t)i;  // bound: never past k
            if (valid) out_slot[it.slot_off + i] = sel ? (int32_t)my : -1;
            run_eq += (uint32_t)__popcll(beq);
            run_sel += (int64_t)__popcll(bsel);
        }
        const uint32_t te = min(teq, take_left);
        run += tgt + te;
        take_left -= te;
    }
}

// A deferred decode (an earlier bucket's, arctopk_exchange_step's `ride`) riding in a launch of
// the current bucket's select: its chunks run as extra 256-thread blocks after the select's own
// (latency-bound) blocks, so the select's latency hides behind the decode's HBM stream.
template <typename T>
struct DecodeRide {
    const SegDev* segs;
    const Chunk* chunks;
    const int32_t* dfirst;  // the chunk table (mode 3)
    const T* packed;
    const int32_t* slotmap;
    T* gE;
    T* out;
    Scale sc;
    int32_t n;    // chunks (blocks); 0: none
    int32_t fin;  // world size 1, pack and decode fused (finalize_chunk): 1 EF14, 2 noef; 0: decode
    T* E;         // (fin) the residual the selected rows are taken from
};

// World size 1, pack + decode in one pass (no packed buffer): the all-reduce is the identity, so
// the decoded bucket is the selected rows' values (x / 1, exact) and zero elsewhere.  EF14: out :=
// E on selected rows, 0 elsewhere, and the selected rows of E := 0 (what k_pack then k_decode
// leave); noef: out is the bucket itself (G, in place), whose unselected elements become 0.  One
// decode chunk (its row range) per 256-thread block.
template <typename T>
__device__ __forceinline__ void finalize_chunk(const SegDev* __restrict__ segs, const Chunk ch,
                                               const int32_t* __restrict__ slotmap, T* __restrict__ E,
                                               T* __restrict__ out, int fin, Scale sc) {
    // the decode's own arithmetic on the selected values (x / 1, rounded to T: bit-identical to
    // k_decode's output from the packed copy, NaNs included)
    auto mean4 = [&](float4 v) { return rnd4<T>(sc(v)); };
    auto mean1 = [&](float v) { return rnd<T>(sc(v)); };
    const SegDev s = segs[ch.seg];
    const int m = (int)s.m;
    const int64_t base = s.offset + ch.row0 * m;
    const int32_t* sm = slotmap + s.row_off + ch.row0;
    const int nr = (int)ch.nrows;
    const bool ef14 = fin == 1;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (s.vec && m >= 256) {  // wave per row, 16-B units: a selected row is copied, the rest zeroed
        constexpr int PQ = kQuadsPer16<T>;  // quads per 16-B unit (fp32 1, bf16 2)
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, mu = m / (4 * PQ);
        constexpr int U = 4;
        float4 zu[PQ];
#pragma unroll
        for (int h = 0; h < PQ; ++h) zu[h] = z4;
        for (int j = wave; j < nr; j += 4) {
            const bool sel = sm[j] >= 0;
            T* op = out + base + (int64_t)j * m;
            T* ep = E + base + (int64_t)j * m;
            if (ef14 && sel) {
                for (int c0 = 0; c0 < mu; c0 += 64 * U) {
                    float4 v[U][PQ];
#pragma unroll
                    for (int u = 0; u < U; ++u) ld16<T, kNtDecode>(ep, min(c0 + u * 64 + lane, mu - 1), v[u]);
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int c = c0 + u * 64 + lane;
                        if (c < mu) {
#pragma unroll
                            for (int h = 0; h < PQ; ++h) v[u][h] = mean4(v[u][h]);
                            st16<T, kNtDecode>(op, c, v[u]);
                            st16<T, kNtDecode>(ep, c, zu);
                        }
                    }
                }
            } else if (!sel) {
                for (int c = lane; c < mu; c += 64) st16<T, kNtDecode>(op, c, zu);
            }
        }
        return;
    }
    // other rows: the chunk's elements as 16-B quads (scalar edges), each element's row from the
    // slot map
    const int64_t cnt = (int64_t)nr * m;
    auto row_of = [&](int64_t e) -> int { return m == 1 ? (int)e : (int)div32((uint32_t)e, s.magic32); };
    auto one = [&](int64_t e) {
        const bool sel = sm[row_of(e)] >= 0;
        if (ef14) {
            float v = 0.f;
            if (sel) {
                v = mean1(ld1<T>(E + base + e));
                st1<T>(E + base + e, 0.f);
            }
            st1<T>(out + base + e, v);
        } else if (!sel) {
            st1<T>(out + base + e, 0.f);
        }
    };
    const int64_t pre = min<int64_t>(cnt, (4 - (base & 3)) & 3);
    for (int64_t e = threadIdx.x; e < pre; e += 256) one(e);
    const int64_t nq = (cnt - pre) >> 2;
    constexpr int UQ = 4;
    for (int64_t q0 = threadIdx.x; q0 < nq; q0 += 256 * UQ) {
        bool sl[UQ][4];
        float4 ev[UQ];
#pragma unroll
        for (int u = 0; u < UQ; ++u) {
            const int64_t e = pre + 4 * min<int64_t>(q0 + u * 256, nq - 1);
            bool any = false;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                sl[u][j] = sm[row_of(e + j)] >= 0;
                any = any || sl[u][j];
            }
            // EF14: the residual quad when any element is selected; noef: the bucket's own quad
            // when it is partly selected (its unselected elements are zeroed in place)
            const bool all = sl[u][0] && sl[u][1] && sl[u][2] && sl[u][3];
            ev[u] = (ef14 ? any : (any && !all)) ? ldq<T, false>((ef14 ? E : out) + base + e, 0) : z4;
        }
#pragma unroll
        for (int u = 0; u < UQ; ++u) {
            if (q0 + u * 256 >= nq) break;
            const int64_t e = pre + 4 * (q0 + u * 256);
            const bool* q = sl[u];
            const bool any = q[0] || q[1] || q[2] || q[3], all = q[0] && q[1] && q[2] && q[3];
            const float4 v = make_float4(q[0] ? ev[u].x : 0.f, q[1] ? ev[u].y : 0.f, q[2] ? ev[u].z : 0.f,
                                         q[3] ? ev[u].w : 0.f);
            if (ef14) {
                stq<T, kNtDecode>(out + base + e, 0, mean4(v));
                if (any)
                    stq<T, false>(E + base + e, 0, make_float4(q[0] ? 0.f : ev[u].x, q[1] ? 0.f : ev[u].y,
                                                               q[2] ? 0.f : ev[u].z, q[3] ? 0.f : ev[u].w));
            } else if (!all) {
                stq<T, false>(out + base + e, 0, v);
            }
        }
    }
    for (int64_t e = pre + 4 * nq + threadIdx.x; e < cnt; e += 256) one(e);
}
template <typename T, int EF>
__device__ __forceinline__ void decode_chunk(const SegDev* __restrict__ segs, const Chunk ch,
                                             const int32_t* __restrict__ dfc,
                                             const T* __restrict__ packed,
                                             const int32_t* __restrict__ slotmap, Scale sc,
                                             T* __restrict__ gE, T* __restrict__ out,
                                             float* __restrict__ dlds);
// The decode of a bucket that is already zero (fin 3: exchange.cpp zeroed it while its packed
// values were on the wire, EF14 / noef): only the selected rows are written, with the values
// decode_chunk writes there (the mean of the all-reduced row, rounded to T); every other element
// keeps the +0 that decode_chunk would have written.
template <typename T>
__device__ __forceinline__ void scatter_chunk(const SegDev* __restrict__ segs, const Chunk ch,
                                              const T* __restrict__ packed, const int32_t* __restrict__ slotmap,
                                              T* __restrict__ out, Scale sc) {
    auto mean4 = [&](float4 v) { return rnd4<T>(sc(v)); };
    auto mean1 = [&](float v) { return rnd<T>(sc(v)); };
    const SegDev s = segs[ch.seg];
    const int m = (int)s.m;
    const int64_t base = s.offset + ch.row0 * m;
    const int32_t* sm = slotmap + s.row_off + ch.row0;
    const T* pk = packed + s.packed_off;
    if (s.vec && m >= 256) {  // decode_chunk's row path: wave per selected row, float4 streams
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, m4 = m >> 2;
        for (int64_t j = wave; j < ch.nrows; j += 4) {
            const int32_t slot = sm[j];
            if (slot < 0) continue;
            const T* pp = pk + (int64_t)slot * m;
            T* op = out + base + j * m;
#pragma unroll 4
            for (int c = lane; c < m4; c += 64) stq<T, kNtDecode>(op, c, mean4(ldq<T, false>(pp, c)));
        }
        return;
    }
    // shorter rows: thread per element of the chunk, the selected ones stored
    const int64_t cnt = ch.nrows * m;
    for (int64_t e = threadIdx.x; e < cnt; e += 256) {
        const int row = m == 1 ? (int)e : (int)div32((uint32_t)e, s.magic32);
        const int32_t slot = sm[row];
        if (slot >= 0) st1<T>(out + base + e, mean1(to_f(pk[(int64_t)slot * m + (e - (int64_t)row * m)])));
    }
}

// chunk c of a ride: its decode, or (world size 1, fin) the fused pack + decode
template <typename T, int EF>
__device__ __forceinline__ void ride_chunk(const DecodeRide<T>& d, int c, float* __restrict__ dlds) {
    if constexpr (EF != ARCTOPK_EF21) {
        if (d.fin) {
            finalize_chunk<T>(d.segs, d.chunks[c], d.slotmap, d.E, d.out, d.fin, d.sc);
            return;
        }
    }
    decode_chunk<T, EF>(d.segs, d.chunks[c], d.dfirst + c, d.packed, d.slotmap, d.sc, d.gE, d.out, dlds);
}

// grid: [write ranges (nflat)] [small selects] [ride decode chunks (dr.n)] [V draw (job.n)]
template <typename T, int EF>
__global__ void __launch_bounds__(kFuseNT) k_arc_write_fused(const MBatch* __restrict__ bp, const RangeGrid g,
                                                             int nflat,
                                                             const uint32_t* __restrict__ keys, MWorkspace* ws,
                                                             const uint32_t* __restrict__ ckey,
                                                             const SegDev* __restrict__ segs,
                                                             const int32_t* __restrict__ small_ids,
                                                             const T* __restrict__ sketch, int R, Scale sc,
                                                             int32_t* __restrict__ rowlist,
                                                             int32_t* __restrict__ slotmap, DecodeRide<T> dr,
                                                             VDrawJob job) {
    if (maybe_draw_v<T>(job, kFuseNT)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
    const int rb = (int)blockIdx.x - ((int)gridDim.x - job.n - dr.n);
    if (rb >= 0) {  // the ride's decode chunks
        ride_chunk<T, EF>(dr, rb, reinterpret_cast<float*>(dyn));
        return;
    }
    if ((int)blockIdx.x >= nflat) {  // the small segments' single-block selects
        select_small_seg<T, kFuseNT>(segs, small_ids[blockIdx.x - nflat], sketch, R, sc, rowlist, slotmap, dyn);
        return;
    }
    int t, r;  // flat grid: the ranges of the batch's items back to back
    if (!ms_locate(g, &t, &r)) return;
    arc_write_fused_range(bp->it[t], t, r, keys, ws, ckey, rowlist, slotmap, dyn);
}

// The write pass of the refine path (ms_arc_write's body, one block per range) with a deferred
// decode riding in the same launch: grid [write ranges] [ride decode chunks (dr.n)].  The write
// blocks are few and latency-bound; the decode's chunks stream beside them instead of in a
// launch of their own after the select.
template <typename T, int EF>
__global__ void __launch_bounds__(256) k_arc_write_ride(const MBatch* __restrict__ bp, const RangeGrid g,
                                                        const uint32_t* __restrict__ keys, MWorkspace* ws,
                                                        int32_t* __restrict__ out_idx, int32_t* __restrict__ out_slot,
                                                        DecodeRide<T> dr) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
    const int nflat = g.first[g.cnt];
    if ((int)blockIdx.x >= nflat) {
        ride_chunk<T, EF>(dr, (int)blockIdx.x - nflat, reinterpret_cast<float*>(dyn));
        return;
    }
    int t, r;
    if (!ms_locate(g, &t, &r)) return;
    ms_write_body<0, true>(*bp, t, r, keys, nullptr, ws, out_idx, nullptr, out_slot, nullptr);
}

// The compact launch of a batch (arc_compact_range per range) with a trailing step's single-block
// selects after its range blocks: the latency-bound selects of a small bucket run beside the
// compact instead of in launches of their own (arctopk_exchange_trail)
template <typename T>
struct SelCarry {
    const SegDev* segs;
    const int32_t* ids;
    const T* sketch;
    int32_t* rowlist;
    int32_t* slotmap;
    int32_t n;  // segments (blocks)
};
template <typename T>
__global__ void __launch_bounds__(256) k_arc_compact_carry(const MBatch* __restrict__ bp, const RangeGrid g,
                                                           const uint32_t* __restrict__ keys, MWorkspace* ws,
                                                           uint32_t* __restrict__ ckey, SelCarry<T> sc, int R,
                                                           Scale scale) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
    const int nflat = g.first[g.cnt];
    if ((int)blockIdx.x >= nflat) {
        select_small_seg<T, kST>(sc.segs, sc.ids[blockIdx.x - nflat], sc.sketch, R, scale, sc.rowlist, sc.slotmap, dyn);
        return;
    }
    int t, r;
    if (!ms_locate(g, &t, &r)) return;
    arc_compact_range(bp->it[t], t, r, keys, ws, ckey);
}

struct KeysGrid {
    int32_t first[kMB + 1];  // first block of each item in the flat key-pass grid
};


// Larger segments: energy keys into global memory, fused with the first radix pass of
// the multi-block select (mselect.h): each block histograms its keys' top 12 bits in LDS
// and merges the non-empty bins into the segment's global histogram.  The bin holding the
// k-th largest key is then derived from that histogram by each block of the next launches
// (ms_arc_digit_local).
template <typename T, int KT>
__global__ void __launch_bounds__(KT) k_arc_keys(const SegDev* __restrict__ segs,
                                                  const int32_t* __restrict__ ids, int first,
                                                  const T* __restrict__ sketch, int R, Scale sc,
                                                  uint32_t* __restrict__ keys, MWorkspace* ws,
                                                  KeysGrid kg, int from_keys) {
    // one 16 KiB histogram (the compacted (bin, count) list is packed into it in place):
    // LDS sets the occupancy, and every block of the grid must be resident in one round
    __shared__ uint32_t h[kMBins];
    __shared__ uint32_t s_nnz;
    // flat grid: item t owns blocks [kg.first[t], kg.first[t + 1])
    int t = 0;
    while ((int)blockIdx.x >= kg.first[t + 1]) ++t;
    const int bx = (int)blockIdx.x - kg.first[t];
    const uint32_t nblk = (uint32_t)(kg.first[t + 1] - kg.first[t]);
    const SegDev s = segs[ids[first + t]];
    for (int i = threadIdx.x; i < kMBins; i += KT) h[i] = 0u;
    if (threadIdx.x == 0) s_nnz = 0u;
    __syncthreads();
    const int stride = (s.kind == ARCTOPK_SEG_RAW) ? 1 : R;
    const int64_t gs = (int64_t)nblk * KT;
    int64_t row = (int64_t)bx * KT + threadIdx.x;
    const T* sk = sketch + s.sketch_off;
    uint32_t* kout = keys + s.row_off;
    // The two edge bins are counted in registers: they can be hot (tied zero rows all land in
    // bin 0), and LDS atomics of a wave on ONE word serialise
    uint32_t c_lo = 0, c_hi = 0;
    auto count = [&](uint32_t key) {
        const uint32_t dg = arc_digit(key);
        if (dg == 0u) ++c_lo;
        else if (dg == (uint32_t)kMBins - 1u) ++c_hi;
        else atomicAdd(&h[dg], 1u);
    };
    if (from_keys && s.keyed) {  // the encode wrote the keys (keys mode): histogram only
        constexpr int UK = 8;
        for (; row < s.n; row += UK * gs) {
            uint32_t kv[UK];
#pragma unroll
            for (int u = 0; u < UK; ++u) kv[u] = kout[min(row + u * gs, s.n - 1)];
#pragma unroll
            for (int u = 0; u < UK; ++u)
                if (row + u * gs < s.n) count(kv[u]);
        }
    }
    if (stride == 4 && (s.sketch_off & 3) == 0) {  // r = 4: one quad load per row, UK rows in flight
        constexpr int UK = 8;
        for (; row < s.n; row += UK * gs) {
            float4 v[UK];
#pragma unroll
            for (int u = 0; u < UK; ++u) v[u] = ldq<T, false>(sk, min(row + u * gs, s.n - 1));
#pragma unroll
            for (int u = 0; u < UK; ++u) {
                const int64_t rr = row + u * gs;
                if (rr < s.n) {
                    const uint32_t key = energy_key(energy4<T>(v[u].x, v[u].y, v[u].z, v[u].w, sc));
                    kout[rr] = key;
                    count(key);
                }
            }
        }
    }
    for (; row < s.n; row += 8 * gs) {  // other r / 1-D tensors: 8 rows in flight as well
        float e[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) e[u] = row_energy(sk + min(row + u * gs, s.n - 1) * stride, R, sc, s.kind);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t rr = row + u * gs;
            if (rr < s.n) {
                const uint32_t key = energy_key(e[u]);
                kout[rr] = key;
                count(key);
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        c_lo += __shfl_xor(c_lo, o, 64);
        c_hi += __shfl_xor(c_hi, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (c_lo) atomicAdd(&h[0], c_lo);
        if (c_hi) atomicAdd(&h[kMBins - 1], c_hi);
    }
    __syncthreads();
    // Merge into the item's global histogram.  Memory-side atomics cost about one wave
    // instruction per 50 ns per CU whatever their lane count, so the non-empty bins are first
    // compacted into a dense LDS list (in place: bin << 20 | count, counts < 2^20 rows per
    // block) and merged by full wave instructions: a few per block instead of 64.
    constexpr int kCountBits = 32 - 12;
    if ((uint64_t)(s.n + nblk - 1) / nblk < (1ull << kCountBits)) {
        constexpr int PB = kMBins / KT;
        const int lane = threadIdx.x & 63;
        const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        uint32_t c[PB];
#pragma unroll
        for (int q = 0; q < PB; ++q) c[q] = h[q * KT + threadIdx.x];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PB; ++q) {
            const bool ne = c[q] != 0u;
            const uint64_t bm = __ballot(ne);
            uint32_t base = 0;
            if (lane == 0 && bm) base = atomicAdd(&s_nnz, (uint32_t)__popcll(bm));
            base = __shfl(base, 0, 64);
            if (ne) h[base + (uint32_t)__popcll(bm & lt)] = ((uint32_t)(q * KT + threadIdx.x) << kCountBits) | c[q];
        }
        __syncthreads();
        const uint32_t nnz = s_nnz;
        for (uint32_t i = threadIdx.x; i < nnz; i += KT) {
            const uint32_t e = h[i];
            atomicAdd(&ws->hist[t][hist_slot((int)(e >> kCountBits))], e & ((1u << kCountBits) - 1u));
        }
    } else {  // > 2^20 rows per block: every non-empty bin on its own
        for (int i = threadIdx.x; i < kMBins; i += KT)
            if (h[i]) atomicAdd(&ws->hist[t][hist_slot(i)], h[i]);
    }
    // (the compact and refine blocks derive the bin of the k-th key from the merged histogram)
}

__device__ __forceinline__ bool row_path(const SegDev& s) { return s.vec && s.m >= 256; }

// ---------------------------------------------------------------------------
// K3 pack
// ---------------------------------------------------------------------------
// EF21 on a quad: D = G - E (rounded to T, the bucket after add_(E, -1)), E_new = E + D
template <typename T>
__device__ __forceinline__ float4 ef21_d(float4 g, float4 e) {
    return rnd4<T>(make_float4(g.x - e.x, g.y - e.y, g.z - e.z, g.w - e.w));
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <typename T, int EF>
__device__ __forceinline__ float4 pack4(const T* __restrict__ G, T* __restrict__ E, int64_t src) {
    float4 v;
    if constexpr (EF == ARCTOPK_EF_NONE) {
        v = ldq<T, false>(G + src, 0);
    } else if constexpr (EF == ARCTOPK_EF14) {
        v = ldq<T, false>(E + src, 0);
        stq<T, false>(E + src, 0, make_float4(0.f, 0.f, 0.f, 0.f));
    } else {
        const float4 ev = ldq<T, false>(E + src, 0);
        v = ef21_d<T>(ldq<T, false>(G + src, 0), ev);
        stq<T, false>(E + src, 0, add4(ev, v));
    }
    return v;
}


// Pack of a row range of an m in {1, 2} fp32 segment (Chunk mode 1): lane per 16-B quad of
// the segment (4 / 2 rows), slot map read alongside; selected rows go to packed[slot * m],
// and (EF14 / EF21) the quad of E is rewritten whole when it holds a selected row.
template <int EF>
__device__ __forceinline__ void pack_stream_small(const SegDev& s, const Chunk& ch,
                                                  const float* __restrict__ G, float* __restrict__ E,
                                                  const int32_t* __restrict__ slotmap,
                                                  float* __restrict__ packed) {
    const int m = (int)s.m;
    const int64_t e0 = s.offset + ch.row0 * m;    // first element (16-B aligned)
    const int nq = (int)((ch.nrows * m + 3) >> 2);  // quads (the last may run past the segment)
    const int64_t seg_end = s.offset + s.n * m;
    const int32_t* sm = slotmap + s.row_off;
    float* pk = packed + s.packed_off;
    constexpr int UQ = 4;
    for (int q0 = threadIdx.x; q0 < nq; q0 += 256 * UQ) {
        float4 g[UQ], e[UQ];
        int32_t sl[UQ][4];
#pragma unroll
        for (int u = 0; u < UQ; ++u) {
            const int q = min(q0 + u * 256, nq - 1);
            const int64_t el = e0 + 4 * (int64_t)q;
            if (el + 4 <= seg_end) {
                if constexpr (EF != ARCTOPK_EF14) g[u] = *reinterpret_cast<const float4*>(G + el);
                if constexpr (EF != ARCTOPK_EF_NONE) e[u] = *reinterpret_cast<const float4*>(E + el);
            } else {  // segment tail: scalar, zero-filled
                float gv[4] = {0.f, 0.f, 0.f, 0.f}, ev[4] = {0.f, 0.f, 0.f, 0.f};
                for (int j = 0; j < 4 && el + j < seg_end; ++j) {
                    if constexpr (EF != ARCTOPK_EF14) gv[j] = G[el + j];
                    if constexpr (EF != ARCTOPK_EF_NONE) ev[j] = E[el + j];
                }
                g[u] = make_float4(gv[0], gv[1], gv[2], gv[3]);
                e[u] = make_float4(ev[0], ev[1], ev[2], ev[3]);
            }
            const int64_t r0 = (el - s.offset) / m;  // first row of the quad
#pragma unroll
            for (int j = 0; j < 4; ++j) sl[u][j] = (j < 4 / m && r0 + j < s.n) ? sm[r0 + j] : -1;
        }
#pragma unroll
        for (int u = 0; u < UQ; ++u) {
            const int q = q0 + u * 256;
            if (q >= nq) break;
            const int64_t el = e0 + 4 * (int64_t)q;
            const float gv[4] = {g[u].x, g[u].y, g[u].z, g[u].w};
            const float ev[4] = {e[u].x, e[u].y, e[u].z, e[u].w};
            float en[4] = {ev[0], ev[1], ev[2], ev[3]};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int rj = j / m;  // row of element j within the quad
                const int32_t slot = sl[u][rj];
                if (slot >= 0) {
                    float v;
                    if constexpr (EF == ARCTOPK_EF_NONE) {
                        v = gv[j];
                    } else if constexpr (EF == ARCTOPK_EF14) {
                        v = ev[j];
                        en[j] = 0.f;
                    } else {
                        v = gv[j] - ev[j];
                        en[j] = ev[j] + v;
                    }
                    pk[(int64_t)slot * m + (j - rj * m)] = v;
                }
            }
            if constexpr (EF != ARCTOPK_EF_NONE) {
                // every quad rewritten (unchanged values where no row is selected): whole
                // lines leave L2 instead of masked partial writes (read-modify-write at HBM)
                if (el + 4 <= seg_end) {
                    *reinterpret_cast<float4*>(E + el) = make_float4(en[0], en[1], en[2], en[3]);
                } else {
                    for (int j = 0; j < 4 && el + j < seg_end; ++j) E[el + j] = en[j];
                }
            }
        }
    }
}

// One pack chunk (256 threads): k_pack's block, or a block of the next bucket's encode launch
// that this bucket's pack rides in (world size 1, PackRide).  rs: LDS for kSmallTileRows rows.
template <typename T, int EF>
__device__ __forceinline__ void pack_chunk(const SegDev* __restrict__ segs, const Chunk ch,
                                           const T* __restrict__ G, T* __restrict__ E,
                                           const int32_t* __restrict__ rowlist,
                                           const int32_t* __restrict__ slotmap,
                                           T* __restrict__ packed, int32_t* __restrict__ dfirst,
                                           int32_t* __restrict__ rs) {
    const SegDev s = segs[ch.seg];
    const int m = (int)s.m;
    if constexpr (sizeof(T) == 4) {
        if (ch.mode == 1) {  // m in {1, 2}: stream every row's quad of E / G with the slot map
            pack_stream_small<EF>(s, ch, reinterpret_cast<const float*>(G), reinterpret_cast<float*>(E),
                                  slotmap, reinterpret_cast<float*>(packed));
            return;
        }
    }
    const int32_t* rl = rowlist + s.sel_off + ch.row0;
    T* dst = packed + s.packed_off + ch.row0 * m;
    if (row_path(s)) {  // wave per selected row: all of a row's loads first, then stores
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int m4 = m >> 2;
        constexpr int U = 8;
        for (int64_t j = wave; j < ch.nrows; j += 4) {
            const int64_t src_row = s.offset + (int64_t)rl[j] * m;
            const T* gp = G + src_row;
            T* ep = E + src_row;
            T* dp = dst + j * m;
            for (int c0 = 0; c0 < m4; c0 += 64 * U) {
                float4 a[U], b[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int c = min(c0 + u * 64 + lane, m4 - 1);
                    if constexpr (EF == ARCTOPK_EF_NONE) a[u] = ldq<T, kNtPack>(gp, c);
                    else if constexpr (EF == ARCTOPK_EF14) a[u] = ldq<T, kNtPack>(ep, c);
                    else { a[u] = ldq<T, kNtPack>(gp, c); b[u] = ldq<T, kNtPack>(ep, c); }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int c = c0 + u * 64 + lane;
                    if (c < m4) {
                        if constexpr (EF == ARCTOPK_EF_NONE) {
                            stq<T, false>(dp, c, a[u]);
                        } else if constexpr (EF == ARCTOPK_EF14) {
                            stq<T, false>(dp, c, a[u]);
                            stq<T, kNtPack>(ep, c, make_float4(0.f, 0.f, 0.f, 0.f));
                        } else {
                            const float4 dv = ef21_d<T>(a[u], b[u]);
                            stq<T, false>(dp, c, dv);
                            stq<T, kNtPack>(ep, c, add4(b[u], dv));
                        }
                    }
                }
            }
        }
        return;
    }
    if (m >= 4 && m < 256) {  // small-m: row list staged in LDS, 32-bit mulhi division
        const int nr = (int)ch.nrows;
        const int32_t before = (threadIdx.x == 0 && ch.row0 > 0) ? rl[-1] : -1;  // the previous slot's row
        for (int r = threadIdx.x; r < nr; r += 256) rs[r] = rl[r];
        __syncthreads();
        if (s.dchunk_rows > 0) {
            // the decode's chunk table (mode 3): chunk l of the segment starts at row l * CR, and
            // its first selected row is slot j for every boundary l * CR in (row(j - 1), row(j)];
            // boundaries past the last selected row get k (the segment's end, then the next
            // segment's first chunk: the same bucket-wide value the next segment would write)
            const int64_t CR = s.dchunk_rows;
            const int64_t nch = (s.n + CR - 1) / CR;
            for (int jl = threadIdx.x; jl < nr; jl += 256) {
                const int64_t j = ch.row0 + jl;
                const int64_t rj = rs[jl];
                const int64_t rp = jl > 0 ? rs[jl - 1] : before;
                for (int64_t l = (rp + CR) / CR; l <= rj / CR; ++l)
                    dfirst[s.dchunk0 + l] = (int32_t)(s.sel_off + j);
                if (j == s.k_rows - 1)
                    for (int64_t l = (rj + CR) / CR; l <= nch; ++l)
                        dfirst[s.dchunk0 + l] = (int32_t)(s.sel_off + s.k_rows);
            }
        }
        const uint32_t cnt = (uint32_t)(nr * m);
        const int64_t dbase = s.packed_off + ch.row0 * m;
        if constexpr (sizeof(T) == 4) {
            if ((m & 1) == 0 && (s.offset & 1) == 0) {
                // even m (3x3 / 5x5 conv rows, 72 / 200 B): 8-B units.  Every unit lies in one
                // row and both ends are 8-B aligned, so a wave's loads cover ~512 contiguous
                // bytes per row run instead of four stride-4 scalar passes over the same lines
                const uint32_t cnt2 = cnt >> 1;
                const float* Gf = reinterpret_cast<const float*>(G);
                float* Ef = reinterpret_cast<float*>(E);
                float* df = reinterpret_cast<float*>(dst);
                constexpr int Q = 8;
                for (uint32_t q0 = threadIdx.x; q0 < cnt2; q0 += 256 * Q) {
                    int64_t src[Q];
                    float2 va[Q], vb[Q];
#pragma unroll
                    for (int u = 0; u < Q; ++u) {
                        const uint32_t e = min(q0 + u * 256, cnt2 - 1) << 1;
                        const uint32_t r = div32(e, s.magic32);
                        src[u] = s.offset + (int64_t)rs[r] * m + (e - r * (uint32_t)m);
                    }
#pragma unroll
                    for (int u = 0; u < Q; ++u) {
                        if constexpr (EF == ARCTOPK_EF_NONE) va[u] = *reinterpret_cast<const float2*>(Gf + src[u]);
                        else if constexpr (EF == ARCTOPK_EF14) va[u] = *reinterpret_cast<const float2*>(Ef + src[u]);
                        else {
                            va[u] = *reinterpret_cast<const float2*>(Gf + src[u]);
                            vb[u] = *reinterpret_cast<const float2*>(Ef + src[u]);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < Q; ++u) {
                        const uint32_t q = q0 + u * 256;
                        if (q < cnt2) {
                            float2 v = va[u];
                            if constexpr (EF == ARCTOPK_EF14) {
                                *reinterpret_cast<float2*>(Ef + src[u]) = make_float2(0.f, 0.f);
                            } else if constexpr (EF == ARCTOPK_EF21) {
                                v = make_float2(va[u].x - vb[u].x, va[u].y - vb[u].y);
                                *reinterpret_cast<float2*>(Ef + src[u]) = make_float2(vb[u].x + v.x, vb[u].y + v.y);
                            }
                            *reinterpret_cast<float2*>(df + 2 * (int64_t)q) = v;
                        }
                    }
                }
                return;
            }
        }
        const int64_t pre = (4 - (dbase & 3)) & 3;
        auto one = [&](uint32_t e) -> float {
            const uint32_t r = div32(e, s.magic32);
            const int64_t src = s.offset + (int64_t)rs[r] * m + (e - r * (uint32_t)m);
            float v;
            if constexpr (EF == ARCTOPK_EF_NONE) {
                v = ld1<T>(G + src);
            } else if constexpr (EF == ARCTOPK_EF14) {
                v = ld1<T>(E + src);
                st1<T>(E + src, 0.f);
            } else {
                const float ev = ld1<T>(E + src);
                v = rnd<T>(ld1<T>(G + src) - ev);
                st1<T>(E + src, ev + v);
            }
            return v;
        };
        for (uint32_t e = threadIdx.x; e < (uint32_t)min<int64_t>(pre, cnt); e += 256) st1<T>(dst + e, one(e));
        const uint32_t body = cnt > pre ? (uint32_t)((cnt - pre) >> 2) : 0u;
        // body: Q float4 of the packed output per thread and round, every gather load of the
        // round issued before any residual store (the compiler may not move a load from E
        // above a store to E; the elements of a chunk are distinct, so nothing aliases)
        constexpr int Q = 4;
        for (uint32_t q0 = threadIdx.x; q0 < body; q0 += 256 * Q) {
            int64_t src[Q][4];
            float va[Q][4], vb[Q][4];
#pragma unroll
            for (int u = 0; u < Q; ++u) {
                const uint32_t e = (uint32_t)pre + (min(q0 + u * 256, body - 1) << 2);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t r = div32(e + j, s.magic32);
                    src[u][j] = s.offset + (int64_t)rs[r] * m + (e + j - r * (uint32_t)m);
                }
            }
#pragma unroll
            for (int u = 0; u < Q; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if constexpr (EF == ARCTOPK_EF_NONE) va[u][j] = ld1<T>(G + src[u][j]);
                    else if constexpr (EF == ARCTOPK_EF14) va[u][j] = ld1<T>(E + src[u][j]);
                    else { va[u][j] = ld1<T>(G + src[u][j]); vb[u][j] = ld1<T>(E + src[u][j]); }
                }
#pragma unroll
            for (int u = 0; u < Q; ++u) {
                const uint32_t q = q0 + u * 256;
                if (q < body) {
                    const uint32_t e = (uint32_t)pre + (q << 2);
                    float vp[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if constexpr (EF == ARCTOPK_EF_NONE) {
                            vp[j] = va[u][j];
                        } else if constexpr (EF == ARCTOPK_EF14) {
                            vp[j] = va[u][j];
                            st1<T>(E + src[u][j], 0.f);
                        } else {
                            vp[j] = rnd<T>(va[u][j] - vb[u][j]);
                            st1<T>(E + src[u][j], vb[u][j] + vp[j]);
                        }
                    }
                    stq<T, false>(dst + e, 0, make_float4(vp[0], vp[1], vp[2], vp[3]));
                }
            }
        }
        for (uint32_t e = (uint32_t)pre + (body << 2) + threadIdx.x; e < cnt; e += 256) st1<T>(dst + e, one(e));
        return;
    }
    if (m <= 3) {  // 1-D tensors (m = 1) and 1x1-conv rows (m = 2): thread per selected row,
                   // every gather load of a round issued before its stores
        constexpr int UR = 8;
        const int nr = (int)ch.nrows;
        for (int j0 = threadIdx.x; j0 < nr; j0 += 256 * UR) {
            int64_t src[UR];
            float va[UR][3], vb[UR][3];
#pragma unroll
            for (int u = 0; u < UR; ++u) {
                src[u] = s.offset + (int64_t)rl[min(j0 + u * 256, nr - 1)] * m;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (c < m) {
                        if constexpr (EF == ARCTOPK_EF_NONE) va[u][c] = ld1<T>(G + src[u] + c);
                        else if constexpr (EF == ARCTOPK_EF14) va[u][c] = ld1<T>(E + src[u] + c);
                        else { va[u][c] = ld1<T>(G + src[u] + c); vb[u][c] = ld1<T>(E + src[u] + c); }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < UR; ++u) {
                const int j = j0 + u * 256;
                if (j < nr) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        if (c < m) {
                            float v = va[u][c];
                            if constexpr (EF == ARCTOPK_EF14) {
                                st1<T>(E + src[u] + c, 0.f);
                            } else if constexpr (EF == ARCTOPK_EF21) {
                                v = rnd<T>(va[u][c] - vb[u][c]);
                                st1<T>(E + src[u] + c, vb[u][c] + v);
                            }
                            st1<T>(dst + (int64_t)j * m + c, v);
                        }
                    }
                }
            }
        }
        return;
    }
    const uint32_t cnt = (uint32_t)(ch.nrows * m);
    if (s.vec) {
        const uint32_t cnt4 = cnt >> 2;
        for (uint32_t q = threadIdx.x; q < cnt4; q += 256) {
            const uint32_t e = q << 2;
            const uint32_t srow = fdiv(e, s.mdiv);
            const uint32_t col = e - srow * (uint32_t)m;
            const int64_t src = s.offset + (int64_t)rl[srow] * m + col;
            stq<T, false>(dst + e, 0, pack4<T, EF>(G, E, src));
        }
    } else {
        for (uint32_t e = threadIdx.x; e < cnt; e += 256) {
            const uint32_t srow = fdiv(e, s.mdiv);
            const uint32_t col = e - srow * (uint32_t)m;
            const int64_t src = s.offset + (int64_t)rl[srow] * m + col;
            float v;
            if constexpr (EF == ARCTOPK_EF_NONE) {
                v = ld1<T>(G + src);
            } else if constexpr (EF == ARCTOPK_EF14) {
                v = ld1<T>(E + src);
                st1<T>(E + src, 0.f);
            } else {
                const float ev = ld1<T>(E + src);
                v = rnd<T>(ld1<T>(G + src) - ev);
                st1<T>(E + src, ev + v);
            }
            st1<T>(dst + e, v);
        }
    }
}

template <typename T, int EF>
__global__ void __launch_bounds__(256) k_pack(const SegDev* __restrict__ segs,
                                              const Chunk* __restrict__ chunks,
                                              const T* __restrict__ G, T* __restrict__ E,
                                              const int32_t* __restrict__ rowlist,
                                              const int32_t* __restrict__ slotmap,
                                              T* __restrict__ packed, int32_t* __restrict__ dfirst) {
    __shared__ int32_t rs[kSmallTileRows];
    pack_chunk<T, EF>(segs, chunks[blockIdx.x], G, E, rowlist, slotmap, packed, dfirst, rs);
}

// ---------------------------------------------------------------------------
// K4 decode
// ---------------------------------------------------------------------------
// One decode chunk (256 threads): k_decode's block, or a block of another launch that a
// deferred decode rides in (k_select_small_dec).  dlds: the small-m chunk tile (dynamic LDS).
template <typename T, int EF>
__device__ __forceinline__ void decode_chunk(const SegDev* __restrict__ segs, const Chunk ch,
                                             const int32_t* __restrict__ dfc,
                                             const T* __restrict__ packed,
                                             const int32_t* __restrict__ slotmap, Scale sc,
                                             T* __restrict__ gE, T* __restrict__ out,
                                             float* __restrict__ dlds) {
    // mean of the all-reduced values (ref values_memory.div_(ws)), rounded to T
    auto mean4 = [&](float4 v) { return rnd4<T>(sc(v)); };
    auto mean1 = [&](float v) { return rnd<T>(sc(v)); };
    const SegDev s = segs[ch.seg];
    const int m = (int)s.m;
    const int64_t base = s.offset + ch.row0 * m;
    const int32_t* sm = slotmap + s.row_off + ch.row0;
    const T* pk = packed + s.packed_off;
    if (ch.mode == 3) {
        // Short rows (4 <= m < 256), chunk of nr rows starting on a quad boundary of the bucket.
        // The pack wrote the bucket-wide index of the chunk's first selected row (dfc[0]) and
        // of the next chunk's (dfc[1]): the chunk's packed rows are one contiguous range, so
        // the slot map, that range and (EF21) gE are all loaded in ONE round trip, staged in
        // LDS (map: row -> slot within the range), and the chunk is written as 16-B quads.
        static_assert(ARCTOPK_SHORT3_CHUNK % 1024 == 0 && ARCTOPK_SHORT3_CHUNK <= 8192,
                      "register staging: chunks of 1024 .. 8192 elements");
        // rows (m >= 4: at most CHUNK / 4), packed values, output quads per thread
        constexpr int UR = ARCTOPK_SHORT3_CHUNK / 1024, UP = ARCTOPK_SHORT3_CHUNK / 256,
                      UG = ARCTOPK_SHORT3_CHUNK / 1024;
        const int nr = (int)ch.nrows, cnt = nr * m;
        const int32_t g0 = dfc[0], g1 = dfc[1];
        const int32_t f0 = g0 - (int32_t)s.sel_off;
        const int nsel = max(0, min(g1 - g0, nr));
        const int np = nsel * m;
        const T* pkc = pk + (int64_t)f0 * m;
        int32_t* lmap = reinterpret_cast<int32_t*>(dlds);
        float* lpk = dlds + ((nr + 3) & ~3);
        int32_t sv[UR];
        float pv[UP];
        [[maybe_unused]] float4 gq[UG];
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int r = (int)threadIdx.x + u * 256;
            sv[u] = r < nr ? sm[r] : -1;
        }
#pragma unroll
        for (int u = 0; u < UP; ++u) {
            const int p = (int)threadIdx.x + u * 256;
            pv[u] = p < np ? to_f(pkc[p]) : 0.f;
        }
        if constexpr (EF == ARCTOPK_EF21) {
#pragma unroll
            for (int u = 0; u < UG; ++u) {
                const int e = 4 * ((int)threadIdx.x + u * 256);
                if (e + 4 <= cnt) {
                    gq[u] = ldq<T, kNtDecode>(gE + base + e, 0);
                } else {
                    float g4[4] = {0.f, 0.f, 0.f, 0.f};
                    for (int j = 0; j < 4 && e + j < cnt; ++j) g4[j] = ld1<T>(gE + base + e + j);
                    gq[u] = make_float4(g4[0], g4[1], g4[2], g4[3]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int r = (int)threadIdx.x + u * 256;
            if (r < nr) lmap[r] = sv[u] >= 0 ? sv[u] - f0 : -1;
        }
#pragma unroll
        for (int u = 0; u < UP; ++u) {
            const int p = (int)threadIdx.x + u * 256;
            if (p < np) lpk[p] = pv[u];
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < UG; ++u) {
            const int e = 4 * ((int)threadIdx.x + u * 256);
            if (e >= cnt) break;
            float o[4];
            bool sel[4], any = false;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ej = min(e + j, cnt - 1);
                const uint32_t r = div32((uint32_t)ej, s.magic32);
                const int c = ej - (int)r * m;
                const int sl = lmap[r];
                sel[j] = sl >= 0 && sl < nsel && e + j < cnt;
                any = any || sel[j];
                float v = sel[j] ? mean1(lpk[sl * m + c]) : 0.f;
                if constexpr (EF == ARCTOPK_EF21) {
                    const float g = j == 0 ? gq[u].x : j == 1 ? gq[u].y : j == 2 ? gq[u].z : gq[u].w;
                    v = sel[j] ? rnd<T>(g + v) : g + 0.f;
                }
                o[j] = v;
            }
            if (e + 4 <= cnt) {
                stq<T, kNtDecode>(out + base + e, 0, make_float4(o[0], o[1], o[2], o[3]));
                if constexpr (EF == ARCTOPK_EF21)
                    if (any) stq<T, false>(gE + base + e, 0, make_float4(o[0], o[1], o[2], o[3]));
            } else {
                for (int j = 0; j < 4 && e + j < cnt; ++j) {
                    st1<T>(out + base + e + j, o[j]);
                    if constexpr (EF == ARCTOPK_EF21)
                        if (sel[j]) st1<T>(gE + base + e + j, o[j]);
                }
            }
        }
        return;
    }
    if constexpr (sizeof(T) == 4) {
        if (ch.mode == 1) {  // m in {1, 2}, 16-B aligned: lane per output quad
            const int nq = (int)((ch.nrows * m + 3) >> 2);
            const int64_t seg_end = s.offset + s.n * m;
            constexpr int UQ = 4;
            for (int q0 = threadIdx.x; q0 < nq; q0 += 256 * UQ) {
                int32_t sl[UQ][4];
                float pv[UQ][4], gv[UQ][4];
#pragma unroll
                for (int u = 0; u < UQ; ++u) {
                    const int q = min(q0 + u * 256, nq - 1);
                    const int rq = (4 * q) / m;  // first row of the quad within the chunk
#pragma unroll
                    for (int j = 0; j < 4; ++j) sl[u][j] = (j < 4 / m && ch.row0 + rq + j < s.n) ? sm[rq + j] : -1;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int32_t slot = sl[u][j / m];
                        pv[u][j] = slot >= 0 ? to_f(pk[(int64_t)slot * m + (j % m)]) : 0.f;
                    }
                    if constexpr (EF == ARCTOPK_EF21) {
                        const int64_t el = base + 4 * (int64_t)q;
#pragma unroll
                        for (int j = 0; j < 4; ++j) gv[u][j] = el + j < seg_end ? to_f(gE[el + j]) : 0.f;
                    }
                }
#pragma unroll
                for (int u = 0; u < UQ; ++u) {
                    const int q = q0 + u * 256;
                    if (q >= nq) break;
                    const int64_t el = base + 4 * (int64_t)q;
                    float o[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const bool sel = sl[u][j / m] >= 0;
                        float v = sel ? mean1(pv[u][j]) : 0.f;
                        if constexpr (EF == ARCTOPK_EF21) {
                            v = rnd<T>(gv[u][j] + v);
                            if (sel && el + j < seg_end) st1<T>(gE + el + j, v);
                        }
                        o[j] = v;
                    }
                    if (el + 4 <= seg_end) {
                        stq<T, kNtDecode>(out + el, 0, make_float4(o[0], o[1], o[2], o[3]));
                    } else {
                        for (int j = 0; j < 4 && el + j < seg_end; ++j) st1<T>(out + el + j, o[j]);
                    }
                }
            }
            return;
        }
        if (ch.mode == 2) {  // 4 <= m < 256 fp32: lane per 16-B output quad, no LDS, no barrier
            // The chunk's elements [e0, e1) of the segment; quads are 16-B aligned in memory,
            // so the chunk's first / last quad may hold elements of a neighbouring chunk:
            // those are masked out (and written element by element).  A quad spans at most two
            // rows (m >= 4): slot and column of its first element, the wrap decided per element.
            const int64_t e0 = ch.row0 * m, e1 = min<int64_t>(s.n, ch.row0 + ch.nrows) * m;
            const int64_t qa = (s.offset + e0) >> 2, qb = (s.offset + e1 + 3) >> 2;
            const int nq = (int)(qb - qa);
            const int32_t* smg = slotmap + s.row_off;
            const int64_t nrow_last = s.n - 1;
            constexpr int UQ = 4;
            for (int q0 = threadIdx.x; q0 < nq; q0 += 256 * UQ) {
                float pv[UQ][4], gv[UQ][4];
                int32_t sl0[UQ], sl1[UQ], col[UQ];
#pragma unroll
                for (int u = 0; u < UQ; ++u) {
                    const int q = min(q0 + u * 256, nq - 1);
                    const int64_t a = ((qa + q) << 2) - s.offset;  // segment element of quad slot 0
                    const int64_t af = max(a, e0);
                    const uint32_t r = fdiv((uint32_t)af, s.mdiv);
                    const int c = (int)(af - (int64_t)r * m) - (int)(af - a);  // column of slot 0 (may be < 0 at the head)
                    col[u] = c;
                    sl0[u] = smg[r];
                    sl1[u] = smg[min<int64_t>((int64_t)r + 1, nrow_last)];
                    if constexpr (EF == ARCTOPK_EF21) {
                        if (a >= e0 && a + 4 <= e1) {
                            const float4 g = ldq<T, kNtDecode>(gE + s.offset + a, 0);
                            gv[u][0] = g.x; gv[u][1] = g.y; gv[u][2] = g.z; gv[u][3] = g.w;
                        } else {
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                gv[u][j] = (a + j >= e0 && a + j < e1) ? to_f(gE[s.offset + a + j]) : 0.f;
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < UQ; ++u) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int cj = col[u] + j;
                        const bool wrap = cj >= m;
                        const int32_t slot = wrap ? sl1[u] : sl0[u];
                        const int cc = wrap ? cj - m : cj;
                        pv[u][j] = (slot >= 0 && cj >= 0) ? to_f(pk[(int64_t)slot * m + cc]) : 0.f;
                    }
                }
#pragma unroll
                for (int u = 0; u < UQ; ++u) {
                    const int q = q0 + u * 256;
                    if (q >= nq) break;
                    const int64_t a = ((qa + q) << 2) - s.offset;
                    float o[4];
                    bool selj[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int cj = col[u] + j;
                        selj[j] = (cj >= m ? sl1[u] : sl0[u]) >= 0;
                        float v = selj[j] ? mean1(pv[u][j]) : 0.f;
                        if constexpr (EF == ARCTOPK_EF21) v = selj[j] ? rnd<T>(gv[u][j] + v) : gv[u][j] + 0.f;
                        o[j] = v;
                    }
                    if (a >= e0 && a + 4 <= e1) {
                        stq<T, kNtDecode>(out + s.offset + a, 0, make_float4(o[0], o[1], o[2], o[3]));
                        if constexpr (EF == ARCTOPK_EF21) {
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                if (selj[j]) st1<T>(gE + s.offset + a + j, o[j]);
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (a + j >= e0 && a + j < e1) {
                                st1<T>(out + s.offset + a + j, o[j]);
                                if constexpr (EF == ARCTOPK_EF21)
                                    if (selj[j]) st1<T>(gE + s.offset + a + j, o[j]);
                            }
                        }
                    }
                }
            }
            return;
        }
    }
    if (row_path(s)) {  // wave per row: one slot lookup per row, float4 streams
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int m4 = m >> 2;
        for (int64_t j = wave; j < ch.nrows; j += 4) {
            const int32_t slot = sm[j];
            T* op = out + base + j * m;
            T* gp = gE + base + j * m;
            if (slot < 0) {
                if constexpr (EF == ARCTOPK_EF21) {
#pragma unroll 4
                    for (int c = lane; c < m4; c += 64) {
                        const float4 g = ldq<T, kNtDecode>(gp, c);
                        stq<T, kNtDecode>(op, c, make_float4(g.x + 0.f, g.y + 0.f, g.z + 0.f, g.w + 0.f));
                    }
                } else {
#pragma unroll 8
                    for (int c = lane; c < m4; c += 64)
                        stq<T, kNtDecode>(op, c, make_float4(0.f, 0.f, 0.f, 0.f));
                }
            } else {
                const T* pp = pk + (int64_t)slot * m;
#pragma unroll 4
                for (int c = lane; c < m4; c += 64) {
                    float4 v = mean4(ldq<T, false>(pp, c));
                    if constexpr (EF == ARCTOPK_EF21) {
                        v = rnd4<T>(add4(ldq<T, kNtDecode>(gp, c), v));
                        stq<T, kNtDecode>(gp, c, v);
                    }
                    stq<T, kNtDecode>(op, c, v);
                }
            }
        }
        return;
    }
    if (m >= 4 && m < 256) {
        // small m (3x3 / 1x1 convs): rows are too short for a wave each.  The chunk is
        // composed in LDS -- fill (zeros, or gE for EF21), then the selected rows, whose
        // packed values are one contiguous range (the row list is ascending) -- and then
        // written once with 16-B streaming stores: no partial-line double writes to HBM.
        // Tile index t = e + a, a = base mod 4, so 16-B output groups are 16-B LDS groups.
        __shared__ int32_t rows_s[kSmallTileRows];
        __shared__ int32_t s_first[4], s_cnt[4];
        const int nr = (int)ch.nrows;
        int32_t first = 0x7FFFFFFF;
        int32_t nsel = 0;
        for (int r = threadIdx.x; r < nr; r += 256) {
            const int32_t sl = sm[r];
            if (sl >= 0) {
                first = min(first, sl);
                ++nsel;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            first = min(first, __shfl_xor(first, o, 64));
            nsel += __shfl_xor(nsel, o, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            s_first[threadIdx.x >> 6] = first;
            s_cnt[threadIdx.x >> 6] = nsel;
        }
        __syncthreads();
        first = min(min(s_first[0], s_first[1]), min(s_first[2], s_first[3]));
        nsel = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        for (int r = threadIdx.x; r < nr; r += 256) {
            const int32_t sl = sm[r];
            if (sl >= 0) rows_s[sl - first] = r;
        }
        const int cnt = nr * m;
        const int a = (int)(base & 3);
        const int ngroups = (a + cnt + 3) >> 2;
        T* const ob = out - a + base;  // ob[t] = out[base + e]: quad-aligned at t % 4 == 0
        // 1. fill
        for (int gi = threadIdx.x; gi < ngroups; gi += 256) {
            const int t0 = gi << 2;
            if (t0 >= a && t0 + 4 <= a + cnt) {
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if constexpr (EF == ARCTOPK_EF21) {
                    const float4 g = ldq<T, kNtDecode>(gE - a + base + t0, 0);
                    v = make_float4(g.x + 0.f, g.y + 0.f, g.z + 0.f, g.w + 0.f);
                }
                *reinterpret_cast<float4*>(dlds + t0) = v;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = t0 + j;
                    if (t >= a && t < a + cnt)
                        dlds[t] = EF == ARCTOPK_EF21 ? ld1<T>(gE + base + t - a) + 0.f : 0.f;
                }
            }
        }
        __syncthreads();
        // 2. the selected rows
        const T* src = pk + (int64_t)first * m;
        const uint32_t np = (uint32_t)(nsel * m);
        for (uint32_t p = threadIdx.x; p < np; p += 256) {
            const uint32_t j = div32(p, s.magic32);
            const int le = rows_s[j] * m + (int)(p - j * (uint32_t)m);
            float v = mean1(to_f(src[p]));
            if constexpr (EF == ARCTOPK_EF21) {
                v = rnd<T>(ld1<T>(gE + base + le) + v);
                st1<T>(gE + base + le, v);
            }
            dlds[le + a] = v;
        }
        __syncthreads();
        // 3. one streaming write of the chunk
        for (int gi = threadIdx.x; gi < ngroups; gi += 256) {
            const int t0 = gi << 2;
            if (t0 >= a && t0 + 4 <= a + cnt) {
                stq<T, kNtDecode>(ob + t0, 0, *reinterpret_cast<const float4*>(dlds + t0));
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = t0 + j;
                    if (t >= a && t < a + cnt) st1<T>(ob + t, dlds[t]);
                }
            }
        }
        return;
    }
    if (m <= 3) {  // 1-D tensors and 1x1-conv rows: thread per row, slot lookups batched
        constexpr int UR = 4;
        const int nr = (int)ch.nrows;
        for (int r0 = threadIdx.x; r0 < nr; r0 += 256 * UR) {
            int32_t sl[UR];
            float pv[UR][3];
#pragma unroll
            for (int u = 0; u < UR; ++u) sl[u] = sm[min(r0 + u * 256, nr - 1)];
#pragma unroll
            for (int u = 0; u < UR; ++u)
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    pv[u][c] = (c < m && sl[u] >= 0) ? to_f(pk[(int64_t)sl[u] * m + c]) : 0.f;
#pragma unroll
            for (int u = 0; u < UR; ++u) {
                const int r = r0 + u * 256;
                if (r < nr) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        if (c < m) {
                            const int64_t e = base + (int64_t)r * m + c;
                            float v = sl[u] >= 0 ? mean1(pv[u][c]) : 0.f;
                            if constexpr (EF == ARCTOPK_EF21) {
                                v = rnd<T>(ld1<T>(gE + e) + v);
                                if (sl[u] >= 0) st1<T>(gE + e, v);
                            }
                            st1<T>(out + e, v);
                        }
                    }
                }
            }
        }
        return;
    }
    const uint32_t cnt = (uint32_t)(ch.nrows * m);
    if (s.vec) {
        const uint32_t cnt4 = cnt >> 2;
        for (uint32_t q = threadIdx.x; q < cnt4; q += 256) {
            const uint32_t e = q << 2;
            const uint32_t row = fdiv(e, s.mdiv);
            const uint32_t col = e - row * (uint32_t)m;
            const int32_t slot = sm[row];
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (slot >= 0) v = mean4(ldq<T, false>(pk + (int64_t)slot * m + col, 0));
            if constexpr (EF == ARCTOPK_EF21) {
                v = rnd4<T>(add4(ldq<T, false>(gE + base + e, 0), v));
                if (slot >= 0) stq<T, false>(gE + base + e, 0, v);
            }
            stq<T, false>(out + base + e, 0, v);
        }
    } else {
        for (uint32_t e = threadIdx.x; e < cnt; e += 256) {
            const uint32_t row = fdiv(e, s.mdiv);
            const uint32_t col = e - row * (uint32_t)m;
            const int32_t slot = sm[row];
            float v = 0.f;
            if (slot >= 0) v = mean1(to_f(pk[(int64_t)slot * m + col]));
            if constexpr (EF == ARCTOPK_EF21) {
                v = rnd<T>(ld1<T>(gE + base + e) + v);
                if (slot >= 0) st1<T>(gE + base + e, v);
            }
            st1<T>(out + base + e, v);
        }
    }
}

template <typename T, int EF>
__global__ void __launch_bounds__(256) k_decode(DecodeRide<T> d) {
    extern __shared__ __attribute__((aligned(16))) float dlds[];  // small-m chunk tile
    ride_chunk<T, EF>(d, (int)blockIdx.x, dlds);
}

// the decode into a bucket that is already zero (fin 3, the zero-ahead drain: only ever the
// backward's last step's own decode, never a ride -- a kernel of its own, so the kernels the
// rides run in keep their code)
template <typename T>
__global__ void __launch_bounds__(256) k_decode_scatter(DecodeRide<T> d) {
    scatter_chunk<T>(d.segs, d.chunks[blockIdx.x], d.packed, d.slotmap, d.out, d.sc);
}

// Two buckets' decodes in one launch (the backward's last exchange step: the previous bucket's
// deferred decode and its own), blocks [0, a.n) of `a`, then `b`'s
template <typename T, int EF>
__global__ void __launch_bounds__(256) k_decode2(DecodeRide<T> a, DecodeRide<T> b) {
    extern __shared__ __attribute__((aligned(16))) float dlds[];
    const int i = (int)blockIdx.x;
    const DecodeRide<T>& d = i < a.n ? a : b;
    const int c = i < a.n ? i : i - a.n;
    ride_chunk<T, EF>(d, c, dlds);
}

// A deferred decode (an earlier bucket's, arctopk_exchange_step's `ride`) riding in the
// single-block select launch of the current bucket: the select blocks are latency-bound
// (a few KiB each), the decode chunks stream the bucket, so the select is hidden behind the
// decode's HBM time instead of idling the GPU between encode and pack.
template <typename T, int EF>
__global__ void __launch_bounds__(kST) k_select_small_dec(const SegDev* __restrict__ segs,
                                                          const int32_t* __restrict__ seg_ids, int nsel,
                                                          const T* __restrict__ sketch, int R, Scale sc,
                                                          int32_t* __restrict__ rowlist,
                                                          int32_t* __restrict__ slotmap, DecodeRide<T> dr,
                                                          VDrawJob job) {
    if (maybe_draw_v<T>(job, kST)) return;  // trailing blocks: the next call's projections
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
    if ((int)blockIdx.x < nsel) {  // first: the latency-bound selects
        select_small_seg<T, kST>(segs, seg_ids[blockIdx.x], sketch, R, sc, rowlist, slotmap, dyn);
        return;
    }
    ride_chunk<T, EF>(dr, (int)blockIdx.x - nsel, reinterpret_cast<float*>(dyn));
}

// WRITE_X = false (EF14 fold): E := x + E only; the caller reads the pre-compression
// bucket from E afterwards (TopK / RandK), so x is not written twice
template <int EF, bool ERR_IN, bool WRITE_X = true>
__global__ void __launch_bounds__(256) k_ef_apply(float* __restrict__ x, float* __restrict__ E,
                                                  int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t n4 = n >> 2;
    float4* x4 = reinterpret_cast<float4*>(x);
    float4* e4 = reinterpret_cast<float4*>(E);
    constexpr bool kReadE = EF == ARCTOPK_EF21 || (EF == ARCTOPK_EF14 && ERR_IN);
    // U quads per lane in flight, nontemporal streams (the bucket is touched once here)
    constexpr int U = 4;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        float4 g[U], e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            g[u] = ld_stream(x4 + i + u * stride);
            if constexpr (kReadE) e[u] = ld_stream(e4 + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float4 v = g[u];
            if constexpr (EF == ARCTOPK_EF14 && ERR_IN) {
                v.x += e[u].x; v.y += e[u].y; v.z += e[u].z; v.w += e[u].w;
            } else if constexpr (EF == ARCTOPK_EF21) {
                v.x -= e[u].x; v.y -= e[u].y; v.z -= e[u].z; v.w -= e[u].w;
            }
            if constexpr (EF == ARCTOPK_EF14) st_stream(e4 + i + u * stride, v);
            if constexpr ((EF != ARCTOPK_EF14 || ERR_IN) && WRITE_X) st_stream(x4 + i + u * stride, v);
        }
    }
    for (; i < n4; i += stride) {
        const float4 v = ef_apply4<EF, ERR_IN>(x4, e4, i);
        if constexpr (EF == ARCTOPK_EF14) e4[i] = v;
        if constexpr ((EF != ARCTOPK_EF14 || ERR_IN) && WRITE_X) x4[i] = v;
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const float v = ef_apply1<float, EF, ERR_IN>(x, E, i);
        if constexpr (EF == ARCTOPK_EF14) E[i] = v;
        if constexpr ((EF != ARCTOPK_EF14 || ERR_IN) && WRITE_X) x[i] = v;
    }
}

// bf16 buckets (TopK / RandK): element-wise, x = rnd(x +- E) as the reference's bf16 add_
template <int EF, bool ERR_IN, bool WRITE_X = true>
__global__ void __launch_bounds__(256) k_ef_apply_bf16(bf16_t* __restrict__ x, bf16_t* __restrict__ E,
                                                       int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float v = ef_apply1<bf16_t, EF, ERR_IN>(x, E, i);
        if constexpr (EF == ARCTOPK_EF14) st1<bf16_t>(E + i, v);
        if constexpr ((EF != ARCTOPK_EF14 || ERR_IN) && WRITE_X) st1<bf16_t>(x + i, v);
    }
}

// sketch of column-split tensors: the parts' fp32 partial sketches summed in part order,
// then rounded to T once (the reference's mm accumulates in fp32 and rounds its output)
template <typename T>
__global__ void __launch_bounds__(256) k_sketch_combine(const SegDev* __restrict__ segs,
                                                        const int32_t* __restrict__ ids, int R,
                                                        const float* __restrict__ part_buf,
                                                        T* __restrict__ sketch) {
    const SegDev s = segs[ids[blockIdx.y]];
    const int64_t cnt = s.n * R;
    const float* pb = part_buf + s.part_off;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256) {
        float v = pb[i];
        for (int q = 1; q < s.nparts; ++q) v = __fadd_rn(v, pb[(int64_t)q * cnt + i]);
        st1<T>(sketch + s.sketch_off + i, v);
    }
}

// a launch that completes `done` itself when given one (hipExtLaunchKernelGGL's stop event)
template <typename... KArgs, typename... Args>
inline void launch_done(void (*k)(KArgs...), dim3 grid, dim3 block, size_t lds, hipStream_t st, hipEvent_t done,
                        Args... args) {
    if (done) hipExtLaunchKernelGGL(k, grid, block, lds, st, nullptr, done, 0, args...);
    else hipLaunchKernelGGL(k, grid, block, lds, st, args...);
}

// one launch (every tile's V slice fits in LDS), then the partial-sketch sums of
// column-split tensors; done: completed by the last of them
template <typename T, int R>
int launch_encode_r(const arctopk_plan* p, const T* G, T* E, int ef, int err_in, const T* V, T* sk,
                    uint32_t* keys, hipStream_t st, PackRide<T> pr, hipEvent_t done = nullptr,
                    EncRide<T> er = EncRide<T>{}, int er_lds = 0, bool er_short = true) {
    hipEvent_t enc_done = p->n_split == 0 ? done : nullptr;
    if (p->n_enc > 0 || pr.n > 0 || er.n > 0) {
        const bool use_e = p->n_enc_e > 0 && (ef == ARCTOPK_EF21 || (ef == ARCTOPK_EF14 && err_in));
        const int nt = use_e ? p->n_enc_e : p->n_enc;
        dim3 grid(nt + pr.n + er.n), block(256);
        // (a riding pack chunk stages up to kSmallTileRows rows of its row list in the same LDS)
        const size_t lds = std::max<size_t>(std::max<size_t>((size_t)p->enc_lds_bytes, (size_t)er_lds),
                                            pr.n ? (size_t)kSmallTileRows * 4 : 0);
        const EncTile* tiles = use_e ? p->d_enc_e : p->d_enc;
        float* pb = p->d_part;
        if (er.n > 0) {  // a trailing step's tiles too: the lean kernel only if both tables are short
            if constexpr (R != 4) return ARCTOPK_EINVAL;  // (instantiated for the default r only)
            else if (p->enc_short && er_short) {
                if (ef == ARCTOPK_EF_NONE)
                    launch_done(&k_encode_carry<T, R, ARCTOPK_EF_NONE, false, false>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr, er);
                else if (ef == ARCTOPK_EF14 && err_in)
                    launch_done(&k_encode_carry<T, R, ARCTOPK_EF14, true, false>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr, er);
                else if (ef == ARCTOPK_EF14)
                    launch_done(&k_encode_carry<T, R, ARCTOPK_EF14, false, false>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr, er);
                else
                    return ARCTOPK_EINVAL;
            } else {
                if (ef == ARCTOPK_EF_NONE)
                    launch_done(&k_encode_carry<T, R, ARCTOPK_EF_NONE, false, true>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr, er);
                else if (ef == ARCTOPK_EF14 && err_in)
                    launch_done(&k_encode_carry<T, R, ARCTOPK_EF14, true, true>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr, er);
                else if (ef == ARCTOPK_EF14)
                    launch_done(&k_encode_carry<T, R, ARCTOPK_EF14, false, true>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr, er);
                else
                    return ARCTOPK_EINVAL;
            }
        } else if (p->enc_short) {  // no wave-per-row tile: the lean kernel
            if (ef == ARCTOPK_EF_NONE)
                launch_done(&k_encode_short<T, R, ARCTOPK_EF_NONE, false>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr);
            else if (ef == ARCTOPK_EF14 && err_in)
                launch_done(&k_encode_short<T, R, ARCTOPK_EF14, true>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr);
            else if (ef == ARCTOPK_EF14)
                launch_done(&k_encode_short<T, R, ARCTOPK_EF14, false>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr);
            else
                launch_done(&k_encode_short<T, R, ARCTOPK_EF21, true>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr);
        } else if (ef == ARCTOPK_EF_NONE)
            launch_done(&k_encode<T, R, ARCTOPK_EF_NONE, false>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr);
        else if (ef == ARCTOPK_EF14 && err_in)
            launch_done(&k_encode<T, R, ARCTOPK_EF14, true>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr);
        else if (ef == ARCTOPK_EF14)
            launch_done(&k_encode<T, R, ARCTOPK_EF14, false>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr);
        else
            launch_done(&k_encode<T, R, ARCTOPK_EF21, true>, grid, block, lds, st, enc_done, p->d_segs, tiles, nt, G, E, V, sk, pb, keys, pr);
        const int e = (int)hipGetLastError();
        if (e) return e;
    }
    if (p->n_split == 0) {
        // (no encode launch at all: nothing for `done` to follow but the stream itself)
        if (done && !(p->n_enc > 0 || pr.n > 0)) return (int)hipEventRecord(done, st);
        return 0;
    }
    const int gx = (int)std::min<int64_t>(256, (p->split_rows_max * R + 255) / 256);
    launch_done(&k_sketch_combine<T>, dim3(gx, p->n_split), dim3(256), 0, st, done, (const SegDev*)p->d_segs,
                (const int32_t*)p->d_split, R, (const float*)p->d_part, sk);
    return (int)hipGetLastError();
}

template <typename T>
int launch_encode(const arctopk_plan* p, const void* grad, void* err, int ef, int err_in, const void* V,
                  void* sketch, uint32_t* keys, hipStream_t st, PackRide<T> pr = PackRide<T>{},
                  hipEvent_t done = nullptr, EncRide<T> er = EncRide<T>{}, int er_lds = 0, bool er_short = true) {
    const T* G = static_cast<const T*>(grad);
    T* E = static_cast<T*>(err);
    const T* Vt = static_cast<const T*>(V);
    T* sk = static_cast<T*>(sketch);
    switch (p->r) {
        case 1: return launch_encode_r<T, 1>(p, G, E, ef, err_in, Vt, sk, keys, st, pr, done, er, er_lds, er_short);
        case 2: return launch_encode_r<T, 2>(p, G, E, ef, err_in, Vt, sk, keys, st, pr, done, er, er_lds, er_short);
        case 3: return launch_encode_r<T, 3>(p, G, E, ef, err_in, Vt, sk, keys, st, pr, done, er, er_lds, er_short);
        case 4: return launch_encode_r<T, 4>(p, G, E, ef, err_in, Vt, sk, keys, st, pr, done, er, er_lds, er_short);
        case 5: return launch_encode_r<T, 5>(p, G, E, ef, err_in, Vt, sk, keys, st, pr, done, er, er_lds, er_short);
        case 6: return launch_encode_r<T, 6>(p, G, E, ef, err_in, Vt, sk, keys, st, pr, done, er, er_lds, er_short);
        case 7: return launch_encode_r<T, 7>(p, G, E, ef, err_in, Vt, sk, keys, st, pr, done, er, er_lds, er_short);
        case 8: return launch_encode_r<T, 8>(p, G, E, ef, err_in, Vt, sk, keys, st, pr, done, er, er_lds, er_short);
    }
    return ARCTOPK_EINVAL;
}

// the trailing step carried by plan p's exchange step (p->x_carry), as its encode ride
template <typename T>
EncRide<T> make_enc_ride(const arctopk_plan* p, int ef, int err_in, int* lds) {
    EncRide<T> er{};
    *lds = 0;
    const arctopk_plan* c = p->x_carry;
    if (!c) return er;
    const bool use_e = c->n_enc_e > 0 && (ef == ARCTOPK_EF21 || (ef == ARCTOPK_EF14 && err_in));
    er.segs = c->d_segs;
    er.tiles = use_e ? c->d_enc_e : c->d_enc;
    er.n = use_e ? c->n_enc_e : c->n_enc;
    er.G = static_cast<const T*>(c->x_t_bucket);
    er.E = static_cast<T*>(c->x_t_err);
    er.V = static_cast<const T*>(c->x_t_V ? c->x_t_V : c->b_V);
    er.sketch = static_cast<T*>(c->b_sketch);
    er.part = c->d_part;
    er.keys = c->any_keyed ? c->d_keys : nullptr;
    *lds = c->enc_lds_bytes;
    return er;
}

Scale make_scale(int32_t ws) {
    Scale sc;
    sc.ws = (float)ws;
    sc.pow2 = (ws & (ws - 1)) == 0;
    sc.inv = 1.0f / (float)ws;
    return sc;
}

template <typename T>
int launch_energy(const arctopk_plan* p, const void* sketch, int32_t ws, uint32_t* keys, float* energy,
                  hipStream_t st) {
    int64_t maxn = 0;
    for (int i = 0; i < p->nseg; ++i) maxn = std::max<int64_t>(maxn, p->h_segs[i].n);
    int gx = (int)std::min<int64_t>(1024, (maxn + 255) / 256);
    dim3 grid(gx, p->nseg);
    hipLaunchKernelGGL(k_energy<T>, grid, dim3(256), 0, st, p->d_segs, p->nseg, static_cast<const T*>(sketch),
                       p->r, make_scale(ws), keys, energy);
    return (int)hipGetLastError();
}

// a deferred decode offered to ride in the select's last launch (see DecodeRide)
struct RideArgs {
    const arctopk_plan* rp;
    int32_t ws, ef;
    void* gerr;
    void* out;
};
// the fused pack + decode of plan rp's deferred step (exchange.cpp sets x_fin at world size 1)
inline int ride_fin(const arctopk_plan* rp, int32_t ef) {
    if (rp->x_fin == 3) return ef == ARCTOPK_EF21 ? 0 : 3;
    return rp->x_fin ? (ef == ARCTOPK_EF14 ? 1 : 2) : 0;
}

template <typename T>
DecodeRide<T> make_ride(const RideArgs* ra) {
    DecodeRide<T> dr{};
    if (!ra) return dr;
    const arctopk_plan* rp = ra->rp;
    dr.segs = rp->d_segs;
    dr.chunks = rp->d_dec;
    dr.dfirst = rp->d_dfirst;
    dr.packed = static_cast<const T*>(rp->b_packed);
    dr.slotmap = rp->b_slotmap;
    dr.gE = static_cast<T*>(ra->gerr);
    dr.out = static_cast<T*>(ra->out);
    dr.sc = make_scale(ra->ws);
    dr.n = rp->n_dec;
    dr.fin = ride_fin(rp, ra->ef);
    if (dr.fin == 3) dr.fin = 0;  // (a ride never follows a zero-ahead; a whole decode is right anyway)
    dr.E = static_cast<T*>(rp->x_err);
    return dr;
}

template <typename T, int EF>
int launch_write_fused(const arctopk_plan* p, int bi, int nflat, int nsm, const uint32_t* ckey, const T* sketch,
                       int32_t ws, int32_t* rowlist, int32_t* slotmap, DecodeRide<T> dr, VDrawJob bj, size_t shm,
                       hipStream_t st) {
    if (shm > 48 * 1024) {
        static const hipError_t ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_arc_write_fused<T, EF>),
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        if (ok != hipSuccess) return (int)ok;
    }
    launch_job_kernel(&k_arc_write_fused<T, EF>, dim3(nflat + nsm + dr.n + bj.n), dim3(kFuseNT), shm, st,
                      (const MBatch*)(p->d_large_batches + bi), ms_range_grid(p->h_large_batches[bi]), nflat,
                      (const uint32_t*)p->d_keys, p->d_mws, ckey,
                      (const SegDev*)p->d_segs, (const int32_t*)p->d_small, sketch, (int)p->r, make_scale(ws),
                      rowlist, slotmap, dr, bj);
    return (int)hipGetLastError();
}

template <typename T, int EF>
int launch_write_ride(const arctopk_plan* p, int bi, int32_t* rowlist, int32_t* slotmap, DecodeRide<T> dr,
                      size_t shm, hipStream_t st) {
    if (shm > 48 * 1024) {
        static const hipError_t ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_arc_write_ride<T, EF>),
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        if (ok != hipSuccess) return (int)ok;
    }
    const RangeGrid g = ms_range_grid(p->h_large_batches[bi]);
    hipLaunchKernelGGL((k_arc_write_ride<T, EF>), dim3(g.first[g.cnt] + dr.n), dim3(256), shm, st,
                       (const MBatch*)(p->d_large_batches + bi), g, (const uint32_t*)p->d_keys, p->d_mws, rowlist,
                       slotmap, dr);
    return (int)hipGetLastError();
}

// ride: a deferred decode that may run in the last select launch (*rode = true if it did)
template <typename T>
int launch_select(const arctopk_plan* p, const void* sketch_, int32_t ws, int32_t* rowlist, int32_t* slotmap,
                  VDrawJob job, bool* drawn, hipStream_t st, const RideArgs* ride = nullptr, bool* rode = nullptr,
                  bool keyed = false) {
    *drawn = false;
    if (rode) *rode = false;
    const T* sketch = static_cast<const T*>(sketch_);
    // with large segments, the small segments' selects run inside the first batch's refine
    if (p->n_small && p->n_large_batches == 0) {
        // one block per segment: 1024 threads once a segment has more than 4096 rows (the
        // radix rounds and the compaction are per-block latency chains)
        constexpr int64_t big_rows = ARCTOPK_SEL_BIG_ROWS;  // rows for 1024 threads (build-time A/B)
        const dim3 grid(p->n_small + job.n);
        static_assert(((kSmallSelRows + 3) & ~3) * 4 + 16 <= kRefineLdsCap * 4, "small-select keys fit the LDS cap");
        if (p->small_lds > 48 * 1024) {  // > 48 KiB of keys: the dynamic LDS attribute
            static const hipError_t lds_ok = hipFuncSetAttribute(
                reinterpret_cast<const void*>(&k_select_small<T, 1024>),
                hipFuncAttributeMaxDynamicSharedMemorySize, kRefineLdsCap * 4);
            if (lds_ok != hipSuccess) return (int)lds_ok;
        }
        if (p->small_lds > big_rows * 4 + 16 || p->small_lds > 48 * 1024)
            launch_job_kernel(&k_select_small<T, 1024>, grid, dim3(1024), (size_t)p->small_lds, st,
                              (const SegDev*)p->d_segs, (const int32_t*)p->d_small, sketch, (int)p->r,
                              make_scale(ws), rowlist, slotmap, job);
        else
            launch_job_kernel(&k_select_small<T, kST>, grid, dim3(kST), (size_t)p->small_lds, st,
                              (const SegDev*)p->d_segs, (const int32_t*)p->d_small, sketch, (int)p->r,
                              make_scale(ws), rowlist, slotmap, job);
        *drawn = true;
    }
    for (int bi = 0; bi < p->n_large_batches; ++bi) {
        const MBatch& b = p->h_large_batches[bi];
        int64_t maxn = 0;
        for (int i = 0; i < b.cnt; ++i) maxn = std::max<int64_t>(maxn, b.it[i].n);
        // Rows per block and blocks per item: about one block per CU for the whole batch, every
        // block resident at once, equal rows per block (the pass is bandwidth-bound: an item
        // with fewer rows per block would finish early and leave its bandwidth share idle), and
        // few blocks, since each block merges its histogram with memory-side atomics on the
        // same hot words (measured on ResNet-50's bucket: 1120 x 256-thread blocks spent ~10 us
        // in that merge tail)
        // (build-time A/B switches: key-pass block size; grid target -- 1024-thread blocks:
        // ~one per CU fits, 263 did not: 2 rounds; rows per block at least)
        constexpr int keys_threads = ARCTOPK_KEYS_THREADS == 256 ? 256 : 1024;
        constexpr int64_t target_blocks = ARCTOPK_KEYS_BLOCKS;
        constexpr int64_t min_rpb = ARCTOPK_KEYS_MIN_ROWS;
        int64_t rows = 0;
        for (int i = 0; i < b.cnt; ++i) rows += b.it[i].n;
        const int64_t rpb = std::max<int64_t>(min_rpb, (rows + target_blocks - 1) / target_blocks);
        KeysGrid kg;
        kg.first[0] = 0;
        for (int i = 0; i < b.cnt; ++i)
            kg.first[i + 1] = kg.first[i] + (int32_t)std::max<int64_t>(
                1, std::min<int64_t>(kMHistBlocks, (b.it[i].n + rpb - 1) / rpb));
        if (keys_threads == 256)
            hipLaunchKernelGGL((k_arc_keys<T, 256>), dim3(kg.first[b.cnt]), dim3(256), 0, st, p->d_segs,
                               p->d_large, bi * kMB, sketch, p->r, make_scale(ws), p->d_keys, p->d_mws, kg,
                               keyed ? 1 : 0);
        else
            hipLaunchKernelGGL((k_arc_keys<T, 1024>), dim3(kg.first[b.cnt]), dim3(1024), 0, st, p->d_segs,
                               p->d_large, bi * kMB, sketch, p->r, make_scale(ws), p->d_keys, p->d_mws, kg,
                               keyed ? 1 : 0);
        int e = 0;
        if (bi == 0 && p->x_carry) {  // the trailing step's selects ride in the compact launch
            const arctopk_plan* c = p->x_carry;
            const SelCarry<T> sc{c->d_segs, c->d_small, static_cast<const T*>(c->b_sketch), c->b_rowlist,
                                 c->b_slotmap, c->n_small};
            const RangeGrid g = ms_range_grid(b);
            hipLaunchKernelGGL(k_arc_compact_carry<T>, dim3(g.first[g.cnt] + sc.n), dim3(256), (size_t)c->small_lds,
                               st, (const MBatch*)(p->d_large_batches + bi), g, (const uint32_t*)p->d_keys, p->d_mws,
                               reinterpret_cast<uint32_t*>(p->d_mws + 1), sc, (int)p->r, make_scale(1));
            e = (int)hipGetLastError();
        } else {
            e = ms_arc_compact(b, p->d_large_batches + bi, p->d_keys, p->d_mws, p->mws_cap, st);
        }
        if (e) return e;
        const int nsm = bi == 0 ? p->n_small : 0;
        VDrawJob bj = job;
        if (bi != 0) bj.n = 0;
        uint32_t* ckey = reinterpret_cast<uint32_t*>(p->d_mws + 1);
        // items of at most kFuseMaxRows rows: the refine runs inside the write blocks (one
        // launch fewer)
        // ... and only while every write block is resident at once: each one carries a refine,
        // so a second round of blocks costs more than the refine launch it saves (28 x [512,
        // 512, 3, 3] as 896 one-range blocks: select 63 -> 74 us; spans of several ranges per
        // block measured slower still, rounds 3 and 4), so larger batches take the refine launch
        int nflat = 0;
        for (int i = 0; i < b.cnt; ++i) nflat += b.it[i].nranges;
        // The small selects sharing the launch run as 256-thread blocks: only when none has
        // more than 4,096 rows (1,024-thread blocks select 8 K-row segments faster than these
        // write blocks finish: ResNet-18's third DDP bucket measured 250 -> 241 GB/s fused)
        if (maxn <= kFuseMaxRows && nflat + nsm + bj.n <= kFuseMaxBlocks &&
            (nsm == 0 || p->small_lds <= 4096 * 4 + 16)) {
            size_t shm = std::max<size_t>((size_t)kFuseCap * 4, nsm ? (size_t)p->small_lds : 0);
            // the deferred decode rides in the last batch's launch (its blocks come after the
            // write blocks, so they do not change which of those are resident at once)
            const bool take = ride && bi == p->n_large_batches - 1 && ride->rp->n_dec > 0 &&
                              ride->rp->dtype == p->dtype && ride->rp->dec_lds_bytes <= 64 * 1024;
            const DecodeRide<T> dr = make_ride<T>(take ? ride : nullptr);
            if (take) shm = std::max<size_t>(shm, (size_t)ride->rp->dec_lds_bytes);
            e = take && ride->ef == ARCTOPK_EF21
                    ? launch_write_fused<T, ARCTOPK_EF21>(p, bi, nflat, nsm, ckey, sketch, ws, rowlist, slotmap, dr,
                                                          bj, shm, st)
                    : launch_write_fused<T, ARCTOPK_EF_NONE>(p, bi, nflat, nsm, ckey, sketch, ws, rowlist, slotmap,
                                                             dr, bj, shm, st);
            if (e) return e;
            if (bi == 0) *drawn = true;
            if (take && rode) *rode = true;
            continue;
        }
        static const hipError_t lds_ok = hipFuncSetAttribute(
            reinterpret_cast<const void*>(&k_arc_refine<T>), hipFuncAttributeMaxDynamicSharedMemorySize,
            kRefineLdsCap * 4);
        if (lds_ok != hipSuccess) return (int)lds_ok;
        if (bi == 0)
            launch_job_kernel(&k_arc_refine<T>, dim3(b.cnt + nsm + bj.n), dim3(kRefineThreads),
                              (size_t)kRefineLdsCap * 4, st, (const MBatch*)(p->d_large_batches + bi), (int)b.cnt,
                              p->d_mws,
                              (const uint32_t*)ckey, (const SegDev*)p->d_segs, (const int32_t*)p->d_small,
                              sketch, (int)p->r, make_scale(ws), rowlist, slotmap, bj);
        else
            hipLaunchKernelGGL(k_arc_refine<T>, dim3(b.cnt + nsm + bj.n), dim3(kRefineThreads),
                               (size_t)kRefineLdsCap * 4, st, p->d_large_batches + bi, (int)b.cnt, p->d_mws, ckey,
                               p->d_segs,
                               p->d_small, sketch, p->r, make_scale(ws), rowlist, slotmap, bj);
        if (bi == 0) *drawn = true;
        e = (int)hipGetLastError();
        if (e) return e;
        // the last batch's write pass carries the deferred decode, as the fused write does
        const bool take = ride && bi == p->n_large_batches - 1 && ride->rp->n_dec > 0 &&
                          ride->rp->dtype == p->dtype && ride->rp->dec_lds_bytes <= 64 * 1024;
        if (take) {
            const DecodeRide<T> dr = make_ride<T>(ride);
            const size_t shm = (size_t)ride->rp->dec_lds_bytes;
            e = ride->ef == ARCTOPK_EF21 ? launch_write_ride<T, ARCTOPK_EF21>(p, bi, rowlist, slotmap, dr, shm, st)
                                         : launch_write_ride<T, ARCTOPK_EF_NONE>(p, bi, rowlist, slotmap, dr, shm, st);
            if (e) return e;
            if (rode) *rode = true;
            continue;
        }
        e = ms_arc_write(b, p->d_large_batches + bi, p->d_keys, p->d_mws, p->mws_cap, rowlist, slotmap, st);
        if (e) return e;
    }
    return (int)hipGetLastError();
}

// `done`: an event the launch itself completes (hipExtLaunchKernelGGL's stop event, carried
// by the kernel's own completion signal): another stream can wait for the pack without a
// marker packet on this stream (a marker between two kernels idles the GPU ~12 us)
template <typename T, int EF>
void pack_launch(dim3 grid, hipStream_t st, hipEvent_t done, const SegDev* segs, const Chunk* ch,
                 const T* grad, T* err, const int32_t* rowlist, const int32_t* slotmap, T* packed,
                 int32_t* dfirst) {
    if (done)
        hipExtLaunchKernelGGL((k_pack<T, EF>), grid, dim3(256), 0, st, nullptr, done, 0, segs, ch, grad, err,
                              rowlist, slotmap, packed, dfirst);
    else
        hipLaunchKernelGGL((k_pack<T, EF>), grid, dim3(256), 0, st, segs, ch, grad, err, rowlist, slotmap,
                           packed, dfirst);
}

template <typename T>
int launch_pack(const arctopk_plan* p, int c0, int c1, const void* grad_, void* err_, int32_t ef,
                const int32_t* rowlist, const int32_t* slotmap, void* packed_, hipStream_t st,
                hipEvent_t done = nullptr) {
    const T* grad = static_cast<const T*>(grad_);
    T* err = static_cast<T*>(err_);
    T* packed = static_cast<T*>(packed_);
    dim3 grid(c1 - c0);
    const Chunk* ch = p->d_pack + c0;
    if (ef == ARCTOPK_EF_NONE)
        pack_launch<T, ARCTOPK_EF_NONE>(grid, st, done, p->d_segs, ch, grad, err, rowlist, slotmap, packed, p->d_dfirst);
    else if (ef == ARCTOPK_EF14)
        pack_launch<T, ARCTOPK_EF14>(grid, st, done, p->d_segs, ch, grad, err, rowlist, slotmap, packed, p->d_dfirst);
    else if (ef == ARCTOPK_EF21)
        pack_launch<T, ARCTOPK_EF21>(grid, st, done, p->d_segs, ch, grad, err, rowlist, slotmap, packed, p->d_dfirst);
    else
        return ARCTOPK_EINVAL;
    return (int)hipGetLastError();
}

// The mode-3 decode chunk table from a slot map alone (the public decode entry points): for
// mode-3 segment s (one block each), entry dchunk0 + l, l in [0, nch], is the bucket-wide index
// of the first selected row at or after row l * CR -- sel_off plus the selected rows before
// it -- exactly what the pack writes (k_pack, small-m branch); entry nch is the next segment's
// first, written alike by both segments when that one is mode 3 too.
__global__ void __launch_bounds__(256) k_dfirst(const SegDev* __restrict__ segs, const int32_t* __restrict__ m3,
                                                const int32_t* __restrict__ slotmap, int32_t* __restrict__ dfirst) {
    const SegDev s = segs[m3[blockIdx.x]];
    const int64_t CR = s.dchunk_rows;
    const int64_t nch = (s.n + CR - 1) / CR;
    const int32_t* sm = slotmap + s.row_off;
    __shared__ int32_t wsum[4];
    int32_t carry = (int32_t)s.sel_off;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t l0 = 0; l0 <= nch; l0 += 256) {
        const int64_t l = l0 + threadIdx.x;
        int32_t cnt = 0;
        if (l < nch)
            for (int64_t r = l * CR, re = min(s.n, (l + 1) * CR); r < re; ++r) cnt += sm[r] >= 0 ? 1 : 0;
        int32_t x = cnt;  // inclusive scan over the wave, then over the block's 4 waves
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int32_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        int32_t before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            if (w < wave) before += wsum[w];
            total += wsum[w];
        }
        if (l <= nch) dfirst[s.dchunk0 + l] = carry + before + x - cnt;
        carry += total;
        __syncthreads();
    }
}

// `done` as in pack_launch (the decode after an inline all-reduce, watched by exchange.cpp)
template <typename T, int EF>
void decode_launch(dim3 grid, size_t lds, hipStream_t st, hipEvent_t done, const DecodeRide<T>& d) {
    if (done)
        hipExtLaunchKernelGGL((k_decode<T, EF>), grid, dim3(256), lds, st, nullptr, done, 0, d);
    else
        hipLaunchKernelGGL((k_decode<T, EF>), grid, dim3(256), lds, st, d);
}

// decode chunks [c0, c1) of plan p; fin (world size 1): the fused pack + decode from residual E
template <typename T>
int launch_decode(const arctopk_plan* p, int c0, int c1, const int32_t* dfirst, const void* packed_,
                  const int32_t* slotmap, int32_t ws, int32_t ef, void* gerr_, void* out_, hipStream_t st,
                  hipEvent_t done = nullptr, int fin = 0, void* E = nullptr) {
    DecodeRide<T> d{};
    d.segs = p->d_segs;
    d.chunks = p->d_dec + c0;
    d.dfirst = dfirst + c0;
    d.packed = static_cast<const T*>(packed_);
    d.slotmap = slotmap;
    d.gE = static_cast<T*>(gerr_);
    d.out = static_cast<T*>(out_);
    d.sc = make_scale(ws);
    d.n = c1 - c0;
    d.fin = fin;
    d.E = static_cast<T*>(E);
    const dim3 grid(c1 - c0);
    const size_t lds = (size_t)p->dec_lds_bytes;
    if (fin == 3) {
        if (done) hipExtLaunchKernelGGL(k_decode_scatter<T>, grid, dim3(256), 0, st, nullptr, done, 0, d);
        else hipLaunchKernelGGL(k_decode_scatter<T>, grid, dim3(256), 0, st, d);
    } else if (ef == ARCTOPK_EF21 && !fin)
        decode_launch<T, ARCTOPK_EF21>(grid, lds, st, done, d);
    else if (ef == ARCTOPK_EF_NONE || ef == ARCTOPK_EF14)
        decode_launch<T, ARCTOPK_EF_NONE>(grid, lds, st, done, d);
    else
        return ARCTOPK_EINVAL;
    return (int)hipGetLastError();
}

}  // namespace

extern "C" int arctopk_encode(const arctopk_plan* p, const void* grad, void* err, int32_t ef,
                              int32_t err_in, const void* V, void* sketch, void* stream) {
    if (!p || !grad || !sketch) return ARCTOPK_EINVAL;
    if (ef != ARCTOPK_EF_NONE && !err) return ARCTOPK_EINVAL;
    if (ef < 0 || ef > 2) return ARCTOPK_EINVAL;
    if (p->info.v_len > 0 && !V) return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (p->dtype == ARCTOPK_BF16) return launch_encode<bf16_t>(p, grad, err, ef, err_in, V, sketch, nullptr, st);
    return launch_encode<float>(p, grad, err, ef, err_in, V, sketch, nullptr, st);
}

namespace arctopk {
// arctopk_encode at world size 1 for this plan's own select (keys mode): multi-block select
// items get their energy keys written into the plan's key buffer instead of their sketch rows
// (the sketch all-reduce is the identity, so the keys are the select's; its key pass then only
// builds the histograms).  Every other segment's sketch is written as arctopk_encode writes it.
int encode_keyed(const arctopk_plan* p, const void* grad, void* err, int32_t ef, int32_t err_in, const void* V,
                 void* sketch, void* stream, const arctopk_plan* rp, const void* rp_grad, void* rp_err, int* rode,
                 void* done) {
    if (rode) *rode = 0;
    if (!p || !grad || !sketch) return ARCTOPK_EINVAL;
    if (ef != ARCTOPK_EF_NONE && !err) return ARCTOPK_EINVAL;
    if (ef < 0 || ef > 2) return ARCTOPK_EINVAL;
    if (p->info.v_len > 0 && !V) return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    uint32_t* keys = p->any_keyed ? p->d_keys : nullptr;
    // the ride: rp's pack (its bound row list, slot map and packed buffer; its bucket and residual)
    // as the launch's first blocks -- same dtype, and buffers distinct from this call's
    const bool take = rp && rode && rp->dtype == p->dtype && rp->device == p->device && rp->n_pack > 0 &&
                      rp->b_rowlist && rp->b_slotmap && rp->b_packed && (ef == ARCTOPK_EF14 ? rp_err : rp_grad) &&
                      (ef != ARCTOPK_EF21 || rp_err) && rp_grad != grad && (!rp_err || rp_err != err);
    if (p->dtype == ARCTOPK_BF16) {
        PackRide<bf16_t> pr{};
        if (take)
            pr = PackRide<bf16_t>{rp->d_segs, rp->d_pack, static_cast<const bf16_t*>(rp_grad), static_cast<bf16_t*>(rp_err),
                                  rp->b_rowlist, rp->b_slotmap, static_cast<bf16_t*>(rp->b_packed), rp->d_dfirst, rp->n_pack};
        int er_lds = 0;
        const EncRide<bf16_t> er = make_enc_ride<bf16_t>(p, ef, err_in, &er_lds);
        const int e = launch_encode<bf16_t>(p, grad, err, ef, err_in, V, sketch, keys, st, pr, (hipEvent_t)done, er,
                                            er_lds, p->x_carry ? p->x_carry->enc_short != 0 : true);
        if (!e && take) *rode = 1;
        return e;
    }
    PackRide<float> pr{};
    if (take)
        pr = PackRide<float>{rp->d_segs, rp->d_pack, static_cast<const float*>(rp_grad), static_cast<float*>(rp_err),
                             rp->b_rowlist, rp->b_slotmap, static_cast<float*>(rp->b_packed), rp->d_dfirst, rp->n_pack};
    int er_lds = 0;
    const EncRide<float> er = make_enc_ride<float>(p, ef, err_in, &er_lds);
    const int e = launch_encode<float>(p, grad, err, ef, err_in, V, sketch, keys, st, pr, (hipEvent_t)done, er, er_lds,
                                       p->x_carry ? p->x_carry->enc_short != 0 : true);
    if (!e && take) *rode = 1;
    return e;
}
}  // namespace arctopk

extern "C" int arctopk_row_energy(const arctopk_plan* p, const void* sketch, int32_t ws,
                                  float* energy, void* stream) {
    if (!p || !sketch || !energy || ws < 1) return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (p->dtype == ARCTOPK_BF16) return launch_energy<bf16_t>(p, sketch, ws, nullptr, energy, st);
    return launch_energy<float>(p, sketch, ws, nullptr, energy, st);
}

namespace arctopk {
// arctopk_select_draw; keyed: the encode of this call ran in keys mode (arctopk::encode_keyed),
// so the multi-block items' keys are in place (world size 1 only)
int select_draw_keyed(const arctopk_plan* p, const void* sketch, int32_t ws, int32_t* rowlist, int32_t* slotmap,
                      const arctopk_plan* next, uint64_t next_seed, void* next_V, bool keyed, void* stream);
}  // namespace arctopk

extern "C" int arctopk_select_draw(const arctopk_plan* p, const void* sketch, int32_t ws,
                                   int32_t* rowlist, int32_t* slotmap, const arctopk_plan* next,
                                   uint64_t next_seed, void* next_V, void* stream) {
    return arctopk::select_draw_keyed(p, sketch, ws, rowlist, slotmap, next, next_seed, next_V, false, stream);
}

int arctopk::select_draw_keyed(const arctopk_plan* p, const void* sketch, int32_t ws, int32_t* rowlist,
                               int32_t* slotmap, const arctopk_plan* next, uint64_t next_seed, void* next_V,
                               bool keyed, void* stream) {
    if (!p || !sketch || !rowlist || !slotmap || ws < 1 || (keyed && ws != 1)) return ARCTOPK_EINVAL;
    if (next && (!next_V || next->dtype != p->dtype || next->device != p->device)) return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    VDrawJob job{};
    if (next && next->n_vchunk) {
        job.segs = next->d_vdraw;
        job.chunks = next->d_vchunk;
        job.V = next_V;
        job.seed = next_seed;
        job.n = next->n_vchunk;
    }
    bool drawn = false;
    const int e = p->dtype == ARCTOPK_BF16
                      ? launch_select<bf16_t>(p, sketch, ws, rowlist, slotmap, job, &drawn, st, nullptr, nullptr, keyed)
                      : launch_select<float>(p, sketch, ws, rowlist, slotmap, job, &drawn, st, nullptr, nullptr, keyed);
    if (e) return e;
    if (job.n && !drawn) return arctopk_draw_projections(next, next_seed, next_V, stream);
    return 0;
}

namespace {
template <typename T>
int launch_select_ride(const arctopk_plan* p, const void* sketch_, int32_t ws, int32_t* rowlist,
                       int32_t* slotmap, VDrawJob job, const arctopk_plan* rp, int32_t rp_ws, int32_t rp_ef,
                       void* rp_gerr, void* rp_out, hipStream_t st) {
    DecodeRide<T> dr;
    dr.segs = rp->d_segs;
    dr.chunks = rp->d_dec;
    dr.dfirst = rp->d_dfirst;
    dr.packed = static_cast<const T*>(rp->b_packed);
    dr.slotmap = rp->b_slotmap;
    dr.gE = static_cast<T*>(rp_gerr);
    dr.out = static_cast<T*>(rp_out);
    dr.sc = make_scale(rp_ws);
    dr.n = rp->n_dec;
    dr.fin = ride_fin(rp, rp_ef);
    if (dr.fin == 3) dr.fin = 0;
    dr.E = static_cast<T*>(rp->x_err);
    const size_t shm = (size_t)std::max(p->small_lds, rp->dec_lds_bytes);
    const dim3 grid(p->n_small + dr.n + job.n);
    const T* sketch = static_cast<const T*>(sketch_);
    if (rp_ef == ARCTOPK_EF21) {
        if (shm > 48 * 1024) {
            static const hipError_t ok = hipFuncSetAttribute(
                reinterpret_cast<const void*>(&k_select_small_dec<T, ARCTOPK_EF21>),
                hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
            if (ok != hipSuccess) return (int)ok;
        }
        launch_job_kernel(&k_select_small_dec<T, ARCTOPK_EF21>, grid, dim3(kST), shm, st, (const SegDev*)p->d_segs,
                          (const int32_t*)p->d_small, p->n_small, sketch, (int)p->r, make_scale(ws), rowlist,
                          slotmap, dr, job);
    } else {
        if (shm > 48 * 1024) {
            static const hipError_t ok = hipFuncSetAttribute(
                reinterpret_cast<const void*>(&k_select_small_dec<T, ARCTOPK_EF_NONE>),
                hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
            if (ok != hipSuccess) return (int)ok;
        }
        launch_job_kernel(&k_select_small_dec<T, ARCTOPK_EF_NONE>, grid, dim3(kST), shm, st,
                          (const SegDev*)p->d_segs, (const int32_t*)p->d_small, p->n_small, sketch, (int)p->r,
                          make_scale(ws), rowlist, slotmap, dr, job);
    }
    return (int)hipGetLastError();
}
}  // namespace

namespace arctopk {
// arctopk_select_draw with the deferred decode of plan rp (its bound packed buffer and slot map,
// rp_ws, rp_ef, gE and output bucket) in the same launch, when this plan's select is one launch
// of 256-thread single-block selects (*rode = 1); otherwise only the select (*rode = 0: the
// caller decodes rp itself).
int select_ride(const arctopk_plan* p, const void* sketch, int32_t ws, int32_t* rowlist, int32_t* slotmap,
                const arctopk_plan* next, uint64_t next_seed, void* next_V, const arctopk_plan* rp,
                int32_t rp_ws, int32_t rp_ef, void* rp_gerr, void* rp_out, int* rode, void* stream, bool keyed) {
    *rode = 0;
    if (keyed && ws != 1) return ARCTOPK_EINVAL;
    constexpr int64_t big_rows = ARCTOPK_SEL_BIG_ROWS;
    const bool rideable = rp && rp->dtype == p->dtype && rp->device == p->device && rp->n_dec > 0 &&
                          rp->b_packed && rp->b_slotmap && rp_out && (rp_ef != ARCTOPK_EF21 || rp_gerr) &&
                          rp->dec_lds_bytes <= 64 * 1024;
    const bool fusable = rideable && p->n_small > 0 && p->n_large_batches == 0 &&
                         !(p->small_lds > big_rows * 4 + 16) && p->small_lds <= 48 * 1024;
    if (rideable && p->n_large_batches > 0) {  // multi-block select: ride in its fused write launch
        if (!p || !sketch || !rowlist || !slotmap || ws < 1 || rp_ws < 1) return ARCTOPK_EINVAL;
        if (next && (!next_V || next->dtype != p->dtype || next->device != p->device)) return ARCTOPK_EINVAL;
        VDrawJob job{};
        if (next && next->n_vchunk) {
            job.segs = next->d_vdraw;
            job.chunks = next->d_vchunk;
            job.V = next_V;
            job.seed = next_seed;
            job.n = next->n_vchunk;
        }
        const RideArgs ra{rp, rp_ws, rp_ef, rp_gerr, rp_out};
        bool drawn = false, took = false;
        hipStream_t st = (hipStream_t)stream;
        const int e = p->dtype == ARCTOPK_BF16
                          ? launch_select<bf16_t>(p, sketch, ws, rowlist, slotmap, job, &drawn, st, &ra, &took, keyed)
                          : launch_select<float>(p, sketch, ws, rowlist, slotmap, job, &drawn, st, &ra, &took, keyed);
        if (e) return e;
        *rode = took ? 1 : 0;
        if (job.n && !drawn) return arctopk_draw_projections(next, next_seed, next_V, stream);
        return 0;
    }
    if (!fusable) return select_draw_keyed(p, sketch, ws, rowlist, slotmap, next, next_seed, next_V, keyed, stream);
    if (!p || !sketch || !rowlist || !slotmap || ws < 1 || rp_ws < 1) return ARCTOPK_EINVAL;
    if (next && (!next_V || next->dtype != p->dtype || next->device != p->device)) return ARCTOPK_EINVAL;
    VDrawJob job{};
    if (next && next->n_vchunk) {
        job.segs = next->d_vdraw;
        job.chunks = next->d_vchunk;
        job.V = next_V;
        job.seed = next_seed;
        job.n = next->n_vchunk;
    }
    hipStream_t st = (hipStream_t)stream;
    const int e = p->dtype == ARCTOPK_BF16
                      ? launch_select_ride<bf16_t>(p, sketch, ws, rowlist, slotmap, job, rp, rp_ws, rp_ef, rp_gerr,
                                                   rp_out, st)
                      : launch_select_ride<float>(p, sketch, ws, rowlist, slotmap, job, rp, rp_ws, rp_ef, rp_gerr,
                                                  rp_out, st);
    if (!e) *rode = 1;
    return e;
}
}  // namespace arctopk

extern "C" int arctopk_select(const arctopk_plan* p, const void* sketch, int32_t ws,
                              int32_t* rowlist, int32_t* slotmap, void* stream) {
    return arctopk_select_draw(p, sketch, ws, rowlist, slotmap, nullptr, 0, nullptr, stream);
}

extern "C" int arctopk_pack_segments(const arctopk_plan* p, int32_t seg_begin, int32_t seg_end,
                                     const void* grad, void* err, int32_t ef,
                                     const int32_t* rowlist, const int32_t* slotmap, void* packed,
                                     void* stream) {
    if (!p || !rowlist || !slotmap || !packed) return ARCTOPK_EINVAL;
    if (seg_begin < 0 || seg_end > p->nseg || seg_begin > seg_end) return ARCTOPK_EINVAL;
    if (ef < 0 || ef > 2) return ARCTOPK_EINVAL;
    if (ef == ARCTOPK_EF_NONE ? !grad : !err) return ARCTOPK_EINVAL;
    if (ef == ARCTOPK_EF21 && !grad) return ARCTOPK_EINVAL;
    const int c0 = p->h_pack_begin[seg_begin], c1 = p->h_pack_begin[seg_end];
    if (c1 == c0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (p->dtype == ARCTOPK_BF16) return launch_pack<bf16_t>(p, c0, c1, grad, err, ef, rowlist, slotmap, packed, st);
    return launch_pack<float>(p, c0, c1, grad, err, ef, rowlist, slotmap, packed, st);
}

extern "C" int arctopk_pack(const arctopk_plan* p, const void* grad, void* err, int32_t ef,
                            const int32_t* rowlist, const int32_t* slotmap, void* packed, void* stream) {
    if (!p) return ARCTOPK_EINVAL;
    return arctopk_pack_segments(p, 0, p->nseg, grad, err, ef, rowlist, slotmap, packed, stream);
}

namespace arctopk {
// arctopk_pack whose kernel completes `done` (exchange.cpp)
int pack_signal(const arctopk_plan* p, const void* grad, void* err, int32_t ef, const int32_t* rowlist,
                const int32_t* slotmap, void* packed, void* stream, void* done) {
    if (!p || !rowlist || !slotmap || !packed || !done) return ARCTOPK_EINVAL;
    if (ef < 0 || ef > 2) return ARCTOPK_EINVAL;
    if (ef == ARCTOPK_EF_NONE ? !grad : !err) return ARCTOPK_EINVAL;
    if (ef == ARCTOPK_EF21 && !grad) return ARCTOPK_EINVAL;
    const int c0 = p->h_pack_begin[0], c1 = p->h_pack_begin[p->nseg];
    if (c1 == c0) return (int)hipEventRecord((hipEvent_t)done, (hipStream_t)stream);
    hipStream_t st = (hipStream_t)stream;
    if (p->dtype == ARCTOPK_BF16)
        return launch_pack<bf16_t>(p, c0, c1, grad, err, ef, rowlist, slotmap, packed, st, (hipEvent_t)done);
    return launch_pack<float>(p, c0, c1, grad, err, ef, rowlist, slotmap, packed, st, (hipEvent_t)done);
}
}  // namespace arctopk

extern "C" int arctopk_decode_segments(const arctopk_plan* p, int32_t seg_begin, int32_t seg_end,
                                       const void* packed, const int32_t* slotmap, int32_t ws,
                                       int32_t ef, void* gerr, void* out, void* stream) {
    if (!p || !packed || !slotmap || !out || ws < 1) return ARCTOPK_EINVAL;
    if (seg_begin < 0 || seg_end > p->nseg || seg_begin > seg_end) return ARCTOPK_EINVAL;
    if (ef < 0 || ef > 2) return ARCTOPK_EINVAL;
    if (ef == ARCTOPK_EF21 && !gerr) return ARCTOPK_EINVAL;
    const int c0 = p->h_dec_begin[seg_begin], c1 = p->h_dec_begin[seg_end];
    if (c1 == c0) return 0;
    hipStream_t st = (hipStream_t)stream;
    // mode-3 chunks read their packed range from a chunk table; the one the plan's pack writes
    // describes the pack's own row list, so here it is derived from the slot map given (the
    // caller may hand any slot map and packed buffer of arctopk_select / arctopk_pack's format)
    if (p->n_m3) {
        hipLaunchKernelGGL(k_dfirst, dim3(p->n_m3), dim3(256), 0, st, p->d_segs, p->d_m3, slotmap, p->d_dfirst_pub);
        const hipError_t he = hipGetLastError();
        if (he != hipSuccess) return (int)he;
    }
    if (p->dtype == ARCTOPK_BF16)
        return launch_decode<bf16_t>(p, c0, c1, p->d_dfirst_pub, packed, slotmap, ws, ef, gerr, out, st);
    return launch_decode<float>(p, c0, c1, p->d_dfirst_pub, packed, slotmap, ws, ef, gerr, out, st);
}

extern "C" int arctopk_decode(const arctopk_plan* p, const void* packed, const int32_t* slotmap,
                              int32_t ws, int32_t ef, void* gerr, void* out, void* stream) {
    if (!p) return ARCTOPK_EINVAL;
    return arctopk_decode_segments(p, 0, p->nseg, packed, slotmap, ws, ef, gerr, out, stream);
}

namespace {
template <typename T>
int launch_decode_pair(const RideArgs& a, const RideArgs& b, hipStream_t st, hipEvent_t done) {
    const DecodeRide<T> da = make_ride<T>(&a), db = make_ride<T>(&b);
    const size_t lds = (size_t)std::max(a.rp->dec_lds_bytes, b.rp->dec_lds_bytes);
    const dim3 grid(da.n + db.n);
    if (a.ef == ARCTOPK_EF21) {
        if (done) hipExtLaunchKernelGGL((k_decode2<T, ARCTOPK_EF21>), grid, dim3(256), lds, st, nullptr, done, 0, da, db);
        else hipLaunchKernelGGL((k_decode2<T, ARCTOPK_EF21>), grid, dim3(256), lds, st, da, db);
    } else {
        if (done) hipExtLaunchKernelGGL((k_decode2<T, ARCTOPK_EF_NONE>), grid, dim3(256), lds, st, nullptr, done, 0, da, db);
        else hipLaunchKernelGGL((k_decode2<T, ARCTOPK_EF_NONE>), grid, dim3(256), lds, st, da, db);
    }
    return (int)hipGetLastError();
}
}  // namespace

namespace arctopk {
// Two plans' whole-bucket decodes in one launch (same dtype and EF class, both with decode
// chunks, LDS within 48 KiB); `done` as in decode_signal (may be null).  Returns
// ARCTOPK_EINVAL when the pair does not qualify (the caller then decodes them one by one).
int decode_pair(const arctopk_plan* pa, int32_t ws_a, int32_t ef_a, void* gerr_a, void* out_a,
                const arctopk_plan* pb, int32_t ws_b, int32_t ef_b, void* gerr_b, void* out_b, void* stream,
                void* done) {
    if (!pa || !pb || !out_a || !out_b || pa->dtype != pb->dtype || ws_a < 1 || ws_b < 1) return ARCTOPK_EINVAL;
    if ((ef_a == ARCTOPK_EF21) != (ef_b == ARCTOPK_EF21) || ef_a < 0 || ef_a > 2 || ef_b < 0 || ef_b > 2)
        return ARCTOPK_EINVAL;
    if (ef_a == ARCTOPK_EF21 && (!gerr_a || !gerr_b)) return ARCTOPK_EINVAL;
    if (pa->n_dec <= 0 || pb->n_dec <= 0 || std::max(pa->dec_lds_bytes, pb->dec_lds_bytes) > 48 * 1024)
        return ARCTOPK_EINVAL;
    if (pa->h_dec_begin[0] != 0 || pb->h_dec_begin[0] != 0) return ARCTOPK_EINVAL;
    const RideArgs a{pa, ws_a, ef_a, gerr_a, out_a}, b{pb, ws_b, ef_b, gerr_b, out_b};
    hipStream_t st = (hipStream_t)stream;
    if (pa->dtype == ARCTOPK_BF16) return launch_decode_pair<bf16_t>(a, b, st, (hipEvent_t)done);
    return launch_decode_pair<float>(a, b, st, (hipEvent_t)done);
}

// The whole-bucket decode of the packed values and slot map this plan's own last pack wrote
// (its chunk table, d_dfirst, describes them); `done` (may be null): an event the kernel
// completes (exchange.cpp)
int decode_signal(const arctopk_plan* p, const void* packed, const int32_t* slotmap, int32_t ws, int32_t ef,
                  void* gerr, void* out, void* stream, void* done) {
    if (!p || !packed || !slotmap || !out || ws < 1) return ARCTOPK_EINVAL;
    if (ef < 0 || ef > 2) return ARCTOPK_EINVAL;
    if (ef == ARCTOPK_EF21 && !gerr) return ARCTOPK_EINVAL;
    const int c0 = p->h_dec_begin[0], c1 = p->h_dec_begin[p->nseg];
    hipStream_t st = (hipStream_t)stream;
    if (c1 == c0) return done ? (int)hipEventRecord((hipEvent_t)done, st) : 0;
    const int fin = ride_fin(p, ef);
    if (p->dtype == ARCTOPK_BF16)
        return launch_decode<bf16_t>(p, c0, c1, p->d_dfirst, packed, slotmap, ws, ef, gerr, out, st, (hipEvent_t)done,
                                     fin, p->x_err);
    return launch_decode<float>(p, c0, c1, p->d_dfirst, packed, slotmap, ws, ef, gerr, out, st, (hipEvent_t)done,
                                fin, p->x_err);
}
}  // namespace arctopk

extern "C" int arctopk_ef_apply(void* x_, void* E_, int64_t n, int32_t ef, int32_t err_in,
                                int32_t dtype, void* stream) {
    if (!x_ || n < 0) return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EINVAL;
    if (ef == ARCTOPK_EF_NONE || n == 0) return 0;
    if (!E_) return ARCTOPK_EINVAL;
    if (dtype == ARCTOPK_BF16) {
        bf16_t* x = static_cast<bf16_t*>(x_);
        bf16_t* E = static_cast<bf16_t*>(E_);
        const dim3 g((unsigned)std::min<int64_t>(8192, (n + 255) / 256));
        hipStream_t st = (hipStream_t)stream;
        if (ef == ARCTOPK_EF14 && err_in)
            hipLaunchKernelGGL((k_ef_apply_bf16<ARCTOPK_EF14, true>), g, dim3(256), 0, st, x, E, n);
        else if (ef == ARCTOPK_EF14)
            hipLaunchKernelGGL((k_ef_apply_bf16<ARCTOPK_EF14, false>), g, dim3(256), 0, st, x, E, n);
        else if (ef == ARCTOPK_EF21)
            hipLaunchKernelGGL((k_ef_apply_bf16<ARCTOPK_EF21, true>), g, dim3(256), 0, st, x, E, n);
        else
            return ARCTOPK_EINVAL;
        return (int)hipGetLastError();
    }
    float* x = static_cast<float*>(x_);
    float* E = static_cast<float*>(E_);
    // float4 path needs 16-B aligned x and E (torch allocations are)
    if (((uintptr_t)x | (uintptr_t)E) & 15) return ARCTOPK_EINVAL;
    const int grid = (int)std::min<int64_t>(8192, (n / 4 + 255) / 256 + 1);
    hipStream_t st = (hipStream_t)stream;
    if (ef == ARCTOPK_EF14 && err_in)
        hipLaunchKernelGGL((k_ef_apply<ARCTOPK_EF14, true>), dim3(grid), dim3(256), 0, st, x, E, n);
    else if (ef == ARCTOPK_EF14)
        hipLaunchKernelGGL((k_ef_apply<ARCTOPK_EF14, false>), dim3(grid), dim3(256), 0, st, x, E, n);
    else if (ef == ARCTOPK_EF21)
        hipLaunchKernelGGL((k_ef_apply<ARCTOPK_EF21, true>), dim3(grid), dim3(256), 0, st, x, E, n);
    else
        return ARCTOPK_EINVAL;
    return (int)hipGetLastError();
}

// EF14 fold for the sparse hooks: E := x + E (err_in) or E := x (first call), x untouched.
// Replaces input_tensor.add_(E) (sparse_hook.py:205) and E.copy_(input_tensor) (:258): the
// caller then selects / gathers from E and decodes into x, so x is written once, by the
// decode, instead of twice.
extern "C" int arctopk_ef14_fold(const void* x_, void* E_, int64_t n, int32_t err_in, int32_t dtype,
                                 void* stream) {
    if (!x_ || !E_ || n < 0) return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EINVAL;
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == ARCTOPK_BF16) {
        bf16_t* x = static_cast<bf16_t*>(const_cast<void*>(x_));
        bf16_t* E = static_cast<bf16_t*>(E_);
        const dim3 g((unsigned)std::min<int64_t>(8192, (n + 255) / 256));
        if (err_in)
            hipLaunchKernelGGL((k_ef_apply_bf16<ARCTOPK_EF14, true, false>), g, dim3(256), 0, st, x, E, n);
        else
            hipLaunchKernelGGL((k_ef_apply_bf16<ARCTOPK_EF14, false, false>), g, dim3(256), 0, st, x, E, n);
        return (int)hipGetLastError();
    }
    float* x = static_cast<float*>(const_cast<void*>(x_));
    float* E = static_cast<float*>(E_);
    if (((uintptr_t)x | (uintptr_t)E) & 15) return ARCTOPK_EINVAL;
    const int grid = (int)std::min<int64_t>(8192, (n / 4 + 255) / 256 + 1);
    if (err_in)
        hipLaunchKernelGGL((k_ef_apply<ARCTOPK_EF14, true, false>), dim3(grid), dim3(256), 0, st, x, E, n);
    else
        hipLaunchKernelGGL((k_ef_apply<ARCTOPK_EF14, false, false>), dim3(grid), dim3(256), 0, st, x, E, n);
    return (int)hipGetLastError();
}

// Test entry point: the device's fp32 -> bf16 rounding (the one every kernel uses) on n
// values, for checking it against c10::BFloat16's round-to-nearest-even on the host.
__global__ void __launch_bounds__(256) k_round_bf16(const float* __restrict__ in, uint16_t* __restrict__ out,
                                                    int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = from_f<bf16_t>(in[i]).u;
}

extern "C" int arctopk_round_bf16(const float* in, uint16_t* out, int64_t n, void* stream) {
    if (!in || !out || n < 0) return ARCTOPK_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_round_bf16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       in, out, n);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// World-size-1 step (arctopk_step): [draw] -> encode -> select (+ the next call's
// projections) -> pack -> decode as plain launches on the caller's stream.  (Replaying the
// step as a captured HIP graph was measured on MI355X / ROCm 7 in round 2: no host time
// saved, 19.0 vs 19.4 us per ResNet-18 bucket call, and device time lost, headline 1193 ->
// 1162 GB/s; it was removed.)
// ---------------------------------------------------------------------------
namespace {
inline int step_mark(void* const* marks, int i, hipStream_t st) {
    if (!marks || !marks[i]) return 0;
    return (int)hipEventRecord((hipEvent_t)marks[i], st);
}
}  // namespace

extern "C" int arctopk_step(const arctopk_plan* p, void* bucket, void* err, void* gerr, int32_t ef,
                            int32_t err_in, int32_t draw, uint64_t seed, const arctopk_plan* next,
                            uint64_t next_seed, void* stream, void* const* marks) {
    if (!p || !bucket || !p->b_sketch) return ARCTOPK_EINVAL;  // unbound plan
    if (next && (!next->b_sketch || next->dtype != p->dtype || next->device != p->device)) return ARCTOPK_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    int e = step_mark(marks, ARCTOPK_MARK_START, st);
    if (!e && draw && p->info.v_len > 0) e = arctopk_draw_projections(p, seed, p->b_V, stream);
    if (!e) e = step_mark(marks, ARCTOPK_MARK_DRAW, st);
    if (!e) e = arctopk::encode_keyed(p, bucket, err, ef, err_in, p->b_V, p->b_sketch, st);
    if (!e) e = step_mark(marks, ARCTOPK_MARK_ENCODE, st);
    if (!e)
        e = arctopk::select_draw_keyed(p, p->b_sketch, 1, p->b_rowlist, p->b_slotmap, next, next_seed,
                                       next ? next->b_V : nullptr, true, st);
    if (!e) e = step_mark(marks, ARCTOPK_MARK_SELECT, st);
    if (!e) e = arctopk_pack(p, bucket, err, ef, p->b_rowlist, p->b_slotmap, p->b_packed, st);
    if (!e) e = step_mark(marks, ARCTOPK_MARK_PACK, st);
    if (!e) e = arctopk::decode_signal(p, p->b_packed, p->b_slotmap, 1, ef, gerr, bucket, st, nullptr);
    if (!e) e = step_mark(marks, ARCTOPK_MARK_DECODE, st);
    return e;
}
