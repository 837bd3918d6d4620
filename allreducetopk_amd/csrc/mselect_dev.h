// Device helpers of the multi-block select shared by mselect.hip and the ARC launches in
// arctopk_kernels.hip (the write pass runs there with a deferred decode riding in its launch).
#pragma once
#include <hip/hip_runtime.h>

#include "mselect.h"

namespace arctopk {

constexpr int kPerLane = kMTile / 256;  // keys per lane of a tile (16)

// key sources: 0 = uint32 keys (ARC energies), 1 = |x| of fp32 x, 2 = |x| of bf16 x (the bf16
// bits widened to the fp32 bit pattern of the same value: exact, so the order is bf16's);
// 3 / 4 = RandK hash keys (rk_key of the index) with fp32 / bf16 x as the value source
template <int SRC>
__device__ __forceinline__ uint32_t load_bits(const uint32_t* __restrict__ keys,
                                              const void* __restrict__ x, int64_t i) {
    if constexpr (SRC == 1 || SRC == 3) return __float_as_uint(static_cast<const float*>(x)[i]);
    else if constexpr (SRC == 2 || SRC == 4) return (uint32_t)static_cast<const uint16_t*>(x)[i] << 16;
    else return keys[i];
}

// |x| for TopK keys: NaN sorts above inf
template <int SRC>
__device__ __forceinline__ uint32_t key_of(uint32_t bits) {
    if constexpr (SRC != 0) return bits & 0x7FFFFFFFu;
    else return bits;
}

// RandK keys: a keyed bijection of the element's index in its tensor (xorshift-multiply rounds,
// each invertible on 32 bits), so the keys of a tensor are distinct and the k largest form a
// uniformly random k-subset -- selected by the same exact radix select as TopK, ascending
__device__ __forceinline__ uint32_t rk_mix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ uint32_t rk_key(uint32_t seed, int64_t i) {
    return rk_mix(rk_mix((uint32_t)i ^ seed) + 0x9E3779B9u * (seed | 1u));
}

// the select key of element i (index within its item)
template <int SRC>
__device__ __forceinline__ uint32_t item_key(const MItem& it, const uint32_t* __restrict__ keys,
                                             const void* __restrict__ x, int64_t i) {
    if constexpr (SRC >= 3) return rk_key(it.hseed, i);
    else return key_of<SRC>(load_bits<SRC>(keys, x, it.key_off + i));
}

// the selected value of x (TopK / RandK outputs), in x's own type
template <int SRC>
__device__ __forceinline__ void store_val(void* __restrict__ out, int64_t j, uint32_t bits) {
    if constexpr (SRC == 1 || SRC == 3) static_cast<float*>(out)[j] = __uint_as_float(bits);
    else if constexpr (SRC == 2 || SRC == 4) static_cast<uint16_t*>(out)[j] = (uint16_t)(bits >> 16);
}

__device__ __forceinline__ uint32_t popc64(uint64_t v) { return (uint32_t)__popcll(v); }

// TopK (!ARC) with zero_x (= x): the tile is rewritten with its selected elements zeroed,
// whole tiles, so no line is left partially dirty -- EF14's `tensor.view(-1)[indices] = 0`
// (sparse_hook.py:104) fused into the pass that already reads every element
// FOLD (RandK hash keys only: the keys do not depend on x, so the select's earlier passes never
// read it): x is the bucket G and zero_x the residual E, and the pass applies EF14 itself --
// v = G + E (FOLD 1; FOLD 2, the first call: v = G), rounded to x's type as the reference's
// tensor.add_(E) (sparse_hook.py:205) -- gathers v, and writes E := v with the selected
// elements zeroed (:104): the separate fold pass over G and E is not needed.
template <int SRC>
__device__ __forceinline__ uint32_t fold_bits(const void* __restrict__ g, const void* __restrict__ e, int64_t i,
                                              int fold) {
    if constexpr (SRC == 3) {
        const float gv = static_cast<const float*>(g)[i];
        return __float_as_uint(fold == 1 ? __fadd_rn(gv, static_cast<const float*>(e)[i]) : gv);
    } else {
        const bf16_t gv = static_cast<const bf16_t*>(g)[i];
        if (fold != 1) return (uint32_t)gv.u << 16;
        const float f = __fadd_rn(to_f(gv), to_f(static_cast<const bf16_t*>(e)[i]));
        return (uint32_t)from_f<bf16_t>(f).u << 16;
    }
}

template <int SRC, bool ARC, int FOLD = 0>
__device__ __forceinline__ void ms_write_body(const MBatch& b, int t, int r, const uint32_t* __restrict__ keys,
                                              const void* __restrict__ x, MWorkspace* ws,
                                              int32_t* __restrict__ out_idx, void* __restrict__ out_val,
                                              int32_t* __restrict__ out_slot, void* zero_x) {
    static_assert(FOLD == 0 || SRC >= 3, "the fused EF14 fold needs keys that do not read x");
    __shared__ uint32_t s_eq[4], s_gt[4];
    const MItem it = b.it[t];
    const uint32_t T = ws->st[t].prefix;
    uint32_t take_left = ws->take_eq[t][r];
    int64_t run = ws->sel_before[t][r];
    const int64_t r0 = (int64_t)r * it.range;
    const int64_t r1 = min<int64_t>(it.n, r0 + it.range);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int64_t tile = r0; tile < r1; tile += kMTile) {
        const int64_t wb = tile + (int64_t)wave * (kMTile / 4);
        uint32_t bits[kPerLane], kv[kPerLane];  // x's bits (TopK: also the key's source), the keys
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) {
            const int64_t i = min<int64_t>(wb + j * 64 + lane, r1 - 1);
            if constexpr (SRC >= 3) {  // RandK: keys from the index; x only for values / zero_x
                kv[j] = rk_key(it.hseed, i);
                if constexpr (FOLD != 0) bits[j] = fold_bits<SRC>(x, zero_x, it.key_off + i, FOLD);
                else bits[j] = x ? load_bits<SRC>(keys, x, it.key_off + i) : 0u;
            } else {
                bits[j] = load_bits<SRC>(keys, x, it.key_off + i);
                kv[j] = key_of<SRC>(bits[j]);
            }
        }
        uint32_t weq = 0, wgt = 0;
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) {
            const bool valid = wb + j * 64 + lane < r1;
            const uint32_t key = kv[j];
            weq += popc64(__ballot(valid && key == T));
            wgt += popc64(__ballot(valid && key > T));
        }
        if (lane == 0) {
            s_eq[wave] = weq;
            s_gt[wave] = wgt;
        }
        __syncthreads();
        uint32_t eqb = 0, gtb = 0, teq = 0, tgt = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            eqb += w < wave ? s_eq[w] : 0u;
            gtb += w < wave ? s_gt[w] : 0u;
            teq += s_eq[w];
            tgt += s_gt[w];
        }
        __syncthreads();
        uint32_t run_eq = eqb;
        int64_t run_sel = run + gtb + min(eqb, take_left);
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) {
            const int64_t i = wb + j * 64 + lane;
            const bool valid = i < r1;
            const uint32_t key = kv[j];
            const bool eq = valid && key == T;
            const bool gt = valid && key > T;
            const uint64_t beq = __ballot(eq);
            const bool sel = gt || (eq && run_eq + popc64(beq & lt) < take_left);
            const uint64_t bsel = __ballot(sel);
            const int64_t my = run_sel + popc64(bsel & lt);
            if (sel && my < it.k) {  // bound: never store past the item's k outputs
                out_idx[it.out_off + my] = (int32_t)i;
                if constexpr (!ARC) {
                    if (out_val) store_val<SRC>(out_val, it.out_off + my, bits[j]);
                }
            }
            if constexpr (ARC) {
                if (valid) out_slot[it.slot_off + i] = sel ? (int32_t)my : -1;
            } else {
                if (zero_x && valid) {
                    if constexpr (SRC == 1 || SRC == 3) static_cast<float*>(zero_x)[it.key_off + i] = sel ? 0.f : __uint_as_float(bits[j]);
                    else if constexpr (SRC == 2 || SRC == 4) static_cast<uint16_t*>(zero_x)[it.key_off + i] = sel ? (uint16_t)0 : (uint16_t)(bits[j] >> 16);
                }
            }
            run_eq += popc64(beq);
            run_sel += popc64(bsel);
        }
        const uint32_t te = min(teq, take_left);
        run += tgt + te;
        take_left -= te;
    }
}

// ARC: one block per range, no atomics: the keys above the first-pass bin are counted and
// the bin's keys are copied (in index order) into the range's own candidate region;
// cnt_gt / cnt_cand per range for the refine.
__device__ inline void arc_compact_range(const MItem it, int t, int r, const uint32_t* __restrict__ keys,
                                         MWorkspace* ws, uint32_t* __restrict__ ckey) {
    __shared__ uint32_t lds[4], s_cnt[4], s_and[4];
    uint32_t d;  // the first-pass bin (keys above it are selected; its keys are the candidates)
    {
        __shared__ uint32_t lds_d[256 + 128];
        uint32_t acc;
        ms_arc_digit_local<256>(ws->hist[t], it.k, lds_d, &d, &acc);
        if (r == 0 && threadIdx.x == 0) {  // the item's state for the refine (next launch)
            MState g;
            arc_bin_state(d, &g.prefix, &g.mask, &g.bit);
            g.cand = 1;
            g.kk = it.k - (int64_t)acc;
            g.p1 = g.prefix;
            g.m1 = g.mask;
            g.ncand = 0;
            ws->st[t] = g;
        }
    }
    const int64_t r0 = (int64_t)r * it.range;
    const int64_t r1 = min<int64_t>(it.n, r0 + it.range);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t* dst = ckey + it.cand_off + r0;
    uint32_t gt = 0, run = 0, kor = 0u, kand = ~0u;
    for (int64_t tile = r0; tile < r1; tile += kMTile) {
        const int64_t wb = tile + (int64_t)wave * (kMTile / 4);
        uint32_t kv[kPerLane];
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) kv[j] = keys[it.key_off + min<int64_t>(wb + j * 64 + lane, r1 - 1)];
        uint64_t bm[kPerLane];
        uint32_t nin = 0;
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) {
            const bool valid = wb + j * 64 + lane < r1;
            const uint32_t dj = arc_digit(kv[j]);
            gt += (valid && dj > d) ? 1u : 0u;
            bm[j] = __ballot(valid && dj == d);
            nin += popc64(bm[j]);
        }
        if (lane == 0) s_cnt[wave] = nin;
        __syncthreads();
        uint32_t base = run, tot = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            base += w < wave ? s_cnt[w] : 0u;
            tot += s_cnt[w];
        }
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) {
            if ((bm[j] >> lane) & 1ull) {
                dst[base + popc64(bm[j] & lt)] = kv[j];
                kor |= kv[j];
                kand &= kv[j];
            }
            base += popc64(bm[j]);
        }
        run += tot;
        __syncthreads();  // s_cnt is rewritten by the next tile
    }
    // block totals: keys above the bin, OR / AND of the bin's keys (one barrier)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        gt += __shfl_xor(gt, o, 64);
        kor |= __shfl_xor(kor, o, 64);
        kand &= __shfl_xor(kand, o, 64);
    }
    if (lane == 0) {
        lds[wave] = gt;
        s_cnt[wave] = kor;
        s_and[wave] = kand;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ws->cnt_gt[t][r] = lds[0] + lds[1] + lds[2] + lds[3];
        ws->cnt_cand[t][r] = run;
        ws->cand_or[t][r] = s_cnt[0] | s_cnt[1] | s_cnt[2] | s_cnt[3];
        ws->cand_and[t][r] = s_and[0] & s_and[1] & s_and[2] & s_and[3];
    }
}

}  // namespace arctopk
