// Multi-block exact top-k selection (see mselect.h for the algorithm).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "mselect.h"

namespace arctopk {
namespace {

template <bool FROM_FLOAT>
__device__ __forceinline__ uint32_t load_key(const uint32_t* __restrict__ keys,
                                             const float* __restrict__ x, int64_t i) {
    if constexpr (FROM_FLOAT) return __float_as_uint(x[i]) & 0x7FFFFFFFu;  // |x|; NaN above inf
    else return keys[i];
}

// item start state.  FROM_FLOAT: |x| keys, only the sign bit is known.  Otherwise the
// caller's key pass left the OR / AND of all keys in the state: their common leading
// bits are fixed, so the first digit falls on varying bits.
template <bool FROM_FLOAT>
__global__ void k_ms_init(MBatch b, MWorkspace* ws) {
    const int t = blockIdx.x;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) ws->hist[t][i] = 0;
    if (threadIdx.x == 0) {
        MState& s = ws->st[t];
        if constexpr (FROM_FLOAT) {
            s.prefix = 0;
            s.mask = 0x80000000u;
            s.bit = 31;
        } else {
            const uint32_t diff = s.kor ^ s.kand;
            const int bit = diff ? 32 - __clz(diff) : 0;
            const uint32_t low = bit == 32 ? 0xFFFFFFFFu : ((1u << bit) - 1u);
            s.prefix = s.kand & ~low;
            s.mask = ~low;
            s.bit = bit;
        }
        s.kk = b.it[t].k;
    }
}

__global__ void k_ms_reset_orand(MWorkspace* ws, int cnt) {
    const int t = threadIdx.x;
    if (t < cnt) {
        ws->st[t].kor = 0u;
        ws->st[t].kand = 0xFFFFFFFFu;
    }
}

template <bool FROM_FLOAT>
__global__ void __launch_bounds__(256) k_ms_hist(MBatch b, const uint32_t* __restrict__ keys,
                                                 const float* __restrict__ x, MWorkspace* ws) {
    __shared__ uint32_t h[4][256];  // one copy per wave: fewer same-address atomics
    const int t = blockIdx.y;
    const MState s = ws->st[t];
    if (s.bit <= 0) return;
    const int w = s.bit < 8 ? s.bit : 8;
    const int shift = s.bit - w;
    const uint32_t dmask = (1u << w) - 1u;
    const int wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4 * 256; i += 256) (&h[0][0])[i] = 0;
    __syncthreads();
    const MItem it = b.it[t];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < it.n; i += (int64_t)gridDim.x * 256) {
        const uint32_t key = load_key<FROM_FLOAT>(keys, x, it.key_off + i);
        if ((key & s.mask) == s.prefix) atomicAdd(&h[wave][(key >> shift) & dmask], 1u);
    }
    __syncthreads();
    const uint32_t c = h[0][threadIdx.x] + h[1][threadIdx.x] + h[2][threadIdx.x] + h[3][threadIdx.x];
    if (c) atomicAdd(&ws->hist[t][threadIdx.x], c);
}

__global__ void k_ms_digit(MBatch b, MWorkspace* ws) {
    const int t = blockIdx.x;
    const int lane = threadIdx.x;
    MState s = ws->st[t];
    if (s.bit > 0) {
        const int w = s.bit < 8 ? s.bit : 8;
        const int shift = s.bit - w;
        uint32_t c[4], sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            c[q] = ws->hist[t][255 - 4 * lane - q];
            sum += c[q];
        }
        uint64_t incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        const uint64_t excl = incl - sum;
        if (excl < (uint64_t)s.kk && incl >= (uint64_t)s.kk) {
            uint64_t acc = excl;
            int q = 0;
            for (; q < 3; ++q) {
                if (acc + c[q] >= (uint64_t)s.kk) break;
                acc += c[q];
            }
            const uint32_t d = 255 - 4 * lane - q;
            MState& g = ws->st[t];
            g.prefix = s.prefix | (d << shift);
            g.mask = s.mask | (((1u << w) - 1u) << shift);
            g.kk = s.kk - (int64_t)acc;
            g.bit = shift;
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) ws->hist[t][4 * lane + q] = 0;
}

template <bool FROM_FLOAT>
__global__ void __launch_bounds__(256) k_ms_count(MBatch b, const uint32_t* __restrict__ keys,
                                                  const float* __restrict__ x, MWorkspace* ws) {
    __shared__ int64_t s_gt[4], s_eq[4];
    const int t = blockIdx.y;
    const MItem it = b.it[t];
    const int64_t per = (it.n + kMRanges - 1) / kMRanges;
    const int64_t r0 = min<int64_t>(it.n, blockIdx.x * per), r1 = min<int64_t>(it.n, r0 + per);
    const uint32_t T = ws->st[t].prefix;
    int64_t gt = 0, eq = 0;
    for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) {
        const uint32_t key = load_key<FROM_FLOAT>(keys, x, it.key_off + i);
        gt += key > T;
        eq += key == T;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        gt += __shfl_xor(gt, o, 64);
        eq += __shfl_xor(eq, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        s_gt[threadIdx.x >> 6] = gt;
        s_eq[threadIdx.x >> 6] = eq;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ws->cnt_gt[t][blockIdx.x] = s_gt[0] + s_gt[1] + s_gt[2] + s_gt[3];
        ws->cnt_eq[t][blockIdx.x] = s_eq[0] + s_eq[1] + s_eq[2] + s_eq[3];
    }
}

__global__ void __launch_bounds__(kMRanges) k_ms_offsets(MBatch b, MWorkspace* ws) {
    __shared__ int64_t buf[kMRanges];
    const int t = blockIdx.x;
    const int i = threadIdx.x;
    const int64_t eq = ws->cnt_eq[t][i];
    buf[i] = eq;
    __syncthreads();
    for (int o = 1; o < kMRanges; o <<= 1) {
        const int64_t y = i >= o ? buf[i - o] : 0;
        __syncthreads();
        buf[i] += y;
        __syncthreads();
    }
    const int64_t eq_before = buf[i] - eq;
    const int64_t need = ws->st[t].kk;
    int64_t take = need - eq_before;
    take = take < 0 ? 0 : (take > eq ? eq : take);
    ws->take_eq[t][i] = take;
    const int64_t sel = ws->cnt_gt[t][i] + take;
    __syncthreads();
    buf[i] = sel;
    __syncthreads();
    for (int o = 1; o < kMRanges; o <<= 1) {
        const int64_t y = i >= o ? buf[i - o] : 0;
        __syncthreads();
        buf[i] += y;
        __syncthreads();
    }
    ws->sel_before[t][i] = buf[i] - sel;
}

// ARC: rows[out_off + slot] = i and slots[slot_off + i] = slot | -1 for every key.
// TopK: idx[out_off + slot] = i, vals[out_off + slot] = x[key_off + i].
template <bool FROM_FLOAT, bool ARC>
__global__ void __launch_bounds__(256) k_ms_write(MBatch b, const uint32_t* __restrict__ keys,
                                                  const float* __restrict__ x, MWorkspace* ws,
                                                  int32_t* __restrict__ out_idx,
                                                  float* __restrict__ out_val,
                                                  int32_t* __restrict__ out_slot) {
    __shared__ uint32_t s_sel[4], s_eq[4];
    const int t = blockIdx.y;
    const MItem it = b.it[t];
    const int64_t per = (it.n + kMRanges - 1) / kMRanges;
    const int64_t r0 = min<int64_t>(it.n, blockIdx.x * per), r1 = min<int64_t>(it.n, r0 + per);
    const uint32_t T = ws->st[t].prefix;
    const int64_t take_eq = ws->take_eq[t][blockIdx.x];
    int64_t slot = ws->sel_before[t][blockIdx.x];
    int64_t eq_seen = 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int64_t base = r0; base < r1; base += 256) {
        const int64_t i = base + threadIdx.x;
        const bool in = i < r1;
        uint32_t key = 0;
        float v = 0.f;
        if (in) {
            if constexpr (FROM_FLOAT) {
                v = x[it.key_off + i];
                key = __float_as_uint(v) & 0x7FFFFFFFu;
            } else {
                key = keys[it.key_off + i];
            }
        }
        const bool gt = in && key > T;
        const bool eq = in && key == T;
        const uint64_t beq = __ballot(eq);
        if (lane == 0) s_eq[wave] = __popcll(beq);
        __syncthreads();
        uint32_t eq_rank = __popcll(beq & lt);
        for (int w = 0; w < wave; ++w) eq_rank += s_eq[w];
        const uint32_t eq_tile = s_eq[0] + s_eq[1] + s_eq[2] + s_eq[3];
        const bool sel = gt || (eq && (eq_seen + eq_rank) < take_eq);
        const uint64_t bsel = __ballot(sel);
        if (lane == 0) s_sel[wave] = __popcll(bsel);
        __syncthreads();
        uint32_t sel_rank = __popcll(bsel & lt);
        for (int w = 0; w < wave; ++w) sel_rank += s_sel[w];
        const uint32_t sel_tile = s_sel[0] + s_sel[1] + s_sel[2] + s_sel[3];
        const int64_t my = slot + sel_rank;
        if (sel && my < it.k) {  // bound: never store past the item's k outputs
            out_idx[it.out_off + my] = (int32_t)i;
            if constexpr (!ARC) out_val[it.out_off + my] = v;
        }
        if constexpr (ARC) {
            if (in) out_slot[it.slot_off + i] = sel ? (int32_t)my : -1;
        }
        slot += sel_tile;
        eq_seen += eq_tile;
        __syncthreads();
    }
}

}  // namespace

int ms_select(const MBatch& b, int64_t maxn, const uint32_t* keys, const float* x, bool arc,
              MWorkspace* ws, int32_t* out_idx, float* out_val, int32_t* out_slot,
              hipStream_t st) {
    const int cnt = b.cnt;
    if (cnt < 1) return 0;
    const int hb = (int)std::max<int64_t>(1, std::min<int64_t>(kMHistBlocks, (maxn + 1023) / 1024));
    if (arc) {
        hipLaunchKernelGGL(k_ms_init<false>, dim3(cnt), dim3(256), 0, st, b, ws);
    } else {
        hipLaunchKernelGGL(k_ms_init<true>, dim3(cnt), dim3(256), 0, st, b, ws);
    }
    for (int pass = 0; pass < 4; ++pass) {
        if (arc)
            hipLaunchKernelGGL(k_ms_hist<false>, dim3(hb, cnt), dim3(256), 0, st, b, keys, x, ws);
        else
            hipLaunchKernelGGL(k_ms_hist<true>, dim3(hb, cnt), dim3(256), 0, st, b, keys, x, ws);
        hipLaunchKernelGGL(k_ms_digit, dim3(cnt), dim3(64), 0, st, b, ws);
    }
    if (arc) {
        hipLaunchKernelGGL(k_ms_count<false>, dim3(kMRanges, cnt), dim3(256), 0, st, b, keys, x, ws);
    } else {
        hipLaunchKernelGGL(k_ms_count<true>, dim3(kMRanges, cnt), dim3(256), 0, st, b, keys, x, ws);
    }
    hipLaunchKernelGGL(k_ms_offsets, dim3(cnt), dim3(kMRanges), 0, st, b, ws);
    if (arc)
        hipLaunchKernelGGL((k_ms_write<false, true>), dim3(kMRanges, cnt), dim3(256), 0, st, b, keys,
                           x, ws, out_idx, out_val, out_slot);
    else
        hipLaunchKernelGGL((k_ms_write<true, false>), dim3(kMRanges, cnt), dim3(256), 0, st, b, keys,
                           x, ws, out_idx, out_val, out_slot);
    return (int)hipGetLastError();
}

int ms_reset_orand(MWorkspace* ws, int cnt, hipStream_t st) {
    hipLaunchKernelGGL(k_ms_reset_orand, dim3(1), dim3(64), 0, st, ws, cnt);
    return (int)hipGetLastError();
}

}  // namespace arctopk
