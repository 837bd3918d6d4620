// Multi-block exact top-k selection (see mselect.h for the algorithm).
//
// Launches per batch: [init (TopK only; ARC's key producer initialises)] -> hist0 ->
// compact -> hist1 -> hist2 -> count -> write.  Each histogram pass picks its digit in
// the last block to finish (ms_arrive_last), the count pass computes the per-range
// offsets the same way: no separate tiny kernels between the passes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "mselect.h"
#include "mselect_dev.h"

namespace arctopk {
namespace {

constexpr int kW1 = 12;  // first-pass digit width (kMBins = 1 << kW1)
constexpr int kW2 = 10;  // refinement digit width (12 + 10 + 10 >= 32 key bits)
constexpr int kCandPerBlock = 2048;     // candidates per block of a refinement pass
#ifndef ARCTOPK_COMPACT_NT
#define ARCTOPK_COMPACT_NT 0            // TopK compact: nontemporal 16-B loads of |x| (A/B switch)
#endif
constexpr int kCompactRanges = 4;       // ranges per block of the TopK / RandK compact pass
constexpr int kSmallSelThreads = 1024;  // threads of the single-block small-item select
constexpr int kCompactStage = 4096;     // candidates a compact block stages in LDS (32 KiB)


// Flat grids of the per-range kernels: block x is range r of item t, items back to back
// (no idle blocks padding small items up to the largest item's range count).
__device__ __forceinline__ bool ms_locate(const MBatch& b, int* t, int* r) {
    int x = (int)blockIdx.x;
    for (int i = 0; i < b.cnt; ++i) {
        const int nr = b.it[i].nranges;
        if (x < nr) {
            *t = i;
            *r = x;
            return true;
        }
        x -= nr;
    }
    return false;
}


static int total_ranges(const MBatch& b) {
    int n = 0;
    for (int i = 0; i < b.cnt; ++i) n += b.it[i].nranges;
    return n;
}

// exclusive block scan of one uint32 per thread (NW waves); *total = block sum
template <int NW>
__device__ __forceinline__ uint32_t block_exscan_u32(uint32_t v, uint32_t* lds, uint32_t* total) {
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
        const uint32_t s = lds[w];
        before += w < wave ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return before + x - v;
}

// TopK start state: |x| keys, only the sign bit is known (RandK hash keys: nothing is)
template <int SRC>
__global__ void __launch_bounds__(256) k_ms_init(MBatch b, MWorkspace* ws) {
    const int t = blockIdx.x;
    ms_init_item(ws, t, b.it[t].k, SRC >= 3 ? 0xFFFFFFFFu : 0x7FFFFFFFu, 0u);
    if (threadIdx.x == 0) ws->done[t].v = 0;
}

// Histogram of the next min(W, bit) undecided bits of the keys matching the prefix:
// PASS 0 scans every key of the item; later passes scan the candidates when the item
// has them.  LDS histogram, merged with one global atomic per non-empty bin; the last
// block then reads (and clears) the global histogram and fixes the digit holding the
// kk-th largest key.  PASS 0 also fixes the candidate bin and mode.
// FOLD (TopK, fp32, PASS 0; the host checks every item is 16-B aligned with n % 4 == 0): x is the
// residual E and g the bucket G; the pass applies EF14 as it streams -- v = G + E (FOLD 1) or G
// (FOLD 2, the first call), E := v -- and histograms |v|, so the separate fold pass over G and E
// (arctopk_ef14_fold) is not needed; the later passes read the folded E
template <int SRC, int PASS, int FOLD = 0>
__global__ void __launch_bounds__(256) k_ms_hist(MBatch b, const uint32_t* __restrict__ keys,
                                                 const void* __restrict__ x, MWorkspace* ws,
                                                 const uint32_t* __restrict__ ckey,
                                                 const float* __restrict__ g = nullptr) {
    static_assert(FOLD == 0 || (SRC == 1 && PASS == 0), "the fold is fp32 TopK's first pass");
    // RandK hash keys are uniform over 32 bits, so every block finds every first-pass bin
    // occupied: their first digit is 8 bits (256 bins to merge per block, not 4,096; the k-th
    // key's bin then holds ~n/256 candidates) and the two refinements 12 bits each (8+12+12)
    constexpr int W = SRC >= 3 ? (PASS == 0 ? 8 : 12) : (PASS == 0 ? kW1 : kW2);
    constexpr int PER = (1 << W) >= 256 ? (1 << W) / 256 : 1;
    __shared__ uint32_t h[1 << W];
    __shared__ uint32_t lds[4];
    const int t = blockIdx.y;
    const MState s = ws->st[t];
    if (s.bit <= 0) return;  // every block: nothing left to decide
    const bool from_cand = PASS > 0 && s.cand;
    const int64_t ncand = from_cand ? (int64_t)ws->ncand[t].v : 0;
    const int64_t nblk = from_cand
        ? min<int64_t>(gridDim.x, max<int64_t>(1, (ncand + kCandPerBlock - 1) / kCandPerBlock))
        : (int64_t)gridDim.x;
    if (blockIdx.x >= nblk) return;  // uniform per block; not counted by the arrival
    const int w = s.bit < W ? s.bit : W;
    const int shift = s.bit - w;
    const uint32_t dmask = (1u << w) - 1u;
    for (int i = threadIdx.x; i < (1 << W); i += 256) h[i] = 0;
    __syncthreads();
    const MItem it = b.it[t];
    const int64_t stride = nblk * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t* src = from_cand ? ckey + it.cand_off : nullptr;
    int64_t n = from_cand ? ncand : it.n;
    if constexpr (PASS == 0 && SRC == 1) {
        // fp32 |x| over the whole item: 16-B nontemporal loads, four in flight per lane (4-B loads
        // left the pass at ~2.7 TB/s: 94 -> 73 us on the headline; plain 16-B loads measured
        // 110 us), then the < 4 tail elements below
        const float* xf = static_cast<const float*>(x) + it.key_off;
        if (FOLD || (reinterpret_cast<uintptr_t>(xf) & 15) == 0) {
            const int64_t n4 = it.n >> 2;
            int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
            auto add4 = [&](float4 v) {
                const uint32_t kq[4] = {__float_as_uint(v.x) & 0x7FFFFFFFu, __float_as_uint(v.y) & 0x7FFFFFFFu,
                                        __float_as_uint(v.z) & 0x7FFFFFFFu, __float_as_uint(v.w) & 0x7FFFFFFFu};
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if ((kq[c] & s.mask) == s.prefix) atomicAdd(&h[(kq[c] >> shift) & dmask], 1u);
            };
            if constexpr (FOLD != 0) {  // (n % 4 == 0: no tail)
                const float* gf = g + it.key_off;
                float* ef = const_cast<float*>(xf);
                auto fold4 = [&](float4 gv, float4 ev) {
                    if constexpr (FOLD == 1) {  // tensor.add_(E) (sparse_hook.py:205): fp32 adds, no contraction
                        gv.x = __fadd_rn(gv.x, ev.x);
                        gv.y = __fadd_rn(gv.y, ev.y);
                        gv.z = __fadd_rn(gv.z, ev.z);
                        gv.w = __fadd_rn(gv.w, ev.w);
                    }
                    return gv;
                };
                for (; q + 3 * stride < n4; q += 4 * stride) {
                    float4 gv[4], ev[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        gv[u] = ldq<float, true>(gf, q + u * stride);
                        if constexpr (FOLD == 1) ev[u] = ldq<float, true>(xf, q + u * stride);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const float4 v = fold4(gv[u], ev[u]);
                        stq<float, true>(ef, q + u * stride, v);
                        add4(v);
                    }
                }
                for (; q < n4; q += stride) {
                    const float4 gv = ldq<float, true>(gf, q);
                    const float4 ev = FOLD == 1 ? ldq<float, true>(xf, q) : gv;
                    const float4 v = fold4(gv, ev);
                    stq<float, true>(ef, q, v);
                    add4(v);
                }
                n = 0;  // nothing left for the scalar loops
            } else {
            for (; q + 3 * stride < n4; q += 4 * stride) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = ldq<float, true>(xf, q + u * stride);
#pragma unroll
                for (int u = 0; u < 4; ++u) add4(v[u]);
            }
            for (; q < n4; q += stride) add4(ldq<float, true>(xf, q));
            i = (n4 << 2) + (int64_t)blockIdx.x * 256 + threadIdx.x;  // the tail, element by element
            }
        }
    }
    for (; i + 3 * stride < n; i += 4 * stride) {  // four loads in flight per lane
        uint32_t k4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            k4[u] = from_cand ? src[i + u * stride] : item_key<SRC>(it, keys, x, i + u * stride);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if ((k4[u] & s.mask) == s.prefix) atomicAdd(&h[(k4[u] >> shift) & dmask], 1u);
    }
    for (; i < n; i += stride) {
        const uint32_t key = from_cand ? src[i] : item_key<SRC>(it, keys, x, i);
        if ((key & s.mask) == s.prefix) atomicAdd(&h[(key >> shift) & dmask], 1u);
    }
    __syncthreads();
    for (int j = threadIdx.x; j <= (int)dmask; j += 256)
        if (h[j]) atomicAdd(&ws->hist[t][hist_slot(j)], h[j]);
    if (!ms_arrive_last(&ws->done[t].v, (uint32_t)nblk)) return;

    // ---- last block: digit of the kk-th largest key (bins scanned from the top)
    const int nb = 1 << w;
    const int per = (nb + 255) / 256;
    ms_take_hist(ws, t, nb, h);  // h is free: the merge above read it before the arrival's barrier
    __syncthreads();
    uint32_t c[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int bin = nb - 1 - ((int)threadIdx.x * per + q);
        c[q] = (q < per && bin >= 0) ? h[bin] : 0u;
        sum += c[q];
    }
    uint32_t total;
    const uint32_t excl = block_exscan_u32<4>(sum, lds, &total);
    const uint64_t kk = (uint64_t)s.kk;
    if ((uint64_t)excl < kk && (uint64_t)excl + sum >= kk) {
        uint64_t acc = excl;
        int q = 0;
        for (; q < per - 1; ++q) {
            if (acc + c[q] >= kk) break;
            acc += c[q];
        }
        const uint32_t d = (uint32_t)(nb - 1 - ((int)threadIdx.x * per + q));
        MState& g = ws->st[t];
        const uint32_t prefix = s.prefix | (d << shift);
        const uint32_t mask = s.mask | ((uint32_t)(nb - 1) << shift);
        g.prefix = prefix;
        g.mask = mask;
        g.kk = s.kk - (int64_t)acc;
        g.bit = shift;
        if (PASS == 0) {
            g.p1 = prefix;
            g.m1 = mask;
            g.cand = (int64_t)c[q] <= it.cand_cap ? 1 : 0;
        }
    }
}

// kCompactRanges consecutive ranges of one item per block: per range, the count of keys above
// the first-pass bin; in candidate mode the bin's keys + local indices are staged in LDS and
// appended to the item's candidate list with ONE counter atomic per block (per full stage): the
// counter is one memory-side word per item, and appends to it serialise -- one per 4,096-key
// tile measured ~70 us on a 16 x 4 M-key batch.  Candidate order does not matter (the later
// passes histogram them and count them by their index's range).
template <int SRC>
__global__ void __launch_bounds__(256) k_ms_compact(MBatch b, const uint32_t* __restrict__ keys,
                                                    const void* __restrict__ x, MWorkspace* ws,
                                                    uint32_t* __restrict__ ckey,
                                                    uint32_t* __restrict__ cidx) {
    __shared__ uint32_t lds[4], s_cnt[4], s_base;
    __shared__ uint32_t s_ck[kCompactStage], s_ci[kCompactStage];
    const int t = blockIdx.y;
    const MItem it = b.it[t];
    const int ra = (int)blockIdx.x * kCompactRanges;
    if (ra >= it.nranges) return;  // uniform per block
    const int rb = min(it.nranges, ra + kCompactRanges);
    const MState s = ws->st[t];
    const uint32_t hi = s.p1 | ~s.m1;  // largest key of the bin
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t staged = 0;  // candidates in the LDS stage (uniform)
    // fp32 |x| keys of a 16-B aligned item of 4k elements: each lane loads 4 quads of a tile (16-B
    // loads); key j of the lane is element 4 (64 (j / 4) + lane) + j % 4 of its wave's quarter
    bool vec = false;
    if constexpr (SRC == 1)
        vec = (it.n & 3) == 0 &&
              (reinterpret_cast<uintptr_t>(static_cast<const float*>(x) + it.key_off) & 15) == 0;
    auto el = [&](int64_t wb, int j) -> int64_t {
        return vec ? wb + 4 * ((j >> 2) * 64 + lane) + (j & 3) : wb + j * 64 + lane;
    };
    auto flush = [&]() {  // uniform; the stage -> the item's list, one counter atomic
        if (threadIdx.x == 0) s_base = atomicAdd(&ws->ncand[t].v, staged);
        __syncthreads();
        const uint32_t base = s_base;
        for (uint32_t q = threadIdx.x; q < staged; q += 256) {
            ckey[it.cand_off + base + q] = s_ck[q];
            cidx[it.cand_off + base + q] = s_ci[q];
        }
        __syncthreads();  // the stage is rewritten next
        staged = 0;
    };
    for (int r = ra; r < rb; ++r) {
        const int64_t r0 = (int64_t)r * it.range;
        const int64_t r1 = min<int64_t>(it.n, r0 + it.range);
        uint32_t gt = 0;
        for (int64_t tile = r0; tile < r1; tile += kMTile) {
            const int64_t wb = tile + (int64_t)wave * (kMTile / 4);
            uint32_t kv[kPerLane];
            bool loaded = false;
            if constexpr (SRC == 1) {
                if (vec) {
                    const float* xf = static_cast<const float*>(x) + it.key_off;
#pragma unroll
                    for (int u = 0; u < kPerLane / 4; ++u) {
                        const int64_t q = min<int64_t>((wb >> 2) + u * 64 + lane, ((r1 - 1) >> 2));
                        const float4 v = ldq<float, ARCTOPK_COMPACT_NT != 0>(xf, q);
                        kv[4 * u + 0] = __float_as_uint(v.x) & 0x7FFFFFFFu;
                        kv[4 * u + 1] = __float_as_uint(v.y) & 0x7FFFFFFFu;
                        kv[4 * u + 2] = __float_as_uint(v.z) & 0x7FFFFFFFu;
                        kv[4 * u + 3] = __float_as_uint(v.w) & 0x7FFFFFFFu;
                    }
                    loaded = true;
                }
            }
            if (!loaded) {
#pragma unroll
                for (int j = 0; j < kPerLane; ++j)
                    kv[j] = item_key<SRC>(it, keys, x, min<int64_t>(wb + j * 64 + lane, r1 - 1));
            }
            uint32_t nin = 0;
#pragma unroll
            for (int j = 0; j < kPerLane; ++j) {
                const bool valid = el(wb, j) < r1;
                gt += (valid && kv[j] > hi) ? 1u : 0u;
                if (s.cand) nin += popc64(__ballot(valid && (kv[j] & s.m1) == s.p1));
            }
            if (s.cand) {  // uniform
                if (lane == 0) s_cnt[wave] = nin;
                __syncthreads();
                const uint32_t tot = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
                uint32_t before = 0;
#pragma unroll
                for (int w = 0; w < 4; ++w) before += w < wave ? s_cnt[w] : 0u;
                __syncthreads();  // s_cnt is rewritten by the next tile
                if (staged + tot > (uint32_t)kCompactStage) flush();
                uint32_t pos = staged + before;
#pragma unroll
                for (int j = 0; j < kPerLane; ++j) {
                    const int64_t i = el(wb, j);
                    const bool in = i < r1 && (kv[j] & s.m1) == s.p1;
                    const uint64_t bm = __ballot(in);
                    if (in) {
                        const uint32_t q = pos + popc64(bm & lt);
                        s_ck[q] = kv[j];
                        s_ci[q] = (uint32_t)i;
                    }
                    pos += popc64(bm);
                }
                staged += tot;
                __syncthreads();  // the stage is complete before a flush reads it
            }
        }
        uint32_t total;
        (void)block_exscan_u32<4>(gt, lds, &total);
        if (threadIdx.x == 0) {
            ws->cnt_gt[t][r] = total;
            ws->cnt_eq[t][r] = 0u;
        }
    }
    if (s.cand && staged) flush();
}

// ARC: one block per range (arc_compact_range, mselect_dev.h)
__global__ void __launch_bounds__(256) k_arc_compact(const MBatch* __restrict__ bp, const RangeGrid g,
                                                     const uint32_t* __restrict__ keys, MWorkspace* ws,
                                                     uint32_t* __restrict__ ckey) {
    int t, r;
    if (!ms_locate(g, &t, &r)) return;
    arc_compact_range(bp->it[t], t, r, keys, ws, ckey);
}

// Per-range counts of the bin's keys > T and == T (T = the final prefix), added to the
// compact pass's counts: from the candidates or, in full mode, by rescanning each
// range.  The last block then turns them into per-range T-equal allowances (lowest
// ranges first) and output offsets.
template <int SRC>
__global__ void __launch_bounds__(256) k_ms_count(MBatch b, const uint32_t* __restrict__ keys,
                                                  const void* __restrict__ x, MWorkspace* ws,
                                                  const uint32_t* __restrict__ ckey,
                                                  const uint32_t* __restrict__ cidx) {
    __shared__ uint32_t lds[4];
    const int t = blockIdx.y;
    const MItem it = b.it[t];
    const MState s = ws->st[t];
    const uint32_t T = s.prefix;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (s.cand) {
        const int64_t n = ws->ncand[t].v;
        for (int64_t c0 = (int64_t)blockIdx.x * 256 + wave * 64; c0 < n; c0 += (int64_t)gridDim.x * 256) {
            const int64_t c = c0 + lane;
            const bool valid = c < n;
            const uint32_t key = valid ? ckey[it.cand_off + c] : 0u;
            const int r = valid ? (int)(cidx[it.cand_off + c] / (uint32_t)it.range) : -1;
            const bool gt = valid && key > T;
            const bool eq = valid && key == T;
            // segmented wave reduction: one atomic pair per distinct range in the wave
            // (candidates are appended block tile by block tile: usually one or two)
            uint64_t pending = __ballot(gt || eq);
            while (pending) {
                const int leader = __ffsll((long long)pending) - 1;
                const int rl = __shfl(r, leader, 64);
                const bool mine = valid && r == rl;
                const uint32_t ng = popc64(__ballot(mine && gt)), ne = popc64(__ballot(mine && eq));
                if (lane == leader) {
                    if (ng) atomicAdd(&ws->cnt_gt[t][rl], ng);
                    if (ne) atomicAdd(&ws->cnt_eq[t][rl], ne);
                }
                pending &= ~__ballot(mine);
            }
        }
    } else {
        for (int r = blockIdx.x; r < it.nranges; r += gridDim.x) {
            const int64_t r0 = (int64_t)r * it.range;
            const int64_t r1 = min<int64_t>(it.n, r0 + it.range);
            uint32_t gt = 0, eq = 0;
            for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) {
                const uint32_t key = item_key<SRC>(it, keys, x, i);
                const bool in = (key & s.m1) == s.p1;
                gt += (in && key > T) ? 1u : 0u;
                eq += key == T ? 1u : 0u;
            }
            uint32_t tg, te;
            (void)block_exscan_u32<4>(gt, lds, &tg);
            (void)block_exscan_u32<4>(eq, lds, &te);
            if (threadIdx.x == 0) {
                if (tg) atomicAdd(&ws->cnt_gt[t][r], tg);
                if (te) atomicAdd(&ws->cnt_eq[t][r], te);
            }
        }
    }
    if (!ms_arrive_last(&ws->done[t].v, gridDim.x)) return;

    // ---- last block: offsets over the item's ranges (4 consecutive ranges per thread)
    const int nr = it.nranges;
    // read-and-clear in range order (contiguous lines per wave instruction), then regroup
    __shared__ uint32_t s_eq[kMMaxRanges], s_gt[kMMaxRanges];
    for (int r = threadIdx.x; r < nr; r += 256) {
        s_eq[r] = ms_take(&ws->cnt_eq[t][r]);
        s_gt[r] = ms_take(&ws->cnt_gt[t][r]);
    }
    __syncthreads();
    uint32_t eq[4], gt[4], se = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = threadIdx.x * 4 + q;
        eq[q] = r < nr ? s_eq[r] : 0u;
        gt[q] = r < nr ? s_gt[r] : 0u;
        se += eq[q];
    }
    uint32_t tot;
    uint32_t eq_before = block_exscan_u32<4>(se, lds, &tot);
    const int64_t need = s.kk;
    uint32_t take[4], ss = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int64_t tk = need - (int64_t)eq_before;
        tk = tk < 0 ? 0 : (tk > eq[q] ? eq[q] : tk);
        take[q] = (uint32_t)tk;
        eq_before += eq[q];
        ss += gt[q] + take[q];
    }
    uint32_t sel_before = block_exscan_u32<4>(ss, lds, &tot);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = threadIdx.x * 4 + q;
        if (r < nr) {
            ws->take_eq[t][r] = take[q];
            ws->sel_before[t][r] = sel_before;
        }
        sel_before += gt[q] + take[q];
    }
}

// One block per range, 4096-key tiles (each wave a contiguous 1024 keys, 16 per lane):
// ballot compaction in index order.  ARC: rows[out_off + slot] = i and the slot map for
// every key; TopK: idx[out_off + slot] = i, vals[out_off + slot] = x[key_off + i].

template <int SRC, bool ARC, int FOLD = 0>
__global__ void __launch_bounds__(256) k_ms_write(MBatch b, const uint32_t* __restrict__ keys,
                                                  const void* __restrict__ x, MWorkspace* ws,
                                                  int32_t* __restrict__ out_idx,
                                                  void* __restrict__ out_val,
                                                  int32_t* __restrict__ out_slot, void* zero_x) {
    int t, r;
    if (!ms_locate(b, &t, &r)) return;
    ms_write_body<SRC, ARC, FOLD>(b, t, r, keys, x, ws, out_idx, out_val, out_slot, zero_x);
}

// ARC: the batch from device memory (plan-resident)
__global__ void __launch_bounds__(256) k_arc_write(const MBatch* __restrict__ bp, const RangeGrid g,
                                                   const uint32_t* __restrict__ keys, MWorkspace* ws,
                                                   int32_t* __restrict__ out_idx, int32_t* __restrict__ out_slot) {
    int t, r;
    if (!ms_locate(g, &t, &r)) return;
    ms_write_body<0, true>(*bp, t, r, keys, nullptr, ws, out_idx, nullptr, out_slot, nullptr);
}

// Single-block select of one small item per block (TopK / RandK tensors of at most kSmallSel keys:
// BatchNorm vectors, biases, small convs): its keys in LDS, four 8-bit radix rounds over them, then
// the ordered write in chunks of the block (ascending indices; ties at the threshold lowest index
// first, as the multi-block select), so a bucket of many small tensors costs one launch per 48 of
// them instead of seven.  FOLD as in k_ms_hist (TopK: E := G + E written while the keys are
// formed; the write pass then reads the folded E) and ms_write_body (RandK: v = G + E formed in
// the write pass, E := v with the selected elements zeroed).
template <int SRC, int FOLD>
__global__ void __launch_bounds__(kSmallSelThreads) k_ms_small(MBatch b, const void* __restrict__ x,
                                                               const void* __restrict__ g, int32_t* __restrict__ out_idx,
                                                               void* __restrict__ out_val, void* zero_x) {
    constexpr int NT = kSmallSelThreads, NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) uint32_t skeys[];
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_w[2][NW];
    __shared__ uint32_t s_digit, s_acc;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const MItem it = b.it[blockIdx.x];
    const int n = (int)it.n;
    for (int i = tid; i < n; i += NT) {
        uint32_t key;
        if constexpr (SRC >= 3) {
            key = rk_key(it.hseed, i);
        } else if constexpr (FOLD != 0) {  // fp32 TopK: E := G (+ E), keyed by |E|
            float v = static_cast<const float*>(g)[it.key_off + i];
            if constexpr (FOLD == 1) v = __fadd_rn(v, static_cast<const float*>(x)[it.key_off + i]);
            static_cast<float*>(const_cast<void*>(x))[it.key_off + i] = v;
            key = __float_as_uint(v) & 0x7FFFFFFFu;
        } else {
            key = item_key<SRC>(it, nullptr, x, i);
        }
        skeys[i] = key;
    }
    __syncthreads();
    uint32_t prefix = 0u, mask = 0u;
    int64_t kk = it.k;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int j = tid; j < 256; j += NT) hist[j] = 0u;
        __syncthreads();
        for (int i = tid; i < n; i += NT) {
            const uint32_t k = skeys[i];
            if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid < 64) {  // lane l: bins 255 - 4l .. 252 - 4l, scanned from the top
            uint32_t c[4], tot = 0u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c[q] = hist[255 - (4 * lane + q)];
                tot += c[q];
            }
            uint32_t incl = tot;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            const uint64_t excl = incl - tot;
            if (excl < (uint64_t)kk && excl + tot >= (uint64_t)kk) {
                uint64_t acc = excl;
                int q = 0;
                for (; q < 3; ++q) {
                    if (acc + c[q] >= (uint64_t)kk) break;
                    acc += c[q];
                }
                s_digit = (uint32_t)(255 - (4 * lane + q));
                s_acc = (uint32_t)acc;
            }
        }
        __syncthreads();
        prefix |= s_digit << shift;
        mask |= 255u << shift;
        kk -= (int64_t)s_acc;
        __syncthreads();  // s_digit / s_acc / hist are rewritten by the next round
    }
    const uint32_t T = prefix;
    const uint32_t take_eq = (uint32_t)kk;  // threshold-equal keys to take, lowest index first
    uint32_t run = 0u, eq_run = 0u;
    for (int c0 = 0; c0 < n; c0 += NT) {
        const int i = c0 + tid;
        const bool valid = i < n;
        const uint32_t key = valid ? skeys[i] : 0u;
        const bool gt = valid && key > T, eq = valid && key == T;
        const uint64_t beq = __ballot(eq);
        if (lane == 0) s_w[0][wave] = popc64(beq);
        __syncthreads();
        uint32_t eq_before = popc64(beq & lt), eq_tot = 0u;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            eq_before += w < wave ? s_w[0][w] : 0u;
            eq_tot += s_w[0][w];
        }
        const bool sel = gt || (eq && eq_run + eq_before < take_eq);
        const uint64_t bsel = __ballot(sel);
        if (lane == 0) s_w[1][wave] = popc64(bsel);
        __syncthreads();
        uint32_t sel_before = popc64(bsel & lt), sel_tot = 0u;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            sel_before += w < wave ? s_w[1][w] : 0u;
            sel_tot += s_w[1][w];
        }
        if (valid) {
            uint32_t bits = 0u;
            if constexpr (SRC >= 3 && FOLD != 0) bits = fold_bits<SRC>(g, zero_x, it.key_off + i, FOLD);
            else if (x && (sel || (SRC >= 3 && zero_x))) bits = load_bits<SRC>(nullptr, x, it.key_off + i);
            const uint32_t pos = run + sel_before;
            if (sel && pos < (uint32_t)it.k) {
                out_idx[it.out_off + pos] = i;
                if (out_val) store_val<SRC>(out_val, it.out_off + pos, bits);
            }
            if (zero_x && (sel || (SRC >= 3 && FOLD != 0))) {  // E[idx] = 0 (:104); RandK fold: E := v elsewhere
                if constexpr (SRC == 1 || SRC == 3) static_cast<float*>(zero_x)[it.key_off + i] = sel ? 0.f : __uint_as_float(bits);
                else static_cast<uint16_t*>(zero_x)[it.key_off + i] = sel ? (uint16_t)0 : (uint16_t)(bits >> 16);
            }
        }
        run += sel_tot;
        eq_run += eq_tot;
        __syncthreads();  // s_w is rewritten by the next chunk
    }
}

}  // namespace

void ms_item_geometry(MItem& it, int max_ranges) {
    const int64_t tiles = (it.n + kMTile - 1) / kMTile;
    max_ranges = std::max(1, std::min(max_ranges, kMMaxRanges));
    const int64_t per = std::max<int64_t>(1, (tiles + max_ranges - 1) / max_ranges);
    it.range = (int32_t)(per * kMTile);
    it.nranges = (int32_t)((it.n + it.range - 1) / it.range);
    // candidates: the k-th key's 12-bit bin; a few % of n on gradient-like data, all of
    // n on degenerate data (e.g. a zero tensor) -> full mode past the cap
    it.cand_cap = it.n <= 65536 ? it.n : std::max<int64_t>(65536, it.n / 8);
    it.hseed = 0;
}

int ms_select_small(const MBatch& b, const void* x, int x_bf16, int32_t* out_idx, void* out_val, void* zero_x,
                    hipStream_t st, bool hashed, int fold, const void* fold_g) {
    if (b.cnt < 1) return 0;
    int64_t maxn = 0;
    for (int i = 0; i < b.cnt; ++i) maxn = std::max(maxn, b.it[i].n);
    if (maxn > kMSmallSel || (fold && (!x || !zero_x || !fold_g || (!hashed && x_bf16)))) return 1001;
    const size_t lds = (size_t)maxn * 4;
    const dim3 grid(b.cnt), block(kSmallSelThreads);
#define MS_SMALL(FF, FO) hipLaunchKernelGGL((k_ms_small<FF, FO>), grid, block, lds, st, b, x, fold_g, out_idx, out_val, zero_x)
    if (hashed) {
        if (fold == 1) { if (x_bf16) MS_SMALL(4, 1); else MS_SMALL(3, 1); }
        else if (fold == 2) { if (x_bf16) MS_SMALL(4, 2); else MS_SMALL(3, 2); }
        else if (x_bf16) MS_SMALL(4, 0);
        else MS_SMALL(3, 0);
    } else {
        if (fold == 1) MS_SMALL(1, 1);
        else if (fold == 2) MS_SMALL(1, 2);
        else if (x_bf16) MS_SMALL(2, 0);
        else MS_SMALL(1, 0);
    }
#undef MS_SMALL
    return (int)hipGetLastError();
}

RangeGrid ms_range_grid(const MBatch& b) {
    RangeGrid g{};
    g.cnt = b.cnt;
    g.first[0] = 0;
    for (int i = 0; i < b.cnt; ++i) g.first[i + 1] = g.first[i] + b.it[i].nranges;
    return g;
}

int64_t ms_workspace_bytes(int64_t cap_total) {
    return (int64_t)sizeof(MWorkspace) + 8 * cap_total;
}

int ms_select(const MBatch& b, int64_t maxn, const uint32_t* keys, const void* x, int x_bf16, bool arc,
              MWorkspace* ws, int64_t cap_total, int32_t* out_idx, void* out_val,
              int32_t* out_slot, void* zero_x, hipStream_t st, bool hashed, int fold, const void* fold_g) {
    if (fold && (!x || !zero_x || arc || (!hashed && (!fold_g || x_bf16)))) return 1001;  // ARCTOPK_EINVAL
    const int cnt = b.cnt;
    if (cnt < 1) return 0;
    int gr = 1;
    for (int i = 0; i < cnt; ++i) {
        const MItem& it = b.it[i];
        if (it.nranges < 1 || it.nranges > kMMaxRanges || it.cand_off < 0 ||
            it.cand_off + it.cand_cap > cap_total || (int64_t)it.range * it.nranges < it.n)
            return 1001;  // ARCTOPK_EINVAL: geometry not from ms_item_geometry
        gr = std::max(gr, it.nranges);
    }
    uint32_t* ckey = reinterpret_cast<uint32_t*>(ws + 1);
    uint32_t* cidx = ckey + cap_total;
    // histogram blocks per item: every block merges its LDS histogram with memory-side
    // atomics on the same hot words, so the batch's total is capped (tuning switch)
    constexpr int64_t hist_total = ARCTOPK_TOPK_HIST_BLOCKS;  // headline TopK: 387 -> 404 GB/s (512: 399, 2048: 387)
    const int hb = (int)std::max<int64_t>(
        1, std::min<int64_t>(std::min<int64_t>(kMHistBlocks, (maxn + 8191) / 8192), hist_total / cnt));
    // the count pass: each block arrives once on the item's one done counter (those arrivals
    // serialise at the memory side), so a few blocks per item stride over its ranges / candidates
    const dim3 gh(hb, cnt), gt(std::min(gr, 32), cnt), gflat(total_ranges(b)),
        gc((gr + kCompactRanges - 1) / kCompactRanges, cnt);
#define MS_LAUNCH(FF, AR)                                                                              \
    do {                                                                                               \
        if (!AR) hipLaunchKernelGGL(k_ms_init<FF>, dim3(cnt), dim3(256), 0, st, b, ws);                \
        hipLaunchKernelGGL((k_ms_hist<FF, 0>), gh, dim3(256), 0, st, b, keys, x, ws, ckey, nullptr);   \
        hipLaunchKernelGGL(k_ms_compact<FF>, gc, dim3(256), 0, st, b, keys, x, ws, ckey, cidx);        \
        hipLaunchKernelGGL((k_ms_hist<FF, 1>), gh, dim3(256), 0, st, b, keys, x, ws, ckey, nullptr);   \
        hipLaunchKernelGGL((k_ms_hist<FF, 2>), gh, dim3(256), 0, st, b, keys, x, ws, ckey, nullptr);   \
        hipLaunchKernelGGL(k_ms_count<FF>, gt, dim3(256), 0, st, b, keys, x, ws, ckey, cidx);          \
        hipLaunchKernelGGL((k_ms_write<FF, AR>), gflat, dim3(256), 0, st, b, keys, x, ws, out_idx,     \
                           out_val, out_slot, zero_x);                                                 \
    } while (0)
    // the RandK select with the EF14 fold in its write pass: the passes before it never read x
#define MS_LAUNCH_FOLD(FF, FO)                                                                         \
    do {                                                                                               \
        hipLaunchKernelGGL(k_ms_init<FF>, dim3(cnt), dim3(256), 0, st, b, ws);                         \
        hipLaunchKernelGGL((k_ms_hist<FF, 0>), gh, dim3(256), 0, st, b, keys, nullptr, ws, ckey, nullptr);\
        hipLaunchKernelGGL(k_ms_compact<FF>, gc, dim3(256), 0, st, b, keys, nullptr, ws, ckey, cidx);  \
        hipLaunchKernelGGL((k_ms_hist<FF, 1>), gh, dim3(256), 0, st, b, keys, nullptr, ws, ckey, nullptr);\
        hipLaunchKernelGGL((k_ms_hist<FF, 2>), gh, dim3(256), 0, st, b, keys, nullptr, ws, ckey, nullptr);\
        hipLaunchKernelGGL(k_ms_count<FF>, gt, dim3(256), 0, st, b, keys, nullptr, ws, ckey, cidx);    \
        hipLaunchKernelGGL((k_ms_write<FF, false, FO>), gflat, dim3(256), 0, st, b, keys, x, ws,       \
                           out_idx, out_val, out_slot, zero_x);                                        \
    } while (0)
    // TopK (fp32) with the EF14 fold in its first histogram pass: x is the residual E
#define MS_LAUNCH_TOPK_FOLD(FO)                                                                        \
    do {                                                                                               \
        hipLaunchKernelGGL(k_ms_init<1>, dim3(cnt), dim3(256), 0, st, b, ws);                          \
        hipLaunchKernelGGL((k_ms_hist<1, 0, FO>), gh, dim3(256), 0, st, b, keys, x, ws, ckey,          \
                           static_cast<const float*>(fold_g));                                         \
        hipLaunchKernelGGL(k_ms_compact<1>, gc, dim3(256), 0, st, b, keys, x, ws, ckey, cidx);         \
        hipLaunchKernelGGL((k_ms_hist<1, 1>), gh, dim3(256), 0, st, b, keys, x, ws, ckey, nullptr);   \
        hipLaunchKernelGGL((k_ms_hist<1, 2>), gh, dim3(256), 0, st, b, keys, x, ws, ckey, nullptr);   \
        hipLaunchKernelGGL(k_ms_count<1>, gt, dim3(256), 0, st, b, keys, x, ws, ckey, cidx);           \
        hipLaunchKernelGGL((k_ms_write<1, false>), gflat, dim3(256), 0, st, b, keys, x, ws, out_idx,   \
                           out_val, out_slot, zero_x);                                                 \
    } while (0)
    if (fold && !hashed) {
        if (fold == 1) MS_LAUNCH_TOPK_FOLD(1);
        else MS_LAUNCH_TOPK_FOLD(2);
        return (int)hipGetLastError();
    }
#undef MS_LAUNCH_TOPK_FOLD
    if (fold) {
        if (x_bf16 && fold == 1) MS_LAUNCH_FOLD(4, 1);
        else if (x_bf16) MS_LAUNCH_FOLD(4, 2);
        else if (fold == 1) MS_LAUNCH_FOLD(3, 1);
        else MS_LAUNCH_FOLD(3, 2);
        return (int)hipGetLastError();
    }
#undef MS_LAUNCH_FOLD
    if (arc)
        MS_LAUNCH(0, true);
    else if (hashed && x_bf16)
        MS_LAUNCH(4, false);
    else if (hashed)
        MS_LAUNCH(3, false);
    else if (x_bf16)
        MS_LAUNCH(2, false);
    else
        MS_LAUNCH(1, false);
#undef MS_LAUNCH
    return (int)hipGetLastError();
}

static int arc_batch_check(const MBatch& b, int64_t cap_total, int* gr) {
    *gr = 1;
    for (int i = 0; i < b.cnt; ++i) {
        const MItem& it = b.it[i];
        if (it.nranges < 1 || it.nranges > kMMaxRanges || it.cand_off < 0 || it.cand_cap < it.n ||
            it.cand_off + it.cand_cap > cap_total || (int64_t)it.range * it.nranges < it.n)
            return 1001;  // ARCTOPK_EINVAL: ARC items need cand_cap >= n
        *gr = std::max(*gr, it.nranges);
    }
    return 0;
}

int ms_arc_compact(const MBatch& b, const MBatch* d_b, const uint32_t* keys, MWorkspace* ws, int64_t cap_total,
                   hipStream_t st) {
    if (b.cnt < 1) return 0;
    int gr;
    if (int e = arc_batch_check(b, cap_total, &gr)) return e;
    uint32_t* ckey = reinterpret_cast<uint32_t*>(ws + 1);
    hipLaunchKernelGGL(k_arc_compact, dim3(total_ranges(b)), dim3(256), 0, st, d_b, ms_range_grid(b), keys, ws,
                       ckey);
    return (int)hipGetLastError();
}

int ms_arc_write(const MBatch& b, const MBatch* d_b, const uint32_t* keys, MWorkspace* ws, int64_t cap_total,
                 int32_t* out_idx, int32_t* out_slot, hipStream_t st) {
    if (b.cnt < 1) return 0;
    int gr;
    if (int e = arc_batch_check(b, cap_total, &gr)) return e;
    hipLaunchKernelGGL(k_arc_write, dim3(total_ranges(b)), dim3(256), 0, st, d_b, ms_range_grid(b), keys, ws,
                       out_idx, out_slot);
    return (int)hipGetLastError();
}

}  // namespace arctopk
