// Multi-block exact top-k selection over uint32 keys, shared by the ARC-TopK large-
// segment select (keys = row-energy bits) and the TopK baseline (keys = |x| bits).
//
// Per item (a tensor / segment) of one batch, three passes over the full key array:
//   hist1   : 12-bit histogram of the leading undecided bits (ARC: below the keys'
//             common prefix, from a block OR/AND fused into the key pass; TopK: below
//             the sign bit) -> digit1 picks the bin B holding the k-th largest key
//   compact : per fixed key range, the count of keys above B; keys inside B are
//             appended to a candidate list (when B holds <= cand_cap keys; otherwise the
//             item stays in "full" mode and later passes rescan the whole key array)
//   refine  : <= 2 more histogram/digit rounds (10 bits each) over the candidates give
//             the exact threshold T and how many T-equal keys to take; per-range counts
//             of candidates > T and == T
//   offsets : scan over ranges: T-equal allowance (lowest ranges first), output offset
//   write   : per range, wave-contiguous 1024-key tiles, ballot compaction in index
//             order: ascending outputs, ties at T lowest index first
// Every launch covers all items of the batch (blockIdx.y = item).
#pragma once
#include "common.h"

namespace arctopk {

constexpr int kMB = 48;            // items per batch (kernel argument size)
constexpr int kMHistBlocks = 512;  // max blocks of a histogram pass per item
constexpr int kMMaxRanges = 1024;  // ranges per item
constexpr int kMTile = 4096;       // keys per block tile (4 waves x 16 x 64)
constexpr int kMBins = 4096;       // first-pass histogram bins (12 bits)

struct MItem {
    int64_t key_off;   // keys / x offset of the item
    int64_t n;         // keys
    int64_t k;         // keys to select
    int64_t out_off;   // output offset (TopK: idx/vals; ARC: row list)
    int64_t slot_off;  // ARC: slot map offset (per key)
    int64_t cand_off;  // candidate-list offset in the workspace
    int64_t cand_cap;  // candidate-list capacity
    int32_t range;     // keys per range (multiple of kMTile)
    int32_t nranges;   // ceil(n / range) <= kMMaxRanges
    uint32_t hseed;    // RandK (hash keys): the tensor's key seed (rk_key)
};

struct MBatch {
    MItem it[kMB];
    int32_t cnt;
};

// Where each item's ranges start in a flat per-range grid (block x = range r of item t),
// passed by value: a block finds its item from kernel arguments instead of walking the
// plan-resident batch's items one dependent load at a time
struct RangeGrid {
    int32_t cnt;             // items
    int32_t first[kMB + 1];  // first block of each item; first[cnt] = blocks
};

struct MState {
    uint32_t prefix, mask;  // decided leading bits
    int32_t bit;            // bits [bit-1 .. 0] still undecided
    int32_t cand;           // 1: candidates were compacted, later passes read only them
    int64_t kk;             // keys still to take among those matching the prefix
    uint32_t p1, m1;        // the first-pass bin (its keys are the candidates)
    uint32_t ncand;         // candidates appended (copied from the padded counter)
    uint32_t pad[7];        // 64 B
};

// Device-scope atomics run at the memory side and serialise per line: every
// contended word gets a 128-B line of its own, and global histogram bins are
// interleaved so neighbouring (equally hot) bins land on different lines.
struct alignas(128) MCounter {
    uint32_t v;
    uint32_t pad[31];
};
__host__ __device__ constexpr int hist_slot(int bin) { return ((bin & 127) << 5) | (bin >> 7); }


struct MWorkspace {
    uint32_t hist[kMB][kMBins];  // indexed by hist_slot(bin)
    MState st[kMB];
    MCounter ncand[kMB];
    MCounter done[kMB];          // blocks of the running kernel that finished, per item
    uint32_t part_or[kMB][kMHistBlocks];   // ARC key pass: per-block OR / AND partials
    uint32_t part_and[kMB][kMHistBlocks];
    uint32_t cnt_gt[kMB][kMMaxRanges];
    uint32_t cnt_eq[kMB][kMMaxRanges];
    uint32_t take_eq[kMB][kMMaxRanges];
    uint32_t sel_before[kMB][kMMaxRanges];
    uint32_t cnt_cand[kMB][kMMaxRanges];   // ARC: candidates of each range (k_arc_compact)
    uint32_t cand_or[kMB][kMMaxRanges];    // ARC: OR / AND of each range's candidates (the bits
    uint32_t cand_and[kMB][kMMaxRanges];   // all candidates share are decided without a round)
    // followed by the candidate lists: uint32 key[cap_total], uint32 index[cap_total]
};

// ---- device helpers shared with the producer of ARC keys (arctopk_kernels.hip) ----

// True in exactly one block per counter: the last of `expected` blocks to arrive.  The
// hand-over follows MI355X_MICROARCH.md's measured counter form: the payload is written
// ONLY with device-scope atomics (performed at the memory side), every wave waits for
// its own (vmcnt(0)) before a workgroup barrier, one lane then adds to the counter, the
// block whose add returns expected-1 is last, and it reads the payload back ONLY with
// device-scope atomics (ms_take) -- so no L2 line is trusted and no release fence (a
// full L2 write-back per block) is needed.  The last block resets the counter.
__device__ inline bool ms_arrive_last(uint32_t* counter, uint32_t expected) {
    __shared__ uint32_t s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = prev + 1u == expected;
        if (last) (void)__hip_atomic_exchange(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last ? 1u : 0u;
    }
    __syncthreads();
    return s_last != 0u;
}

__device__ inline uint32_t ms_take(uint32_t* p) {  // read-and-clear at the memory side
    return __hip_atomic_exchange(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Read-and-clear bins [0, nb) of item t's global histogram into lds_h[bin] (nb a power of
// two <= kMBins; all threads of the block; the caller syncs before reading lds_h).  The
// atomics walk the histogram in slot order, so a wave instruction covers whole 128-B lines
// (bin order puts every lane on a line of its own: memory-side atomics then run ~17x
// slower, which made this read-back the longest step of the last block).
__device__ inline void ms_take_hist(MWorkspace* ws, int t, int nb, uint32_t* lds_h) {
    const int g = nb >= 128 ? nb >> 7 : 1;  // bins per 128-B line
    for (int j = threadIdx.x; j < nb; j += blockDim.x) {
        const int line = j / g, q = j - line * g;
        const int bin = nb >= 128 ? q * 128 + line : j;
        lds_h[bin] = ms_take(&ws->hist[t][(line << 5) | q]);
    }
}

// Start state of item t (all threads of one block): histogram cleared, the keys' common
// leading bits decided (kor / kand = OR / AND of all keys; TopK: |x| keys, kor = ~0).
__device__ inline void ms_init_item(MWorkspace* ws, int t, int64_t k, uint32_t kor, uint32_t kand) {
    for (int i = threadIdx.x; i < kMBins; i += blockDim.x) ws->hist[t][i] = 0;
    if (threadIdx.x == 0) {
        MState& s = ws->st[t];
        const uint32_t diff = kor ^ kand;
        const int bit = diff ? 32 - __clz(diff) : 0;
        const uint32_t low = bit == 32 ? 0xFFFFFFFFu : ((1u << bit) - 1u);
        s.prefix = kand & ~low;
        s.mask = ~low;
        s.bit = bit;
        s.kk = k;
        s.cand = 0;
        s.ncand = 0;
        s.p1 = s.prefix;
        s.m1 = s.mask;
        ws->ncand[t].v = 0;
    }
}

// ARC first pass: every block of the fused key kernel merges its LDS histogram of the keys'
// top 12 value bits (bits 30..19: energies are non-negative and NaN maps to 0x7FFFFFFF, so
// bit 31 is always clear) into ws->hist[t]; the blocks of the next launches find the bin
// holding the k-th largest key there (ms_arc_digit_local) and start the item in candidate
// mode on that bin (cand_cap = n for ARC items: every key of the bin fits).  A first-pass bin
// spans 1/16 of an octave of energy.
constexpr int kArcShift = 31 - 12;
__device__ __forceinline__ uint32_t arc_digit(uint32_t key) { return key >> kArcShift; }
// the bin d as a radix state: its bit prefix
__device__ inline void arc_bin_state(uint32_t d, uint32_t* prefix, uint32_t* mask, int32_t* bit) {
    *prefix = d << kArcShift;
    *mask = ~((1u << kArcShift) - 1u);
    *bit = kArcShift;
}

// The first-pass digit derived by every ARC compact block from the merged histogram that an
// EARLIER launch (the key pass) finished, with plain loads (no last-block hand-off in the key
// pass).  Two levels over the slot layout (slot L*32 + g holds bin g*128 + L): with NT a
// multiple of 32, thread tid's PER slots all belong to bin group g = tid & 31, so group
// totals need no transposition; wave 0 picks the group holding the k-th largest key, then
// the bin inside it from that group's 128 counts.  lds: NT + 128 words.  Returns the bin d
// and the keys above it (acc); all NT threads.
template <int NT>
__device__ inline void ms_arc_digit_local(const uint32_t* __restrict__ hist_t, int64_t k, uint32_t* lds,
                                          uint32_t* d_out, uint32_t* acc_out) {
    static_assert(NT % 64 == 0 && kMBins % NT == 0 && kMBins == 32 * 128, "slot layout");
    constexpr int PER = kMBins / NT;  // slots per thread
    constexpr int SUB = NT / 32;      // threads per bin group
    __shared__ uint32_t s_g, s_acc, s_d, s_acc2;
    const int tid = threadIdx.x, lane = tid & 63;
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        c[q] = hist_t[q * NT + tid];  // coalesced: slot q * NT + tid
        sum += c[q];
    }
    lds[tid] = sum;
    __syncthreads();
    if (tid < 64) {  // lane j < 32: group 31 - j (descending bins)
        uint32_t tot = 0;
        if (lane < 32)
            for (int j = 0; j < SUB; ++j) tot += lds[(31 - lane) + 32 * j];
        uint32_t incl = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        const uint64_t excl = incl - tot;
        if (lane < 32 && excl < (uint64_t)k && excl + tot >= (uint64_t)k) {
            s_g = (uint32_t)(31 - lane);
            s_acc = (uint32_t)excl;
        }
    }
    __syncthreads();
    const uint32_t g = s_g;
    if ((uint32_t)(tid & 31) == g) {
#pragma unroll
        for (int q = 0; q < PER; ++q) lds[NT + q * SUB + (tid >> 5)] = c[q];  // lds[NT + L]
    }
    __syncthreads();
    if (tid < 64) {  // lane j: L = 127 - 2j, 126 - 2j
        const uint32_t a0 = lds[NT + 127 - 2 * lane], a1 = lds[NT + 126 - 2 * lane];
        const uint32_t two = a0 + a1;
        uint32_t incl = two;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        const uint64_t excl = (uint64_t)s_acc + incl - two;
        if (excl < (uint64_t)k && excl + two >= (uint64_t)k) {
            const bool first = excl + a0 >= (uint64_t)k;
            s_d = g * 128u + (uint32_t)(first ? 127 - 2 * lane : 126 - 2 * lane);
            s_acc2 = (uint32_t)(first ? excl : excl + a0);
        }
    }
    __syncthreads();
    *d_out = s_d;
    *acc_out = s_acc2;
}


// host-side geometry of one item: fills range / nranges / cand_cap (cand_off by caller)
void ms_item_geometry(MItem& it, int max_ranges = kMMaxRanges);
// workspace bytes for batches whose candidate capacities sum to <= cap_total
int64_t ms_workspace_bytes(int64_t cap_total);

// Launch the whole selection for one batch.  arc: keys come from `keys`, whose producer
// kernel already ran ms_init_item for every item (with the keys' OR / AND); outputs are
// the ascending row list + per-key slot map.  !arc: keys are |x| of `x`; outputs are
// ascending indices + gathered values.  cap_total: candidate slots in the workspace
// (the items' cand_off + cand_cap must fit).  The workspace's `done` counters must be
// zero before the first use (hipMemset once; every kernel leaves them zero).
// zero_x (TopK only, = x or null): write x back with the selected elements zeroed
// hashed (RandK): the keys are rk_key(it.hseed, index) instead of |x| -- the k largest of these
// distinct keys are a uniformly random k-subset, emitted in ascending index order; x (may be null:
// indices only) is then only the source of the gathered values and of zero_x
// fold (1: EF14 with a residual, 2: EF14's first call).  hashed: x is the bucket G and zero_x the
// residual E; the write pass forms v = G (+ E) itself, gathers it and writes E := v with the
// selected elements zeroed (mselect_dev.h, fold_bits).  TopK (fp32, every item 16-B aligned with
// n % 4 == 0): x = zero_x is the residual E and fold_g the bucket G; the first histogram pass
// writes E := G (+ E) as it streams, the later passes read it
int ms_select(const MBatch& b, int64_t maxn, const uint32_t* keys, const void* x, int x_bf16, bool arc,
              MWorkspace* ws, int64_t cap_total, int32_t* out_idx, void* out_val,
              int32_t* out_slot, void* zero_x, hipStream_t st, bool hashed = false, int fold = 0,
              const void* fold_g = nullptr);

// TopK / RandK items of at most kMSmallSel keys: one 1,024-thread block per item of the batch (keys in
// LDS, 8-bit radix rounds, ordered write); the same outputs as ms_select (x / zero_x / fold / fold_g
// as there).  ARCTOPK_EINVAL if an item is larger.
constexpr int kMSmallSel = 12288;  // 48 KiB of LDS keys
int ms_select_small(const MBatch& b, const void* x, int x_bf16, int32_t* out_idx, void* out_val, void* zero_x,
                    hipStream_t st, bool hashed, int fold, const void* fold_g);

// ARC selection after the fused key kernel (keys + first-pass histogram + digit, every
// item in candidate mode), in three launches per batch: ms_arc_compact (per range: the
// bin's keys -> that range's own region of the candidate list, the counts of candidates
// and of keys above the bin; no atomics), then the refine (arctopk_kernels.hip: one block
// per item fixes the remaining bits from the candidates and computes per-range offsets;
// the single-block selects of the small segments share that launch), then ms_arc_write
// (ascending row list and slot map).  ARC candidate regions: range r of item t owns
// ckey[cand_off + r * range, + range) (cand_cap = n).
// (b: the host copy for grid geometry; d_b: the same batch in device memory, read by the kernels)
int ms_arc_compact(const MBatch& b, const MBatch* d_b, const uint32_t* keys, MWorkspace* ws, int64_t cap_total,
                   hipStream_t st);
int ms_arc_write(const MBatch& b, const MBatch* d_b, const uint32_t* keys, MWorkspace* ws, int64_t cap_total,
                 int32_t* out_idx, int32_t* out_slot, hipStream_t st);
// the flat per-range grid of a batch (host)
RangeGrid ms_range_grid(const MBatch& b);

// block x of a flat per-range grid -> (item t, range r); false past the last range
__device__ __forceinline__ bool ms_locate(const RangeGrid& g, int* t, int* r) {
    const int x = (int)blockIdx.x;
    if (x >= g.first[g.cnt]) return false;
    int lo = 0, hi = g.cnt - 1;  // last item with first <= x (binary search over kernel arguments)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (g.first[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    *t = lo;
    *r = x - g.first[lo];
    return true;
}
// candidate keys the ARC refine stages in LDS (more are read from their ranges' regions)
constexpr int kRefineLdsCap = 32768;

}  // namespace arctopk
