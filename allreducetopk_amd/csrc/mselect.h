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
};

struct MBatch {
    MItem it[kMB];
    int32_t cnt;
};

struct MState {
    uint32_t prefix, mask;  // decided leading bits
    int32_t bit;            // bits [bit-1 .. 0] still undecided
    int32_t cand;           // 1: candidates were compacted, later passes read only them
    int64_t kk;             // keys still to take among those matching the prefix
    uint32_t kor, kand;     // OR / AND of all keys (ARC start)
    uint32_t p1, m1;        // the first-pass bin (its keys are the candidates)
    uint32_t ncand;         // candidates appended
    uint32_t pad;
};

struct MWorkspace {
    uint32_t hist[kMB][kMBins];
    MState st[kMB];
    uint32_t cnt_gt[kMB][kMMaxRanges];
    uint32_t cnt_eq[kMB][kMMaxRanges];
    uint32_t take_eq[kMB][kMMaxRanges];
    uint32_t sel_before[kMB][kMMaxRanges];
    // followed by the candidate lists: uint32 key[cap_total], uint32 index[cap_total]
};

// host-side geometry of one item: fills range / nranges / cand_cap (cand_off by caller)
void ms_item_geometry(MItem& it);
// workspace bytes for batches whose candidate capacities sum to <= cap_total
int64_t ms_workspace_bytes(int64_t cap_total);

// Launch the whole selection for one batch.  arc = true: keys come from `keys` and the
// item states already hold the keys' OR / AND (ms_reset_orand before the key pass);
// outputs are the ascending row list + per-key slot map.  arc = false: keys are |x| of
// `x`; outputs are ascending indices + gathered values.  cap_total: candidate slots in
// the workspace (the items' cand_off + cand_cap must fit).
int ms_select(const MBatch& b, int64_t maxn, const uint32_t* keys, const float* x, bool arc,
              MWorkspace* ws, int64_t cap_total, int32_t* out_idx, float* out_val,
              int32_t* out_slot, hipStream_t st);
int ms_reset_orand(MWorkspace* ws, int cnt, hipStream_t st);

}  // namespace arctopk
