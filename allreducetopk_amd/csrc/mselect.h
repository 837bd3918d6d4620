// Multi-block exact top-k selection over uint32 keys, shared by the ARC-TopK large-
// segment select (keys = row-energy bits) and the TopK baseline (keys = |x| bits).
//
// Per item (a tensor / segment) of one batch:
//   start   : known leading bits (ARC: the keys' common prefix from a block OR/AND
//             reduction fused into the key pass; TopK: the sign bit), k still to take
//   hist(p) : every block histograms the next <= 8 varying bits of the keys that match
//             the prefix (per-wave LDS copies against same-bin contention), merged into
//             one global histogram per item with one atomic per bin
//   digit(p): one wave per item picks the digit holding the k-th largest key
//   count   : fixed range partition per item: per-range counts of keys > T and == T
//   offsets : scan over ranges: threshold-equal allowance (lowest ranges first) and
//             output offset per range
//   write   : per-range ballot compaction: ascending indices; ties at T lowest first
// Every launch covers all items of the batch (blockIdx.y = item).
#pragma once
#include "common.h"

namespace arctopk {

constexpr int kMB = 48;          // items per batch (kernel argument size)
constexpr int kMHistBlocks = 512;
constexpr int kMRanges = 256;    // compaction ranges per item

struct MItem {
    int64_t key_off;   // keys / x offset of the item
    int64_t n;         // keys
    int64_t k;         // keys to select
    int64_t out_off;   // output offset (TopK: idx/vals; ARC: row list)
    int64_t slot_off;  // ARC: slot map offset (per key)
};

struct MBatch {
    MItem it[kMB];
    int32_t cnt;
};

struct MState {
    uint32_t prefix, mask;
    int32_t bit;       // bits [bit-1 .. 0] still undecided
    int32_t pad;
    int64_t kk;        // keys still to take among those matching the prefix
    uint32_t kor, kand;  // OR / AND of all keys (ARC start)
};

struct MWorkspace {
    uint32_t hist[kMB][256];
    MState st[kMB];
    int64_t cnt_gt[kMB][kMRanges];
    int64_t cnt_eq[kMB][kMRanges];
    int64_t take_eq[kMB][kMRanges];
    int64_t sel_before[kMB][kMRanges];
};

// Launch the whole selection for one batch (11 launches).  arc = true: keys come from
// `keys` and the item states already hold the keys' OR / AND (ms_reset_orand before the
// key pass); outputs are the ascending row list + per-key slot map.  arc = false: keys
// are |x| of `x`; outputs are ascending indices + gathered values.
int ms_select(const MBatch& b, int64_t maxn, const uint32_t* keys, const float* x, bool arc,
              MWorkspace* ws, int32_t* out_idx, float* out_val, int32_t* out_slot, hipStream_t st);
int ms_reset_orand(MWorkspace* ws, int cnt, hipStream_t st);

}  // namespace arctopk
