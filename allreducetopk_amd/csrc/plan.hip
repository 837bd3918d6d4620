// Bucket plan: geometry of every gradient view (reference cal_k / reshape rules),
// buffer offsets, and the work tables of the encode / pack / decode kernels.
// Built once per bucket layout; nothing here runs per call.
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <new>
#include <numeric>
#include <vector>

#include "common.h"
#include "mselect.h"

using namespace arctopk;

namespace {

int build_segments(const int64_t* dims, const int32_t* ndims, int32_t ntensors, int r, double ratio,
                   std::vector<arctopk_segment>& segs, arctopk_plan_info& info) {
    int64_t off = 0, sk = 0, vo = 0, po = 0, ro = 0, so = 0, vals = 0;
    const int64_t* d = dims;
    for (int i = 0; i < ntensors; ++i) {
        const int nd = ndims[i];
        if (nd < 1) return ARCTOPK_EINVAL;  // 0-dim: shape[-1] fails in the reference
        int64_t numel = 1;
        for (int j = 0; j < nd; ++j) numel *= d[j];
        arctopk_segment s;
        std::memset(&s, 0, sizeof(s));
        s.offset = off;
        if (nd == 1) {                      // ref :19-41
            s.kind = ARCTOPK_SEG_RAW;
            s.n = numel;
            s.m = 1;
        } else if (nd == 2) {               // ref :44-47
            s.kind = ARCTOPK_SEG_SKETCH;
            s.n = d[0];
            s.m = d[1];
        } else {                            // ref :72-77
            const int64_t t = d[nd - 1];
            s.kind = ARCTOPK_SEG_SKETCH;
            s.m = 2 * t * t;
            if (s.m == 0) return ARCTOPK_EEMPTY;
            s.n = numel / s.m;
            if (s.n * s.m != numel) return ARCTOPK_ERESHAPE;
        }
        if (numel == 0 || s.n == 0 || s.m == 0) return ARCTOPK_EEMPTY;
        if (numel >= (int64_t(1) << 31)) return ARCTOPK_EINVAL;  // 32-bit in-segment indexing
        if (s.kind == ARCTOPK_SEG_SKETCH && s.m * r >= (int64_t(1) << 31)) return ARCTOPK_EINVAL;  // V: m * r
        // k = max(1, int(n * ratio)): float64 product, truncation (ref cal_k :173-187)
        int64_t k = (int64_t)((double)s.n * ratio);
        if (k < 1) k = 1;
        if (k > s.n) return ARCTOPK_EINVAL;  // torch.topk raises for k > n
        s.k_rows = k;
        s.sketch_off = sk;
        sk += (s.kind == ARCTOPK_SEG_RAW) ? s.n : s.n * r;
        s.v_off = (s.kind == ARCTOPK_SEG_RAW) ? -1 : vo;
        if (s.kind == ARCTOPK_SEG_SKETCH) vo += s.m * r;
        s.packed_off = po;
        po += k * s.m;
        vals += k * s.m;
        po = (po + 3) & ~int64_t(3);  // 16-B aligned segments: vector pack / decode paths
        s.row_off = ro;
        ro += s.n;
        s.sel_off = so;
        so += k;
        segs.push_back(s);
        off += numel;
        d += nd;
    }
    info.numel = off;
    info.sketch_len = sk;
    info.v_len = vo;
    info.packed_len = po;
    info.values_len = vals;
    info.sel_rows = so;
    info.rows_total = ro;
    info.nseg = ntensors;
    info.r = r;
    return 0;
}

}  // namespace

extern "C" int arctopk_plan_create(const int64_t* dims, const int32_t* ndims, int32_t ntensors,
                                   int32_t r, double compress_ratio, int32_t dtype, int32_t device,
                                   arctopk_plan** out) {
    if (!dims || !ndims || !out || ntensors < 1) return ARCTOPK_EINVAL;
    if (r < 1 || r > kMaxR) return ARCTOPK_EINVAL;
    if (!(compress_ratio > 0.0) || compress_ratio > 1.0) return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EDTYPE;
    *out = nullptr;

    std::vector<arctopk_segment> segs;
    arctopk_plan_info info;
    std::memset(&info, 0, sizeof(info));
    int st = build_segments(dims, ndims, ntensors, r, compress_ratio, segs, info);
    if (st) return st;

    std::vector<SegDev> dsegs(segs.size());
    std::vector<int32_t> small_ids, large_ids, split_ids;
    // Single-block selects up to kSmallSelRows rows -- but in a bucket that has multi-block
    // items anyway, only the ones that fit 256-thread blocks: the rest join the multi-block
    // batch, so the batch's write launch can host the small selects (and a deferred decode)
    // and the separate refine launch is not needed
    bool any_large = false;
    for (const arctopk_segment& s : segs) any_large = any_large || s.n > kSmallSelRows;
    const int64_t small_cap = any_large ? (int64_t)ARCTOPK_SMALL_SEL_ROWS_MIXED : (int64_t)kSmallSelRows;
    int64_t small_rows = 0;
    std::vector<EncTile> enc;
    std::vector<Chunk> pack, dec;
    std::vector<int32_t> pack_begin, dec_begin;
    int lds = 0;
    int64_t dec_lds = 0;
    // Encode work sizing: tiles of wave-per-row segments hold enough rows that the
    // bucket yields ~kEncTargetBlocks blocks (a bucket may hold ONE tensor: a DDP bucket
    // of a 46 MB MLP weight must still fill 256 CUs), within [8K, 64K] elements per block.
    int64_t row_work = 0;
    for (const arctopk_segment& s : segs)
        if (s.kind != ARCTOPK_SEG_RAW && !(s.m < kSmallM && (kTileRows * s.m + s.m * r) * 4 <= 65536))
            row_work += s.n * s.m;
    const int64_t target = kEncTargetBlocks;
    // (small buckets: tiles down to ARCTOPK_ENC_MIN_TILE elements -- at least one row per wave --
    // so a bucket of a few rows spreads them over waves instead of walking them in sequence)
    const int64_t tile_elems = std::min<int64_t>(65536, std::max<int64_t>(ARCTOPK_ENC_MIN_TILE, row_work / target));
    static_assert(ARCTOPK_ENC_MIN_TILE <= 65536, "encode tiles hold at most 64 Ki elements");
    // a second table for the fp32 kernels that also stream E (EF14 after the first call, EF21):
    // tensors of at least ARCTOPK_ENC_E_MIN_ROWS rows (embeddings) get tiles sized for twice the
    // block target (A/B: Llama-1B embedding bucket 1,072 -> 1,137 GB/s, RoBERTa 994 -> 1,008;
    // for every tensor it cost the headline 1 % and the G-only and bf16 kernels 2-3 %)
    const int64_t tile_elems_e = std::min<int64_t>(
        65536, std::max<int64_t>(ARCTOPK_ENC_MIN_TILE, row_work / (int64_t)ARCTOPK_ENC_TARGET_BLOCKS_E));
    std::vector<EncTile> enc_e;
    bool any_e = false;
    // chunk sizes (build-time A/B switches, common.h): short rows (m < 256) and the m <= 2
    // streams get smaller chunks, more blocks in flight (ResNet-50 1x1 mix, 2048-element
    // stream pack chunks: 346 -> 356 GB/s; 4096-element decode chunks: +3 %)
    constexpr int64_t pack_elems = ARCTOPK_PACK_CHUNK, dec_elems = ARCTOPK_DEC_CHUNK;
    constexpr int64_t stream_pack_elems = ARCTOPK_STREAM_PACK_CHUNK;
    constexpr int64_t short_dec_elems = ARCTOPK_SHORT_DEC_CHUNK;
    int64_t part_len = 0, split_rows_max = 0;
    // vector paths: 16-B encode units (4 fp32 / 8 bf16 elements) need m and the offset to be
    // multiples of va; pack / decode quads need 4
    const int64_t va = dtype == ARCTOPK_BF16 ? 8 : 4;
    for (size_t i = 0; i < segs.size(); ++i) {
        const arctopk_segment& s = segs[i];
        SegDev& g = dsegs[i];
        g.offset = s.offset; g.n = s.n; g.m = s.m; g.k_rows = s.k_rows;
        g.sketch_off = s.sketch_off; g.v_off = s.v_off; g.packed_off = s.packed_off;
        g.row_off = s.row_off; g.sel_off = s.sel_off; g.kind = s.kind;
        g.vec = (s.m % va == 0 && s.offset % va == 0) ? 1 : 0;  // packed_off is 4-aligned
        g.mdiv = make_fastdiv((uint32_t)s.m);
        g.magic32 = s.m > 1 ? (uint32_t)(((1ull << 32) + (uint64_t)s.m - 1) / (uint64_t)s.m) : 0u;
        g.nparts = 1;
        g.part_off = 0;
        if (s.n <= small_cap) {
            small_ids.push_back((int32_t)i);
            small_rows = std::max<int64_t>(small_rows, s.n);
        } else {
            large_ids.push_back((int32_t)i);
        }
        // ---- encode tiles
        if (s.kind == ARCTOPK_SEG_RAW) {
            const int64_t per = 4096;
            for (int64_t e = 0; e < s.n; e += per)
                for (std::vector<EncTile>* dst : {&enc, &enc_e})
                    dst->push_back(EncTile{(int32_t)i, ENC_RAW, e, std::min(per, s.n - e), 0, 1, -1, 1});
        } else if (s.m < kSmallM && (kTileRows * s.m + s.m * r) * 4 <= 65536) {
            // rows per tile: ~kSmallTileBytes of the tensor (multiples of 256 rows), so the
            // smallest m (1x1 convs, m = 2) does not run thousands of 2 KiB blocks
            const int64_t tr = std::max<int64_t>(kTileRows, kSmallTileBytes / (4 * s.m) / kTileRows * kTileRows);
            for (int64_t row = 0; row < s.n; row += tr)
                for (std::vector<EncTile>* dst : {&enc, &enc_e})
                    dst->push_back(EncTile{(int32_t)i, ENC_TILE, row, std::min<int64_t>(tr, s.n - row),
                                           0, (int32_t)s.m, -1, 1});
            lds = std::max<int>(lds, (int)(std::min(tr, s.n) * s.m * 4 + ((s.m * r + 3) & ~3) * 4));
        } else {
            const int mode = g.vec ? ENC_ROW_VEC : ENC_ROW_SCALAR;
            // columns per part: V^T slice [r][clen] within kVLdsMaxBytes (multiple of 4)
            const int64_t max_cols = (kVLdsMaxBytes / (4 * r)) / va * va;
            const int nparts = (int)((s.m + max_cols - 1) / max_cols);
            int64_t clen = (s.m + nparts - 1) / nparts;
            clen = (clen + va - 1) / va * va;
            if (nparts > 1) {
                g.nparts = nparts;
                g.part_off = part_len;
                part_len += (int64_t)nparts * s.n * r;
                split_ids.push_back((int32_t)i);
                split_rows_max = std::max<int64_t>(split_rows_max, s.n);
            }
            for (int tab = 0; tab < 2; ++tab)
            for (int part = 0; part < nparts; ++part) {
                const bool big = s.n >= (int64_t)ARCTOPK_ENC_E_MIN_ROWS;
                any_e = any_e || (tab && big);
                const int64_t te = tab && big ? tile_elems_e : tile_elems;
                const int64_t c0 = part * clen;
                const int64_t cl = std::min<int64_t>(clen, s.m - c0);
                // tiles: this part's share of the block target, rounded to nearest (a bucket of
                // equal tensors gets exactly the target: a whole number of resident rounds, no
                // partial last round), within [te / 64 Ki-element, one per 4 rows]
                const double work = (double)s.n * (double)cl;
                int64_t ntiles = std::llround(work / (double)te);
                ntiles = std::max<int64_t>(ntiles, (int64_t)std::ceil(work / 65536.0));
                ntiles = std::min<int64_t>(ntiles, std::max<int64_t>(1, s.n / 4));
                ntiles = std::max<int64_t>(ntiles, 1);
                std::vector<EncTile>& dst = tab ? enc_e : enc;
                // tile ti holds rows ti, ti + ntiles, ...: consecutive blocks read adjacent rows
                for (int64_t ti = 0; ti < ntiles; ++ti)
                    dst.push_back(EncTile{(int32_t)i, mode, ti, (s.n - ti + ntiles - 1) / ntiles,
                                          (int32_t)c0, (int32_t)cl, nparts > 1 ? part : -1, (int32_t)ntiles});
                lds = std::max<int>(lds, (int)(cl * r * 4));
            }
        }
        // keys mode (world size 1): a multi-block select item's encode writes the energy keys its
        // key pass would form from the sketch (unsplit 2-D / ND tensors)
        g.keyed = (s.n > small_cap && s.kind == ARCTOPK_SEG_SKETCH && g.nparts == 1) ? 1 : 0;
        g.pad_k = 0;
        // ---- pack chunks: selected rows, ~kChunkElems elements each (small m: at most
        //      kSmallTileRows rows, the size of the kernels' LDS row/slot table)
        pack_begin.push_back((int32_t)pack.size());
        dec_begin.push_back((int32_t)dec.size());
        const bool small_tile = s.m >= 4 && s.m < 256;
        // (rows of >= 256 elements go one per wave: at least 4 rows per chunk)
        const int64_t min_rows = s.m >= 256 ? 4 : 1;
        // 1-D tensors and 1x1-conv rows (m = 1, 2) with 16-B aligned data stream over ALL rows
        // with the slot map (mode 1: one 16-B quad of E per lane, whole quads rewritten):
        // their 4- and 8-B rows are too short for per-row gathers
        const bool stream_small = (s.m == 1 || s.m == 2) && s.offset % 4 == 0 && dtype == ARCTOPK_F32;
        if (stream_small) {
            const int64_t per = (stream_pack_elems / s.m + 3) / 4 * 4;  // quads never straddle chunks
            for (int64_t row = 0; row < s.n; row += per)
                pack.push_back(Chunk{(int32_t)i, 1, row, std::min(per, s.n - row)});
        } else {
            int64_t per = std::max<int64_t>(min_rows, pack_elems / s.m);
            if (small_tile) per = std::min<int64_t>(per, kSmallTileRows);
            for (int64_t j = 0; j < s.k_rows; j += per)
                pack.push_back(Chunk{(int32_t)i, 0, j, std::min(per, s.k_rows - j)});
        }
        // ---- decode chunks: all rows
        g.dchunk0 = (int32_t)dec.size();
        g.dchunk_rows = 0;
        // mode 3 (short rows, quad-aligned data): chunks of <= ARCTOPK_SHORT3_CHUNK elements whose
        // first elements are quad-aligned (rows per chunk a multiple of 4 / gcd(m, 4))
        const int64_t q3 = 4 / std::gcd<int64_t>(s.m, 4);
        if (small_tile && s.offset % 4 == 0 &&
            (int64_t)ARCTOPK_SHORT3_CHUNK / s.m >= q3) {
            const int64_t per = (int64_t)ARCTOPK_SHORT3_CHUNK / s.m / q3 * q3;
            g.dchunk_rows = (int32_t)per;
            for (int64_t row = 0; row < s.n; row += per)
                dec.push_back(Chunk{(int32_t)i, 3, row, std::min(per, s.n - row)});
            dec_lds = std::max<int64_t>(dec_lds, (std::min(per, s.n) * (s.m + 1) + 12) * 4);  // + alignment, quad lead
        } else if (small_tile && dtype == ARCTOPK_F32) {
            // mode 2: lane per 16-B output quad, rows of whole chunks (no LDS tile)
            const int64_t per = std::max<int64_t>(1, (int64_t)ARCTOPK_QUAD_DEC_CHUNK / s.m);
            for (int64_t row = 0; row < s.n; row += per)
                dec.push_back(Chunk{(int32_t)i, 2, row, std::min(per, s.n - row)});
        } else {
            int64_t per = std::max<int64_t>(min_rows, (s.m < 256 ? short_dec_elems : dec_elems) / s.m);
            if (stream_small) per = (per + 3) / 4 * 4;  // mode 1: whole quads per chunk
            if (small_tile)  // the chunk tile lives in LDS: <= 64 KiB
                per = std::min<int64_t>(std::min<int64_t>(per, kSmallTileRows), 16000 / s.m);
            for (int64_t row = 0; row < s.n; row += per)
                dec.push_back(Chunk{(int32_t)i, stream_small ? 1 : 0, row, std::min(per, s.n - row)});
            if (small_tile) dec_lds = std::max<int64_t>(dec_lds, (std::min(per, s.n) * s.m + 4) * 4);
        }
    }

    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return (int)e;
    arctopk_plan* p = new (std::nothrow) arctopk_plan;
    if (!p) return ARCTOPK_EINVAL;
    std::memset(p, 0, sizeof(*p));
    p->device = device;
    p->dtype = dtype;
    p->r = r;
    p->ratio = compress_ratio;
    p->nseg = (int)segs.size();
    p->info = info;
    p->h_segs = new arctopk_segment[segs.size()];
    std::copy(segs.begin(), segs.end(), p->h_segs);
    p->n_enc = (int)enc.size();
    p->n_enc_e = dtype == ARCTOPK_F32 && any_e ? (int)enc_e.size() : 0;
    p->n_pack = (int)pack.size();
    p->n_dec = (int)dec.size();
    pack_begin.push_back((int32_t)pack.size());
    dec_begin.push_back((int32_t)dec.size());
    p->h_pack_begin = new int32_t[pack_begin.size()];
    p->h_dec_begin = new int32_t[dec_begin.size()];
    std::copy(pack_begin.begin(), pack_begin.end(), p->h_pack_begin);
    std::copy(dec_begin.begin(), dec_begin.end(), p->h_dec_begin);
    p->enc_lds_bytes = lds;
    // the lean encode kernel for tables of short rows (its blocks are latency-bound: more of them
    // resident at once), up to a few rounds of blocks -- a large bucket streams faster at
    // k_encode's occupancy (28 x [512, 512, 3, 3]: 14,336 tiles, 134 -> 139 us lean)
    p->enc_short = (int)enc.size() <= ARCTOPK_ENC_SHORT_MAX_TILES;
    for (const EncTile& et : enc) p->enc_short = p->enc_short && (et.mode == ENC_RAW || et.mode == ENC_TILE);
    p->dec_lds_bytes = (int)dec_lds;
    p->n_small = (int)small_ids.size();
    for (const SegDev& g : dsegs) p->any_keyed = p->any_keyed || g.keyed;
    p->n_large = (int)large_ids.size();
    p->small_lds = (int)(((small_rows + 3) & ~3) * 4 + 16);
#define ALLOC_COPY(dst, vec)                                                                  \
    do {                                                                                      \
        e = hipMalloc((void**)&dst, std::max<size_t>(1, vec.size() * sizeof(vec[0])));        \
        if (e == hipSuccess && !vec.empty())                                                  \
            e = hipMemcpy(dst, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice); \
        if (e != hipSuccess) { arctopk_plan_destroy(p); return (int)e; }                      \
    } while (0)
    ALLOC_COPY(p->d_segs, dsegs);
    ALLOC_COPY(p->d_enc, enc);
    if (p->n_enc_e) ALLOC_COPY(p->d_enc_e, enc_e);
    ALLOC_COPY(p->d_pack, pack);
    ALLOC_COPY(p->d_dec, dec);
    e = hipMalloc((void**)&p->d_dfirst, (dec.size() + 1) * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemset(p->d_dfirst, 0, (dec.size() + 1) * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc((void**)&p->d_dfirst_pub, (dec.size() + 1) * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemset(p->d_dfirst_pub, 0, (dec.size() + 1) * sizeof(int32_t));
    if (e != hipSuccess) { arctopk_plan_destroy(p); return (int)e; }
    {
        std::vector<int32_t> m3;
        for (size_t i = 0; i < dsegs.size(); ++i)
            if (dsegs[i].dchunk_rows > 0) m3.push_back((int32_t)i);
        p->n_m3 = (int)m3.size();
        ALLOC_COPY(p->d_m3, m3);
    }
    ALLOC_COPY(p->d_small, small_ids);
    ALLOC_COPY(p->d_large, large_ids);
    ALLOC_COPY(p->d_split, split_ids);
    p->n_split = (int)split_ids.size();
    p->split_rows_max = split_rows_max;
    if (part_len > 0) {
        e = hipMalloc((void**)&p->d_part, (size_t)part_len * sizeof(float));
        if (e != hipSuccess) { arctopk_plan_destroy(p); return (int)e; }
    }
    if (!large_ids.empty()) {
        p->n_large_batches = (int)((large_ids.size() + kMB - 1) / kMB);
        p->h_large_batches = new MBatch[p->n_large_batches];
        for (int bi = 0; bi < p->n_large_batches; ++bi) {
            MBatch& b = p->h_large_batches[bi];
            b.cnt = (int32_t)std::min<size_t>(kMB, large_ids.size() - (size_t)bi * kMB);
            int64_t cap = 0;
            for (int i = 0; i < b.cnt; ++i) {
                const arctopk_segment& sg = segs[large_ids[(size_t)bi * kMB + i]];
                MItem& it = b.it[i];
                it.key_off = sg.row_off;
                it.n = sg.n;
                it.k = sg.k_rows;
                it.out_off = sg.sel_off;
                it.slot_off = sg.row_off;
                ms_item_geometry(it);
                it.cand_cap = it.n;  // ARC: every key of the first-pass bin is a candidate
                it.cand_off = cap;
                cap += it.cand_cap;
            }
            p->mws_cap = std::max(p->mws_cap, cap);
        }
        e = hipMalloc((void**)&p->d_large_batches, sizeof(MBatch) * (size_t)p->n_large_batches);
        if (e == hipSuccess)
            e = hipMemcpy(p->d_large_batches, p->h_large_batches, sizeof(MBatch) * (size_t)p->n_large_batches,
                          hipMemcpyHostToDevice);
        if (e != hipSuccess) { arctopk_plan_destroy(p); return (int)e; }
        e = hipMalloc((void**)&p->d_mws, (size_t)ms_workspace_bytes(p->mws_cap));
        if (e != hipSuccess) { arctopk_plan_destroy(p); return (int)e; }
        // arrival counters start at zero (each select kernel leaves them zero)
        e = hipMemset(p->d_mws, 0, sizeof(MWorkspace));
        if (e != hipSuccess) { arctopk_plan_destroy(p); return (int)e; }
    }
    {  // device projection draws
        std::vector<VDraw> vd(segs.size());
        int nvd = 0;
        uint64_t adv = 0;
        const int ve = vdraw_table(segs.data(), (int)segs.size(), r, device, vd.data(), &nvd, &adv);
        if (ve) { arctopk_plan_destroy(p); return ve; }
        vd.resize(nvd);
        p->n_vdraw = nvd;
        p->vdraw_advance = adv;
        for (const VDraw& d : vd) p->vdraw_max = std::max<int64_t>(p->vdraw_max, d.numel);
        ALLOC_COPY(p->d_vdraw, vd);
        std::vector<VChunk> vc;
        for (int i = 0; i < nvd; ++i)
            for (int64_t lo = 0; lo < vd[i].numel; lo += kVChunk)
                vc.push_back({i, (uint32_t)lo, (uint32_t)std::min<int64_t>(vd[i].numel, lo + kVChunk)});
        p->n_vchunk = (int)vc.size();
        ALLOC_COPY(p->d_vchunk, vc);
    }
#undef ALLOC_COPY
    e = hipMalloc((void**)&p->d_keys, std::max<size_t>(4, info.rows_total * sizeof(uint32_t)));
    if (e != hipSuccess) { arctopk_plan_destroy(p); return (int)e; }
    *out = p;
    return 0;
}

// A plan over segments [seg_begin, seg_end) of `parent` (a group of consecutive tensors of the
// bucket): its own work tables, the parent's geometry and projection draws.  A tensor's
// geometry depends on (kind, n, m) only, so each segment is planned as a [n] (RAW) or [n, m]
// (SKETCH) tensor; the draw table keeps the parent's Philox offsets (a tensor's V is the one
// the whole bucket's draw gives it), with V offsets relative to the group's first SKETCH tensor.
// The group's offsets differ from the parent's by the group's base offsets, which must keep
// every alignment the kernels test (16-B units: multiples of 8 elements).
extern "C" int arctopk_plan_group(const arctopk_plan* parent, int32_t seg_begin, int32_t seg_end,
                                  arctopk_plan** out) {
    if (!parent || !out || seg_begin < 0 || seg_end > parent->nseg || seg_begin >= seg_end) return ARCTOPK_EINVAL;
    *out = nullptr;
    const arctopk_segment& b0 = parent->h_segs[seg_begin];
    if (b0.offset % 8 || b0.sketch_off % 8 || b0.packed_off % 8 || b0.row_off % 4)
        return ARCTOPK_EINVAL;
    int64_t vbase = -1;
    for (int i = seg_begin; i < seg_end && vbase < 0; ++i)
        if (parent->h_segs[i].kind == ARCTOPK_SEG_SKETCH) vbase = parent->h_segs[i].v_off;
    if (vbase > 0 && vbase % 8) return ARCTOPK_EINVAL;
    std::vector<int64_t> dims;
    std::vector<int32_t> nd;
    for (int i = seg_begin; i < seg_end; ++i) {
        const arctopk_segment& s = parent->h_segs[i];
        dims.push_back(s.n);
        if (s.kind == ARCTOPK_SEG_SKETCH) dims.push_back(s.m);
        nd.push_back(s.kind == ARCTOPK_SEG_SKETCH ? 2 : 1);
    }
    arctopk_plan* c = nullptr;
    int e = arctopk_plan_create(dims.data(), nd.data(), (int32_t)nd.size(), parent->r, parent->ratio,
                                parent->dtype, parent->device, &c);
    if (e) return e;
    for (int i = seg_begin; i < seg_end; ++i) {  // same geometry, offsets shifted by the base
        const arctopk_segment& s = parent->h_segs[i];
        const arctopk_segment& g = c->h_segs[i - seg_begin];
        if (g.kind != s.kind || g.n != s.n || g.m != s.m || g.k_rows != s.k_rows ||
            g.offset != s.offset - b0.offset || g.sketch_off != s.sketch_off - b0.sketch_off ||
            g.packed_off != s.packed_off - b0.packed_off || g.sel_off != s.sel_off - b0.sel_off ||
            g.row_off != s.row_off - b0.row_off ||
            (s.kind == ARCTOPK_SEG_SKETCH && g.v_off != s.v_off - vbase)) {
            arctopk_plan_destroy(c);
            return ARCTOPK_EINVAL;
        }
    }
    // the parent's draws of this group's SKETCH tensors
    std::vector<VDraw> vd(parent->nseg);
    int nvd = 0;
    uint64_t adv = 0;
    e = vdraw_table(parent->h_segs, parent->nseg, parent->r, parent->device, vd.data(), &nvd, &adv);
    if (e) { arctopk_plan_destroy(c); return e; }
    std::vector<VDraw> mine;
    for (int i = 0, j = 0; i < parent->nseg; ++i) {
        if (parent->h_segs[i].kind != ARCTOPK_SEG_SKETCH) continue;
        if (i >= seg_begin && i < seg_end) {
            VDraw d = vd[j];
            d.v_off -= vbase;
            mine.push_back(d);
        }
        ++j;
    }
    std::vector<VChunk> vc;
    for (size_t i = 0; i < mine.size(); ++i)
        for (int64_t lo = 0; lo < mine[i].numel; lo += kVChunk)
            vc.push_back({(int32_t)i, (uint32_t)lo, (uint32_t)std::min<int64_t>(mine[i].numel, lo + kVChunk)});
    hipError_t he = hipSetDevice(parent->device);
    if (c->d_vdraw) (void)hipFree(c->d_vdraw);
    if (c->d_vchunk) (void)hipFree(c->d_vchunk);
    c->d_vdraw = nullptr;
    c->d_vchunk = nullptr;
    if (he == hipSuccess) he = hipMalloc((void**)&c->d_vdraw, std::max<size_t>(1, mine.size() * sizeof(VDraw)));
    if (he == hipSuccess && !mine.empty())
        he = hipMemcpy(c->d_vdraw, mine.data(), mine.size() * sizeof(VDraw), hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMalloc((void**)&c->d_vchunk, std::max<size_t>(1, vc.size() * sizeof(VChunk)));
    if (he == hipSuccess && !vc.empty())
        he = hipMemcpy(c->d_vchunk, vc.data(), vc.size() * sizeof(VChunk), hipMemcpyHostToDevice);
    if (he != hipSuccess) { arctopk_plan_destroy(c); return (int)he; }
    c->n_vdraw = (int)mine.size();
    c->n_vchunk = (int)vc.size();
    c->vdraw_advance = parent->vdraw_advance;  // (the bucket's: reseeds use the parent's)
    *out = c;
    return 0;
}

extern "C" int arctopk_plan_describe(const int64_t* dims, const int32_t* ndims, int32_t ntensors,
                                     int32_t r, double compress_ratio, arctopk_segment* segs_out,
                                     arctopk_plan_info* info) {
    if (!dims || !ndims || !info || ntensors < 1) return ARCTOPK_EINVAL;
    if (r < 1 || r > kMaxR) return ARCTOPK_EINVAL;
    if (!(compress_ratio > 0.0) || compress_ratio > 1.0) return ARCTOPK_EINVAL;
    std::vector<arctopk_segment> segs;
    std::memset(info, 0, sizeof(*info));
    int st = build_segments(dims, ndims, ntensors, r, compress_ratio, segs, *info);
    if (st) return st;
    if (segs_out) std::copy(segs.begin(), segs.end(), segs_out);
    return 0;
}

extern "C" int arctopk_plan_destroy(arctopk_plan* p) {
    if (!p) return 0;
    (void)hipSetDevice(p->device);
    if (p->d_segs) (void)hipFree(p->d_segs);
    if (p->d_enc) (void)hipFree(p->d_enc);
    if (p->d_enc_e) (void)hipFree(p->d_enc_e);
    if (p->d_pack) (void)hipFree(p->d_pack);
    if (p->d_dec) (void)hipFree(p->d_dec);
    if (p->d_dfirst) (void)hipFree(p->d_dfirst);
    if (p->d_dfirst_pub) (void)hipFree(p->d_dfirst_pub);
    if (p->d_m3) (void)hipFree(p->d_m3);
    if (p->d_keys) (void)hipFree(p->d_keys);
    if (p->d_small) (void)hipFree(p->d_small);
    if (p->d_large) (void)hipFree(p->d_large);
    if (p->d_split) (void)hipFree(p->d_split);
    if (p->d_part) (void)hipFree(p->d_part);
    delete[] p->h_segs;
    delete[] p->h_pack_begin;
    arctopk::exchange_forget(p);  // before its events go
    if (p->x_ev_packed) (void)hipEventDestroy((hipEvent_t)p->x_ev_packed);
    if (p->x_ev_ar) (void)hipEventDestroy((hipEvent_t)p->x_ev_ar);
    if (p->x_ev_dec) (void)hipEventDestroy((hipEvent_t)p->x_ev_dec);
    if (p->x_ev_enc) (void)hipEventDestroy((hipEvent_t)p->x_ev_enc);
    if (p->x_ev_join) (void)hipEventDestroy((hipEvent_t)p->x_ev_join);
    delete[] p->h_large_batches;
    if (p->d_large_batches) (void)hipFree(p->d_large_batches);
    if (p->d_mws) (void)hipFree(p->d_mws);
    if (p->d_vdraw) (void)hipFree(p->d_vdraw);
    if (p->d_vchunk) (void)hipFree(p->d_vchunk);
    delete[] p->h_dec_begin;
    delete p;
    return 0;
}

extern "C" int arctopk_plan_query(const arctopk_plan* p, arctopk_plan_info* info) {
    if (!p || !info) return ARCTOPK_EINVAL;
    *info = p->info;
    return 0;
}

extern "C" int arctopk_plan_segment(const arctopk_plan* p, int32_t i, arctopk_segment* seg) {
    if (!p || !seg || i < 0 || i >= p->nseg) return ARCTOPK_EINVAL;
    *seg = p->h_segs[i];
    return 0;
}

extern "C" int arctopk_event_create(void** event) {
    if (!event) return ARCTOPK_EINVAL;
    hipEvent_t e = nullptr;
    const hipError_t st = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice);
    *event = st == hipSuccess ? (void*)e : nullptr;
    return (int)st;
}

extern "C" int arctopk_event_create_timed(void** event) {
    if (!event) return ARCTOPK_EINVAL;
    hipEvent_t e = nullptr;
    const hipError_t st = hipEventCreateWithFlags(&e, hipEventReleaseToDevice);
    *event = st == hipSuccess ? (void*)e : nullptr;
    return (int)st;
}

extern "C" int arctopk_event_elapsed_ms(float* ms, void* start, void* end) {
    if (!ms || !start || !end) return ARCTOPK_EINVAL;
    return (int)hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end);
}

extern "C" int arctopk_event_destroy(void* event) {
    return event ? (int)hipEventDestroy((hipEvent_t)event) : 0;
}

extern "C" int arctopk_event_record(void* event, void* stream) {
    if (!event) return ARCTOPK_EINVAL;
    return (int)hipEventRecord((hipEvent_t)event, (hipStream_t)stream);
}

extern "C" int arctopk_event_wait(void* stream, void* event) {
    if (!event) return ARCTOPK_EINVAL;
    return (int)hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0);
}

extern "C" int arctopk_event_query(void* event) {
    if (!event) return ARCTOPK_EINVAL;
    const hipError_t st = hipEventQuery((hipEvent_t)event);
    if (st == hipSuccess) return 0;
    if (st == hipErrorNotReady) return 1;
    return (int)st;
}

#ifndef ARCTOPK_SRC_HASH
#define ARCTOPK_SRC_HASH "unknown0000000000"
#endif
// "src:<hash>" is the build recipe's source hash (allreducetopk_amd/build.py): the loader
// refuses a library built from other sources than the ones next to it
extern "C" const char* arctopk_version(void) {
    return "libarctopk 0.2 gfx950 (ARC-TopK encode/select/pack/decode, TopK/RandK) src:" ARCTOPK_SRC_HASH;
}
