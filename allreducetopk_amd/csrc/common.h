// Shared device-side structures of libarctopk (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arctopk.h"

// Build-time tuning constants (build(defines=[...]) makes A/B variants; the product library
// has no run-time tuning knobs and one code path per feature).  Selects:
#ifndef ARCTOPK_ENC_SHORT_MAX_TILES
#define ARCTOPK_ENC_SHORT_MAX_TILES 8192  // largest tile table of the lean short-row encode kernel
#endif
#ifndef ARCTOPK_SEL_BIG_ROWS
#define ARCTOPK_SEL_BIG_ROWS 4096      // single-block select: 1024 threads above this many rows
#endif
#ifndef ARCTOPK_SMALL_SEL_ROWS_MIXED
#define ARCTOPK_SMALL_SEL_ROWS_MIXED 4096  // single-block selects beside multi-block items: at most this many rows
#endif
#ifndef ARCTOPK_KEYS_THREADS
#define ARCTOPK_KEYS_THREADS 1024      // multi-block select key pass: block size (256 or 1024)
#endif
#ifndef ARCTOPK_KEYS_BLOCKS
#define ARCTOPK_KEYS_BLOCKS 224        // ... grid target per batch
#endif
#ifndef ARCTOPK_KEYS_MIN_ROWS
#define ARCTOPK_KEYS_MIN_ROWS 4096     // ... rows per block at least
#endif
#ifndef ARCTOPK_FUSE_MAX_ROWS
#define ARCTOPK_FUSE_MAX_ROWS 262144   // largest item whose refine runs in the write blocks
#endif
#ifndef ARCTOPK_ZERO_AHEAD
#define ARCTOPK_ZERO_AHEAD 1           // the backward's last exchange step (EF14 / noef) zeroes its bucket
#endif                                 //   while its packed values are on the wire; its decode then
                                       //   writes the selected rows only (exchange.cpp) ...
#ifndef ARCTOPK_ZERO_AHEAD_MIN_BYTES
#define ARCTOPK_ZERO_AHEAD_MIN_BYTES (64ll << 20)  // ... for buckets of at least this many bytes (a
#endif                                 //   small bucket's decode is short, the memset launch is not)
#ifndef ARCTOPK_FUSE_CAP
#define ARCTOPK_FUSE_CAP 8192         // candidates a fused write block stages in LDS (more: swept from L2)
#endif
#ifndef ARCTOPK_QUAD_DEC_CHUNK
#define ARCTOPK_QUAD_DEC_CHUNK 8192    // short-row (4 <= m < 256) fp32 decode, lane per output quad: elements per chunk
#endif
#ifndef ARCTOPK_TOPK_HIST_BLOCKS
#define ARCTOPK_TOPK_HIST_BLOCKS 1024  // TopK select: histogram blocks per batch
#endif
// Plans:
#ifndef ARCTOPK_ENC_TARGET_BLOCKS
#define ARCTOPK_ENC_TARGET_BLOCKS 2048 // encode blocks a bucket's wave-per-row work aims at
#endif
#ifndef ARCTOPK_PACK_CHUNK
#define ARCTOPK_PACK_CHUNK 8192        // elements per pack chunk (rows >= 256)
#endif
#ifndef ARCTOPK_DEC_CHUNK
#define ARCTOPK_DEC_CHUNK 8192         // elements per decode chunk (rows >= 256)
#endif
#ifndef ARCTOPK_STREAM_PACK_CHUNK
#define ARCTOPK_STREAM_PACK_CHUNK 2048 // elements per m <= 2 stream-pack chunk
#endif
#ifndef ARCTOPK_SHORT_DEC_CHUNK
#define ARCTOPK_SHORT_DEC_CHUNK 4096   // elements per short-row (m < 256) decode chunk
#endif
#ifndef ARCTOPK_SHORT3_CHUNK
#define ARCTOPK_SHORT3_CHUNK 4096      // short-row decode of quad-aligned tensors (mode 3): elements per
#endif                                 // chunk at most (LDS: 4 (m + 1) / m B each)
#ifndef ARCTOPK_ENC_TARGET_BLOCKS_E
#define ARCTOPK_ENC_TARGET_BLOCKS_E 4096  // ... for the fp32 kernels that also stream E (large tensors)
#endif
#ifndef ARCTOPK_ENC_E_MIN_ROWS
#define ARCTOPK_ENC_E_MIN_ROWS 16384   // ... for tensors of at least this many rows
#endif
#ifndef ARCTOPK_ENC_MIN_TILE
#define ARCTOPK_ENC_MIN_TILE 2048      // fewest elements per wave-per-row encode tile
                                       // (A/B: ResNet-18 DDP buckets 292 -> 304 GB/s vs 8192)
#endif
#ifndef ARCTOPK_ENC_UNITS_G_ONLY
#define ARCTOPK_ENC_UNITS_G_ONLY 4     // fp32 encode without E loads: 16-B units per lane per step
#endif
#ifndef ARCTOPK_ENC_UNITS_GE
#define ARCTOPK_ENC_UNITS_GE 4         // fp32 encode with E loads: 16-B units of G (and of E) per lane per step
#endif
#ifndef ARCTOPK_ENC_UNITS_BF16
#define ARCTOPK_ENC_UNITS_BF16 4       // bf16 encode rows: 16-B units per lane per step
#endif

namespace arctopk {

constexpr int kMaxR = 8;           // sketch rank supported by the kernels
constexpr int kTileRows = 256;     // row granule of a small-m encode tile (thread per row)
#ifndef ARCTOPK_SMALL_TILE_BYTES
#define ARCTOPK_SMALL_TILE_BYTES 16384  // 16 KiB: ResNet-18 DDP buckets 228 -> 234 GB/s, large buckets unchanged
#endif
constexpr int kSmallTileBytes = ARCTOPK_SMALL_TILE_BYTES;  // tensor bytes per small-m encode tile
constexpr int kSmallM = 64;        // m below this: thread-per-row tiles; else wave-per-row
constexpr int kVLdsMaxBytes = 64 * 1024;  // V staged in LDS up to this size, else read from L2
constexpr int kChunkElems = 8192;  // target elements per pack/decode work chunk (8192 beat
                                   // 16384 by 3 % on the headline, one 2048-row per wave)
constexpr int kEncTargetBlocks = ARCTOPK_ENC_TARGET_BLOCKS;  // (measured: 2048 beats 1024 on
                                                              // 256 CUs at 3 blocks/CU)
#ifndef ARCTOPK_SMALL_SEL_ROWS
#define ARCTOPK_SMALL_SEL_ROWS 15360
#endif
// rows up to this: one block per segment, keys in LDS (at most 32752: the refine launch
// that also runs these selects has 128 KiB of dynamic LDS; past 48 KiB the 1024-thread
// select kernel gets the attribute).  Measured: a 32000-row segment takes 54 us in one
// block vs 33 us multi-block, so the single block stops at 15360 rows.
constexpr int kSmallSelRows = ARCTOPK_SMALL_SEL_ROWS;

// 32-bit quotient by a runtime divisor: q = mulhi64(x, ceil(2^64/d)) is exact for
// x, d < 2^32 (the fractional error x/2^64 < 1/d never crosses an integer).
struct FastDiv {
    uint64_t magic;
    uint32_t d;
    uint32_t pad;
};

__host__ inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    f.pad = 0;
    f.magic = (d <= 1) ? 0 : (~0ull / d) + 1ull;
    return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv& f) {
    return f.d <= 1 ? x : (uint32_t)__umul64hi((uint64_t)x, f.magic);
}

struct SegDev {
    int64_t offset, n, m, k_rows, sketch_off, v_off, packed_off, row_off, sel_off;
    int32_t kind;
    int32_t vec;       // 1: m % 4 == 0 and offset % 4 == 0 and packed_off % 4 == 0
    FastDiv mdiv;      // division by m
    uint32_t magic32;  // ceil(2^32 / m): exact quotient for x < 2^32 / m (in-tile indices)
    int32_t nparts;    // encode column parts (V slice of each fits in LDS); 1 = unsplit
    int64_t part_off;  // nparts > 1: partial sketches at part_buf[part_off + (p * n + row) * r]
    int32_t dchunk0;      // decode mode 3 (short rows): global index of the segment's first decode
    int32_t dchunk_rows;  // chunk, and rows per chunk (0: the segment has no mode-3 chunks)
    int32_t keyed;        // multi-block select item whose encode can emit its energy keys directly
    int32_t pad_k;        // (at world size 1: the sketch all-reduce is the identity)
};

__device__ __forceinline__ uint32_t div32(uint32_t x, uint32_t magic) { return __umulhi(x, magic); }

// Streaming (nontemporal) 16-B accesses for data touched once per kernel: measured on the
// encode pattern (read G, E; write E; 256 MiB each) 6.5 TB/s with nt loads vs 4.9 TB/s
// plain (scripts/stream_probe.hip).
typedef float v4f_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_stream(const float4* p) {
    const v4f_t v = __builtin_nontemporal_load(reinterpret_cast<const v4f_t*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_stream(float4* p, float4 v) {
    __builtin_nontemporal_store(v4f_t{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f_t*>(p));
}
template <bool NT>
__device__ __forceinline__ float4 ld4(const float4* p) {
    if constexpr (NT) return ld_stream(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(float4* p, float4 v) {
    if constexpr (NT) st_stream(p, v);
    else *p = v;
}
// ---- bucket element types: fp32 and bf16 ---------------------------------------------
// bf16 is stored as its 16 bits; arithmetic happens in fp32 and every value the
// reference rounds to bf16 (each aten op on a bf16 tensor: float compute, then
// round-to-nearest-even, NaN -> 0x7FC0, as c10::BFloat16) is rounded here the same way.
struct bf16_t {
    uint16_t u;
};
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16_t x) { return __uint_as_float((uint32_t)x.u << 16); }
template <typename T> __device__ __forceinline__ T from_f(float f);
template <> __device__ __forceinline__ float from_f<float>(float f) { return f; }
// gfx950 converts two floats to packed bf16 with round-to-nearest-even in one instruction
// (v_cvt_pk_bf16_f32); only NaN needs fixing up to c10's canonical 0x7FC0
typedef float f2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
    uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(f2_t{a, b}, bf2_t));
    if (a != a) u = (u & 0xFFFF0000u) | 0x7FC0u;
    if (b != b) u = (u & 0x0000FFFFu) | 0x7FC00000u;
    return u;
}
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float f) {
    return bf16_t{(uint16_t)(cvt_pk_bf16(f, 0.0f) & 0xFFFFu)};
}
// value after the reference's rounding to T (identity for fp32)
template <typename T> __device__ __forceinline__ float rnd(float f) { return to_f(from_f<T>(f)); }
template <typename T> __device__ __forceinline__ float4 rnd4(float4 v) {
    if constexpr (sizeof(T) == 2) {
        const uint32_t a = cvt_pk_bf16(v.x, v.y), b = cvt_pk_bf16(v.z, v.w);
        return make_float4(__uint_as_float(a << 16), __uint_as_float(a & 0xFFFF0000u),
                           __uint_as_float(b << 16), __uint_as_float(b & 0xFFFF0000u));
    } else {
        return v;
    }
}

// quad I/O: elements 4q .. 4q+3 of p (p 4-element aligned); fp32: 16 B, bf16: 8 B
typedef unsigned int u2_t __attribute__((ext_vector_type(2)));
template <typename T, bool NT> __device__ __forceinline__ float4 ldq(const T* p, int64_t q);
template <> __device__ __forceinline__ float4 ldq<float, false>(const float* p, int64_t q) {
    return reinterpret_cast<const float4*>(p)[q];
}
template <> __device__ __forceinline__ float4 ldq<float, true>(const float* p, int64_t q) {
    return ld_stream(reinterpret_cast<const float4*>(p) + q);
}
__device__ __forceinline__ float4 unpack_bf16x4(u2_t w) {
    return make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xFFFF0000u),
                       __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xFFFF0000u));
}
__device__ __forceinline__ u2_t pack_bf16x4(float4 v) {
    return u2_t{cvt_pk_bf16(v.x, v.y), cvt_pk_bf16(v.z, v.w)};
}
template <> __device__ __forceinline__ float4 ldq<bf16_t, false>(const bf16_t* p, int64_t q) {
    return unpack_bf16x4(reinterpret_cast<const u2_t*>(p)[q]);
}
template <> __device__ __forceinline__ float4 ldq<bf16_t, true>(const bf16_t* p, int64_t q) {
    return unpack_bf16x4(__builtin_nontemporal_load(reinterpret_cast<const u2_t*>(p) + q));
}
template <typename T, bool NT> __device__ __forceinline__ void stq(T* p, int64_t q, float4 v);
template <> __device__ __forceinline__ void stq<float, false>(float* p, int64_t q, float4 v) {
    reinterpret_cast<float4*>(p)[q] = v;
}
template <> __device__ __forceinline__ void stq<float, true>(float* p, int64_t q, float4 v) {
    st_stream(reinterpret_cast<float4*>(p) + q, v);
}
template <> __device__ __forceinline__ void stq<bf16_t, false>(bf16_t* p, int64_t q, float4 v) {
    reinterpret_cast<u2_t*>(p)[q] = pack_bf16x4(v);
}
template <> __device__ __forceinline__ void stq<bf16_t, true>(bf16_t* p, int64_t q, float4 v) {
    __builtin_nontemporal_store(pack_bf16x4(v), reinterpret_cast<u2_t*>(p) + q);
}
// 16-B unit I/O: the quads of 16 bytes at unit c of p (p 16-B aligned): fp32 one quad,
// bf16 two quads (8 elements)
template <typename T> constexpr int kQuadsPer16 = 16 / (4 * (int)sizeof(T));
typedef unsigned int u4_t __attribute__((ext_vector_type(4)));
template <typename T, bool NT>
__device__ __forceinline__ void ld16(const T* p, int64_t c, float4 (&q)[kQuadsPer16<T>]) {
    if constexpr (sizeof(T) == 4) {
        q[0] = ldq<T, NT>(p, c);
    } else {
        const u4_t* w4 = reinterpret_cast<const u4_t*>(p) + c;
        const u4_t w = NT ? __builtin_nontemporal_load(w4) : *w4;
        q[0] = unpack_bf16x4(u2_t{w.x, w.y});
        q[1] = unpack_bf16x4(u2_t{w.z, w.w});
    }
}
// a 16-B unit kept as loaded (4 VGPRs whatever T), unpacked only where it is consumed: holding
// bf16 units unpacked doubled the encode's load registers and spilled them to scratch
template <typename T, bool NT>
__device__ __forceinline__ u4_t ld16raw(const T* p, int64_t c) {
    const u4_t* w4 = reinterpret_cast<const u4_t*>(p) + c;
    return NT ? __builtin_nontemporal_load(w4) : *w4;
}
template <typename T>
__device__ __forceinline__ void unpack16(u4_t w, float4 (&q)[kQuadsPer16<T>]) {
    if constexpr (sizeof(T) == 4) {
        q[0] = make_float4(__uint_as_float(w.x), __uint_as_float(w.y), __uint_as_float(w.z), __uint_as_float(w.w));
    } else {
        q[0] = unpack_bf16x4(u2_t{w.x, w.y});
        q[1] = unpack_bf16x4(u2_t{w.z, w.w});
    }
}
template <typename T, bool NT>
__device__ __forceinline__ void st16(T* p, int64_t c, const float4 (&q)[kQuadsPer16<T>]) {
    if constexpr (sizeof(T) == 4) {
        stq<T, NT>(p, c, q[0]);
    } else {
        const u2_t a = pack_bf16x4(q[0]), b = pack_bf16x4(q[1]);
        const u4_t w = u4_t{a.x, a.y, b.x, b.y};
        u4_t* w4 = reinterpret_cast<u4_t*>(p) + c;
        if constexpr (NT) __builtin_nontemporal_store(w, w4);
        else *w4 = w;
    }
}
// scalar I/O
template <typename T, bool NT = false> __device__ __forceinline__ float ld1(const T* p) {
    if constexpr (NT) {
        if constexpr (sizeof(T) == 4) return __builtin_nontemporal_load(reinterpret_cast<const float*>(p));
        else return to_f(bf16_t{__builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(p))});
    } else {
        return to_f(*p);
    }
}
template <typename T, bool NT = false> __device__ __forceinline__ void st1(T* p, float v) {
    if constexpr (NT) {
        if constexpr (sizeof(T) == 4) __builtin_nontemporal_store(v, reinterpret_cast<float*>(p));
        else __builtin_nontemporal_store(from_f<bf16_t>(v).u, reinterpret_cast<uint16_t*>(p));
    } else {
        *p = from_f<T>(v);
    }
}

// streaming (nontemporal) hints: the pack's E accesses, the decode's output stores, the
// encode's G / E loads and E stores (each measured faster than plain accesses)
constexpr bool kNtPack = true;
constexpr bool kNtDecode = true;
constexpr bool kEncNtLoad = true;
constexpr bool kEncNtStore = true;
constexpr int kSmallTileRows = 1024;  // rows of a small-m pack/decode chunk (LDS slot table)

// encode tile modes
enum : int32_t { ENC_ROW_VEC = 0, ENC_ROW_SCALAR = 1, ENC_TILE = 2, ENC_RAW = 3 };

struct EncTile {
    int32_t seg;
    int32_t mode;
    int64_t row0;      // first row (RAW: first element)
    int64_t nrows;     // rows (RAW: elements)
    int32_t c0, clen;  // row modes: column range (multiple of 4 apart when vectorised)
    int32_t part;      // -1: whole rows -> sketch; else column part -> partial sketch
    int32_t rstride;   // row modes: the tile's rows are row0 + q * rstride, q < nrows
                       // (tiles of a segment interleave, so the blocks in flight stream one
                       // advancing window of the tensor instead of scattered row ranges)
};

struct VDraw {         // one SKETCH tensor's torch.randn(m, r, device=...) draw (vdraw.hip)
    int64_t v_off;     // element offset in the projection buffer
    int64_t numel;     // m * r
    uint64_t stride;   // threads of torch's grid-stride launch: 256 * grid
    uint64_t offset;   // Philox offset at this draw (after the bucket's manual_seed)
};
int vdraw_table(const arctopk_segment* segs, int nseg, int r, int device, VDraw* out, int* nout,
                uint64_t* advance);
constexpr int kVChunk = 1024;  // elements of V per draw block
struct VChunk {        // one draw block's element range [lo, hi) of draw `entry`
    int32_t entry;
    uint32_t lo, hi;
};
struct VDrawJob {      // a projection draw riding in the trailing blocks of another launch
    const VDraw* segs;
    const VChunk* chunks;
    void* V;
    uint64_t seed;
    int32_t n;         // trailing blocks (one chunk each); 0: no draw
};

struct Chunk {         // pack: selected-row range (mode 0) or row range (mode 1); decode: row range
    int32_t seg;
    int32_t mode;      // 1: m in {1, 2}, fp32, 16-B aligned: quad streams over every row;
                       // decode 2: 4 <= m < 256 fp32, lane per output quad;
                       // decode 3: 4 <= m < 256, quad-aligned chunks: the chunk's slot map and
                       //   packed rows staged in LDS, the packed range read from the chunk
                       //   table the pack wrote (d_dfirst), one round trip for the data
    int64_t row0;
    int64_t nrows;
};

}  // namespace arctopk

namespace arctopk { struct MBatch; struct MWorkspace; }

struct arctopk_plan {
    int device;
    int dtype;                    // ARCTOPK_F32 / ARCTOPK_BF16 (bucket element type)
    int r;
    double ratio;
    int nseg;
    arctopk_plan_info info;
    arctopk_segment* h_segs;      // host copy
    arctopk::SegDev* d_segs;
    arctopk::EncTile* d_enc;      // encode tiles (k_encode)
    int n_enc;
    arctopk::EncTile* d_enc_e;    // encode tiles of the fp32 kernels that also stream E (0: use d_enc)
    int n_enc_e;
    int enc_lds_bytes;            // dynamic LDS of the encode launch
    int enc_short;                // no wave-per-row tile in the tables: k_encode_short
    float* d_part;                // partial sketches of column-split segments
    int32_t* d_split;             // ids of column-split segments
    int n_split;
    int64_t split_rows_max;
    arctopk::Chunk* d_pack;
    int n_pack;
    arctopk::Chunk* d_dec;
    int n_dec;
    int32_t* h_pack_begin;        // [nseg + 1]: first pack chunk of each segment
    int32_t* h_dec_begin;         // [nseg + 1]: first decode chunk of each segment
    int dec_lds_bytes;            // dynamic LDS of the decode launch (small-m chunk tiles)
    int32_t* d_dfirst;            // [n_dec + 1]: per decode chunk, the bucket-wide index (sel_off +
                                  // slot) of its first selected row; written by the pack from the
                                  // row list, read by mode-3 decode chunks (and the next entry)
    int32_t* d_dfirst_pub;        // [n_dec + 1]: the same table, derived from the slot map handed to
                                  // the public decode entry points (k_dfirst), never the pack's
    int32_t* d_m3;                // segments with mode-3 decode chunks, and their number
    int n_m3;
    uint32_t* d_keys;             // select workspace: one key per row
    int any_keyed;                // some segment is `keyed` (SegDev)
    int32_t* d_small;             // segments selected by the fused one-block kernel
    int n_small;
    int small_lds;                // bytes of LDS keys for the largest small segment
    int32_t* d_large;             // segments whose keys go through global memory
    int n_large;
    arctopk::MBatch* h_large_batches;   // multi-block select items (host)
    arctopk::MBatch* d_large_batches;   // ... and their device copy (ARC kernels read it there:
                                        // a 3 KiB by-value kernel argument costs ~2 us per launch)
    int n_large_batches;
    arctopk::MWorkspace* d_mws;         // multi-block select workspace
    int64_t mws_cap;                    // its candidate slots
    arctopk::VDraw* d_vdraw;            // device projection draws (vdraw.hip)
    int n_vdraw;
    int64_t vdraw_max;                  // largest m * r
    uint64_t vdraw_advance;             // Philox offset after the bucket's draws
    arctopk::VChunk* d_vchunk;          // the draws cut into kVChunk-element blocks
    int n_vchunk;
    void* b_sketch;                     // buffers bound by arctopk_plan_bind (arctopk_step)
    int32_t* b_rowlist;
    int32_t* b_slotmap;
    void* b_packed;
    void* b_V;
    void* x_ev_packed;                  // exchange step (exchange.cpp): packed values ready,
    void* x_ev_ar;                      // ... and their all-reduce done
    int x_deferred;                     // a decode waits for arctopk_exchange_finish, on:
    void* x_bucket;                     //   the bucket,
    void* x_gerr;                       //   the global residual (EF21),
    int x_ef, x_ws;                     //   the EF mode and world size of that call
    int x_fin;                          // 1: world size 1, EF14 / noef: no pack; the decode is the
                                        //   fused pack + decode from the residual x_err (finalize);
                                        // 3: the bucket is already zero, the decode writes only the
                                        //   selected rows (scatter_chunk)
    int x_pack;                         // its pack is deferred too (world size 1): enqueued in the
    void* x_err;                        //   next call's encode launch, or by exchange_finish; the
                                        //   residual it gathers from
    void* x_ev_dec;                     // completed by an inline decode after a collective
    void* x_stream;                     // the select stream the deferred step's select, pack and
                                        //   decode run on (NULL: the caller's stream)
    void* x_ev_enc;                     // recorded on the caller's stream after the encode (and
                                        //   the sketch all-reduce) when a select stream takes over
    void* x_ev_join;                    // recorded on the select stream after the decode, for the
                                        //   stream that finishes the step to wait on
    // a trailing step (arctopk_exchange_trail): recorded, not enqueued; the next exchange step
    // carries its encode tiles and single-block selects in its own launches
    int x_trail;
    void* x_t_bucket;
    void* x_t_err;
    void* x_t_gerr;
    const void* x_t_V;
    int x_t_ef, x_t_err_in;
    const arctopk_plan* x_carry;        // during an exchange step: the trailing plan its encode and
                                        //   compact launches carry (encode_keyed, launch_select)
};
namespace arctopk {
// keyed: the call's encode ran in keys mode (encode_keyed; world size 1 only)
int select_ride(const arctopk_plan* p, const void* sketch, int32_t ws, int32_t* rowlist, int32_t* slotmap,
                const arctopk_plan* next, uint64_t next_seed, void* next_V, const arctopk_plan* rp,
                int32_t rp_ws, int32_t rp_ef, void* rp_gerr, void* rp_out, int* rode, void* stream,
                bool keyed = false);
int select_draw_keyed(const arctopk_plan* p, const void* sketch, int32_t ws, int32_t* rowlist, int32_t* slotmap,
                      const arctopk_plan* next, uint64_t next_seed, void* next_V, bool keyed, void* stream);
// keyed encode; rp (may be null): a plan whose deferred pack (its bound buffers, bucket rp_grad
// and residual rp_err, the same EF mode and dtype) rides in the launch: *rode = 1 when it did;
// done (may be null): an event the encode's last kernel completes itself (its stop event: no
// marker packet on the stream)
int encode_keyed(const arctopk_plan* p, const void* grad, void* err, int32_t ef, int32_t err_in, const void* V,
                 void* sketch, void* stream, const arctopk_plan* rp = nullptr, const void* rp_grad = nullptr,
                 void* rp_err = nullptr, int* rode = nullptr, void* done = nullptr);
int decode_pair(const arctopk_plan* pa, int32_t ws_a, int32_t ef_a, void* gerr_a, void* out_a,
                const arctopk_plan* pb, int32_t ws_b, int32_t ef_b, void* gerr_b, void* out_b, void* stream,
                void* done);
int pack_signal(const arctopk_plan* p, const void* grad, void* err, int32_t ef, const int32_t* rowlist,
                const int32_t* slotmap, void* packed, void* stream, void* done);
// the decode of the plan's own last pack (its chunk table); `done` (may be null) completed by the kernel
int decode_signal(const arctopk_plan* p, const void* packed, const int32_t* slotmap, int32_t ws, int32_t ef,
                  void* gerr, void* out, void* stream, void* done);
// the watchdog stops looking at a plan's events (arctopk_plan_destroy)
void exchange_forget(arctopk_plan* p);
// the emulated wire communicator (wire.hip): one all-reduce's local cost on an R-rank ring
struct WireParams {
    int32_t ranks;      // ranks of the emulated ring
    double busbw_gbs;   // bus bandwidth it is paced to
    double latency_us;  // fixed cost per all-reduce
    int32_t blocks;     // workgroups (the collective's CU footprint)
};
int wire_allreduce(const WireParams& w, void* buf, int64_t bytes, hipStream_t st, hipEvent_t done);
}
