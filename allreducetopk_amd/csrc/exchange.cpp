// Exchange step: one bucket call of the ARC-TopK hook at world size > 1 (or forced at 1),
// collectives included, enqueued by ONE host call.
//
// The reference blocks on two NCCL all-reduces per bucket (group_topk_hook_no_reshape.py:58
// per tensor, :280 for the packed values).  Here every call is stream-ordered:
//
//   caller's stream   : [draw V] -> encode -> all_reduce(sketch) -> select (+ next V) -> pack
//                       -> decode of the PREVIOUS bucket (after its all-reduce)
//   all-reduce stream : all_reduce(packed)          (waits for the pack kernel's own signal)
//
// so the packed values of bucket b are on the wire while the caller's stream encodes,
// selects and packs bucket b+1; the decode of b then follows on the caller's stream, where
// it does not compete with the next encode for HBM and needs no event of its own.  The last
// bucket of a backward runs inline (its all-reduce and decode on the caller's stream, after
// the previous bucket's decode): nothing is left in flight when the hook returns for it.
//
// Collectives go through an arctopk_comm: an RCCL communicator this library owns (RCCL is
// resolved at run time from the library torch itself loaded, so the process holds one RCCL),
// or a caller-supplied callback (tests drive the same orchestration over gloo).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "common.h"

namespace {

struct Rccl {
    void* handle = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;
std::string g_rccl_path;

// RCCL entry points from `path` (already loaded by torch: dlopen returns that copy)
int rccl_load(const char* path, const Rccl** out) {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl.handle) {
        if (path && *path && g_rccl_path != path) return ARCTOPK_EINVAL;  // one RCCL per process
        *out = &g_rccl;
        return 0;
    }
    const char* p = (path && *path) ? path : "librccl.so.1";
    void* h = dlopen(p, RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen(p, RTLD_NOW);
    if (!h) return ARCTOPK_ENOCOMM;
    Rccl r;
    r.handle = h;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce) {
        dlclose(h);
        return ARCTOPK_ENOCOMM;
    }
    g_rccl = r;
    g_rccl_path = p;
    *out = &g_rccl;
    return 0;
}

// RCCL status -> ABI status (ARCTOPK_ECOMM + ncclResult_t)
int rccl_status(ncclResult_t r) { return r == ncclSuccess ? 0 : ARCTOPK_ECOMM + (int)r; }

}  // namespace

struct arctopk_comm {
    int kind;  // 0: RCCL, 1: callback
    int nranks;
    int rank;
    int device;
    ncclComm_t nccl;
    const Rccl* rccl;
    arctopk_allreduce_fn fn;
    void* ctx;
};

extern "C" int arctopk_comm_unique_id(const char* rccl_path, void* id_out) {
    if (!id_out) return ARCTOPK_EINVAL;
    const Rccl* r = nullptr;
    int e = rccl_load(rccl_path, &r);
    if (e) return e;
    ncclUniqueId id;
    e = rccl_status(r->get_unique_id(&id));
    if (e) return e;
    std::memcpy(id_out, &id, sizeof(id));
    return 0;
}

extern "C" int arctopk_comm_init_rccl(const char* rccl_path, const void* id, int32_t nranks, int32_t rank,
                                      int32_t device, arctopk_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return ARCTOPK_EINVAL;
    *out = nullptr;
    const Rccl* r = nullptr;
    int e = rccl_load(rccl_path, &r);
    if (e) return e;
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess) return (int)he;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t c = nullptr;
    e = rccl_status(r->comm_init_rank(&c, nranks, uid, rank));
    if (e) return e;
    arctopk_comm* m = new (std::nothrow) arctopk_comm;
    if (!m) {
        r->comm_destroy(c);
        return ARCTOPK_EINVAL;
    }
    *m = arctopk_comm{0, nranks, rank, device, c, r, nullptr, nullptr};
    *out = m;
    return 0;
}

extern "C" int arctopk_comm_init_callback(arctopk_allreduce_fn fn, void* ctx, int32_t nranks, int32_t rank,
                                          arctopk_comm** out) {
    if (!fn || !out || nranks < 1 || rank < 0 || rank >= nranks) return ARCTOPK_EINVAL;
    arctopk_comm* m = new (std::nothrow) arctopk_comm;
    if (!m) return ARCTOPK_EINVAL;
    *m = arctopk_comm{1, nranks, rank, -1, nullptr, nullptr, fn, ctx};
    *out = m;
    return 0;
}

extern "C" int arctopk_comm_destroy(arctopk_comm* c) {
    if (!c) return 0;
    int e = 0;
    if (c->kind == 0 && c->nccl) e = rccl_status(c->rccl->comm_destroy(c->nccl));
    delete c;
    return e;
}

extern "C" int arctopk_comm_size(const arctopk_comm* c) { return c ? c->nranks : -ARCTOPK_EINVAL; }

// SUM all-reduce in place, stream-ordered (the reference's dist.all_reduce, :58, :280)
extern "C" int arctopk_comm_allreduce(arctopk_comm* c, void* buf, int64_t count, int32_t dtype, void* stream) {
    if (!c || (!buf && count) || count < 0) return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EDTYPE;
    if (count == 0) return 0;
    if (c->kind == 1) return c->fn(c->ctx, buf, count, dtype, stream);
    return rccl_status(c->rccl->all_reduce(buf, buf, (size_t)count, dtype == ARCTOPK_BF16 ? ncclBfloat16 : ncclFloat32,
                                           ncclSum, c->nccl, (hipStream_t)stream));
}

namespace {

inline int mark(void* const* marks, int i, hipStream_t st) {
    if (!marks || !marks[i]) return 0;
    return (int)hipEventRecord((hipEvent_t)marks[i], st);
}

int ensure_event(void** ev, unsigned flags) {
    if (*ev) return 0;
    hipEvent_t e = nullptr;
    const hipError_t st = hipEventCreateWithFlags(&e, flags);
    if (st != hipSuccess) return (int)st;
    *ev = e;
    return 0;
}

}  // namespace

// The deferred decode of plan p's last exchange step, on `stream`: after that step's packed
// all-reduce (a stream wait only when the host does not already see it complete).
namespace {
int wait_ar(arctopk_plan* p, hipStream_t st) {
    if (p->x_deferred != 1) return 0;  // 2: no all-reduce on another stream
    const hipError_t q = hipEventQuery((hipEvent_t)p->x_ev_ar);
    if (q == hipErrorNotReady) return (int)hipStreamWaitEvent(st, (hipEvent_t)p->x_ev_ar, 0);
    return q == hipSuccess ? 0 : (int)q;
}
}  // namespace

extern "C" int arctopk_exchange_finish(arctopk_plan* p, void* stream, void* const* marks) {
    if (!p) return ARCTOPK_EINVAL;
    if (!p->x_deferred) return 0;
    hipStream_t st = (hipStream_t)stream;
    int e = wait_ar(p, st);
    if (!e) e = mark(marks, ARCTOPK_MARK_PACKED_AR, st);
    if (!e) e = arctopk_decode(p, p->b_packed, p->b_slotmap, p->x_ws, p->x_ef, p->x_gerr, p->x_bucket, stream);
    if (!e) e = mark(marks, ARCTOPK_MARK_DECODE, st);
    if (!e) p->x_deferred = 0;
    return e;
}

extern "C" int arctopk_exchange_step(arctopk_plan* p, void* bucket, void* err, void* gerr, int32_t ef,
                                     int32_t err_in, int32_t draw, uint64_t seed, const arctopk_plan* next,
                                     uint64_t next_seed, arctopk_comm* sketch_comm, arctopk_comm* packed_comm,
                                     void* stream, void* ar_stream, int32_t defer, arctopk_plan* ride,
                                     void* const* ride_marks, arctopk_plan* const* finish,
                                     void* const* const* finish_marks, int32_t nfinish, const void* V,
                                     void* const* marks) {
    if (!p || !bucket || !p->b_sketch || !sketch_comm != !packed_comm || nfinish < 0 || (nfinish && !finish))
        return ARCTOPK_EINVAL;
    if (sketch_comm && sketch_comm->nranks != packed_comm->nranks) return ARCTOPK_EINVAL;
    if (next && (!next->b_sketch || next->dtype != p->dtype || next->device != p->device)) return ARCTOPK_EINVAL;
    // deferring with a collective needs the all-reduce stream (the decode waits for its event)
    if (defer && packed_comm && (!ar_stream || ar_stream == stream)) return ARCTOPK_EINVAL;
    if (ride && (ride == p || !ride->x_deferred)) return ARCTOPK_EINVAL;
    const int ws = packed_comm ? packed_comm->nranks : 1;
    hipStream_t st = (hipStream_t)stream, as = (hipStream_t)ar_stream;
    // this bucket's own deferred decode, if a caller never finished it (the hook always does)
    int e = arctopk_exchange_finish(p, stream, nullptr);
    if (!e) e = mark(marks, ARCTOPK_MARK_START, st);
    if (!V) V = p->b_V;
    if (!e && draw && p->info.v_len > 0) e = arctopk_draw_projections(p, seed, const_cast<void*>(V), stream);
    if (!e) e = mark(marks, ARCTOPK_MARK_DRAW, st);
    if (!e) e = arctopk_encode(p, bucket, err, ef, err_in, V, p->b_sketch, stream);
    if (!e) e = mark(marks, ARCTOPK_MARK_ENCODE, st);
    // one all-reduce for every tensor's sketch (the reference: one per tensor, :33, :58, :88)
    if (!e && sketch_comm) e = arctopk_comm_allreduce(sketch_comm, p->b_sketch, p->info.sketch_len, p->dtype, stream);
    if (!e) e = mark(marks, ARCTOPK_MARK_SKETCH_AR, st);
    if (e) return e;
    // the select, with an earlier bucket's deferred decode riding in the same launch when
    // both fit (the select's latency hides behind the decode's stream)
    int rode = 0;
    if (ride) {
        if ((e = wait_ar(ride, st)) || (e = mark(ride_marks, ARCTOPK_MARK_PACKED_AR, st))) return e;
        e = arctopk::select_ride(p, p->b_sketch, ws, p->b_rowlist, p->b_slotmap, next, next_seed,
                                 next ? next->b_V : nullptr, ride, ride->x_ws, ride->x_ef, ride->x_gerr,
                                 ride->x_bucket, &rode, stream);
        if (!e && rode) {
            ride->x_deferred = 0;
            e = mark(ride_marks, ARCTOPK_MARK_DECODE, st);
        }
        if (!e && !rode) {  // a separate decode launch after the select
            e = arctopk_decode(ride, ride->b_packed, ride->b_slotmap, ride->x_ws, ride->x_ef, ride->x_gerr,
                               ride->x_bucket, stream);
            if (!e) ride->x_deferred = 0;
            if (!e) e = mark(ride_marks, ARCTOPK_MARK_DECODE, st);
        }
    } else {
        e = arctopk_select_draw(p, p->b_sketch, ws, p->b_rowlist, p->b_slotmap, next, next_seed,
                                next ? next->b_V : nullptr, stream);
    }
    if (!e) e = mark(marks, ARCTOPK_MARK_SELECT, st);
    if (e) return e;
    const bool signal = defer && packed_comm;
    if (signal) {
        // the pack kernel completes x_ev_packed itself (no marker packet on the caller's
        // stream, where one idles the GPU several us); the all-reduce stream waits for it
        if ((e = ensure_event(&p->x_ev_packed, 0)) ||
            (e = ensure_event(&p->x_ev_ar, hipEventDisableTiming | hipEventReleaseToDevice)))
            return e;
        e = arctopk::pack_signal(p, bucket, err, ef, p->b_rowlist, p->b_slotmap, p->b_packed, stream,
                                 p->x_ev_packed);
    } else {
        e = arctopk_pack(p, bucket, err, ef, p->b_rowlist, p->b_slotmap, p->b_packed, stream);
    }
    if (!e) e = mark(marks, ARCTOPK_MARK_PACK, st);
    if (e) return e;
    if (signal) {  // the index-free all-reduce of the packed values (:280) on its own stream
        hipError_t he = hipStreamWaitEvent(as, (hipEvent_t)p->x_ev_packed, 0);
        if (he != hipSuccess) return (int)he;
        if ((e = arctopk_comm_allreduce(packed_comm, p->b_packed, p->info.packed_len, p->dtype, as))) return e;
        he = hipEventRecord((hipEvent_t)p->x_ev_ar, as);
        if (he != hipSuccess) return (int)he;
    }
    // earlier buckets' deferred decodes the caller wants done now (in its order)
    for (int32_t i = 0; i < nfinish && !e; ++i)
        if (finish[i] && finish[i] != p) e = arctopk_exchange_finish(finish[i], stream, finish_marks ? finish_marks[i] : nullptr);
    if (e) return e;
    if (defer) {
        p->x_deferred = signal ? 1 : 2;
        p->x_bucket = bucket;
        p->x_gerr = gerr;
        p->x_ef = ef;
        p->x_ws = ws;
        return 0;
    }
    if (packed_comm) e = arctopk_comm_allreduce(packed_comm, p->b_packed, p->info.packed_len, p->dtype, stream);
    if (!e) e = mark(marks, ARCTOPK_MARK_PACKED_AR, st);
    if (!e) e = arctopk_decode(p, p->b_packed, p->b_slotmap, ws, ef, gerr, bucket, stream);
    if (!e) e = mark(marks, ARCTOPK_MARK_DECODE, st);
    return e;
}
