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

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace {

struct Rccl {
    void* handle = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_init_rank_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_finalize)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    ncclResult_t (*get_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    bool nonblocking() const { return comm_init_rank_config && comm_abort && get_async_error; }
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
    r.comm_init_rank_config =
        reinterpret_cast<decltype(r.comm_init_rank_config)>(dlsym(h, "ncclCommInitRankConfig"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.comm_finalize = reinterpret_cast<decltype(r.comm_finalize)>(dlsym(h, "ncclCommFinalize"));
    r.comm_abort = reinterpret_cast<decltype(r.comm_abort)>(dlsym(h, "ncclCommAbort"));
    r.get_async_error = reinterpret_cast<decltype(r.get_async_error)>(dlsym(h, "ncclCommGetAsyncError"));
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

int64_t now_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// the caller's current device, restored on every return path
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace

struct arctopk_comm {
    enum Kind { RCCL = 0, CALLBACK = 1, WIRE = 2 };
    int kind = RCCL;
    int nranks = 1;
    int rank = 0;
    int device = -1;
    ncclComm_t nccl = nullptr;           // RCCL: null once aborted
    const Rccl* rccl = nullptr;
    bool nonblocking = false;
    arctopk_allreduce_fn fn = nullptr;   // callback
    void* ctx = nullptr;
    int64_t timeout_ms = 0;              // RCCL: watchdog deadline (0: no watchdog)
    std::atomic<int> err{0};             // sticky failure status
    std::mutex mu;                       // RCCL calls of the caller vs the watchdog's abort
    arctopk::WireParams wire{};          // WIRE
    // WIRE: the communicator's operations run one after another whatever stream they are issued
    // on, as RCCL serialises the collectives of one communicator: each emulated all-reduce
    // completes wire_ev (its kernel's own completion signal), and one issued on another stream
    // than the previous first waits for it
    hipEvent_t wire_ev = nullptr;
    hipStream_t wire_last = nullptr;
    bool wire_used = false;
};

namespace {

// Abort one RCCL communicator (caller holds c->mu), leaving `status` sticky.
void abort_locked(arctopk_comm* c, int status) {
    int expected = 0;
    c->err.compare_exchange_strong(expected, status);
    if (c->kind == arctopk_comm::RCCL && c->nccl) {
        if (c->rccl->comm_abort) (void)c->rccl->comm_abort(c->nccl);
        else (void)c->rccl->comm_destroy(c->nccl);  // (no abort entry point: best effort)
        c->nccl = nullptr;
    }
}

// Watchdog: the library's RCCL communicators created with a timeout, and the completion
// events of the collectives the exchange step enqueued on them (each keyed by its event,
// re-armed when the event is recorded again).  Polls every kPollMs.
class Watchdog {
  public:
    static Watchdog& get() {
        static Watchdog w;
        return w;
    }
    void add(arctopk_comm* c) {
        std::lock_guard<std::mutex> lk(mu_);
        comms_.push_back(c);
        if (!th_.joinable()) th_ = std::thread([this] { loop(); });
    }
    void remove(arctopk_comm* c) {
        std::lock_guard<std::mutex> lk(mu_);
        comms_.erase(std::remove(comms_.begin(), comms_.end(), c), comms_.end());
        items_.erase(std::remove_if(items_.begin(), items_.end(), [c](const Item& i) { return i.c == c; }),
                     items_.end());
    }
    // the collective of `c` ordered before event `ev` (just recorded) must complete in time
    void watch(arctopk_comm* c, void* ev) {
        if (!c || c->kind != arctopk_comm::RCCL || c->timeout_ms <= 0 || !ev) return;
        const int64_t t = now_ms();
        std::lock_guard<std::mutex> lk(mu_);
        for (Item& i : items_)
            if (i.ev == ev) {
                i.c = c;
                i.t = t;
                return;
            }
        items_.push_back(Item{c, ev, t});
    }
    void forget_event(void* ev) {
        if (!ev) return;
        std::lock_guard<std::mutex> lk(mu_);
        items_.erase(std::remove_if(items_.begin(), items_.end(), [ev](const Item& i) { return i.ev == ev; }),
                     items_.end());
    }
    // abort every RCCL communicator of the library (a failed peer breaks all of them)
    void fail_all(int status) {
        std::lock_guard<std::mutex> lk(mu_);
        fail_all_locked(status);
    }
    ~Watchdog() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        if (th_.joinable()) th_.join();
    }

  private:
    struct Item {
        arctopk_comm* c;
        void* ev;
        int64_t t;
    };
    static constexpr int kPollMs = 20;
    void fail_all_locked(int status) {
        for (arctopk_comm* c : comms_) {
            std::lock_guard<std::mutex> lc(c->mu);
            abort_locked(c, status);
        }
        items_.clear();
    }
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        while (!stop_) {
            cv_.wait_for(lk, std::chrono::milliseconds(kPollMs));
            if (stop_) break;
            int fail = 0;
            for (arctopk_comm* c : comms_) {
                std::lock_guard<std::mutex> lc(c->mu);
                if (c->err.load() || !c->nccl) continue;
                ncclResult_t st = ncclSuccess;
                if (c->rccl->get_async_error && c->rccl->get_async_error(c->nccl, &st) == ncclSuccess &&
                    st != ncclSuccess && st != ncclInProgress) {
                    fail = rccl_status(st);
                    break;
                }
            }
            const int64_t t = now_ms();
            for (size_t i = 0; !fail && i < items_.size();) {
                const hipError_t q = hipEventQuery((hipEvent_t)items_[i].ev);
                if (q == hipErrorNotReady) {
                    if (t - items_[i].t > items_[i].c->timeout_ms) fail = ARCTOPK_ETIMEOUT;
                    ++i;
                } else {  // complete (or no longer a valid record): nothing to watch
                    items_[i] = items_.back();
                    items_.pop_back();
                }
            }
            if (fail) {
                if (teardown_on_failure()) {
                    // as ProcessGroupNCCL's async error handling: work queued behind the failed
                    // collective (decode, copy-back, optimizer step) would run on partially
                    // reduced buffers once the aborted kernels exit, so the process ends here,
                    // before any abort (ncclCommAbort may wait for the device; exiting releases
                    // the communicators and the peers' own watchdogs see this rank gone)
                    std::fprintf(stderr,
                                 "[arctopk] exchange watchdog: a collective failed or stayed pending past the "
                                 "timeout (status %d); ending the process so that no partially reduced "
                                 "update is applied (ARCTOPK_ASYNC_ERROR_HANDLING=0 or 2: abort the "
                                 "communicators and raise from the hook instead)\n",
                                 fail);
                    std::fflush(stderr);
                    std::_Exit(1);
                }
                fail_all_locked(fail);
            }
        }
    }
    // ARCTOPK_ASYNC_ERROR_HANDLING, else TORCH_NCCL_ASYNC_ERROR_HANDLING, with torch's meaning:
    // 1 / 3 (torch's default): tear the process down; 0 / 2: abort the communicators only
    static bool teardown_on_failure() {
        const char* v = std::getenv("ARCTOPK_ASYNC_ERROR_HANDLING");
        if (!v || !*v) v = std::getenv("TORCH_NCCL_ASYNC_ERROR_HANDLING");
        if (!v || !*v) return true;
        return v[0] == '1' || v[0] == '3';
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<arctopk_comm*> comms_;
    std::vector<Item> items_;
    std::thread th_;
    bool stop_ = false;
};

// a communicator's sticky failure, if any (checked before any work is enqueued on it)
inline int comm_failed(const arctopk_comm* c) { return c ? c->err.load() : 0; }

}  // namespace

namespace arctopk {
void exchange_forget(arctopk_plan* p) {
    if (!p) return;
    Watchdog::get().forget_event(p->x_ev_packed);
    Watchdog::get().forget_event(p->x_ev_ar);
    Watchdog::get().forget_event(p->x_ev_dec);
}
}  // namespace arctopk

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

extern "C" int arctopk_comm_init_rccl_timeout(const char* rccl_path, const void* id, int32_t nranks,
                                              int32_t rank, int32_t device, int64_t timeout_ms,
                                              arctopk_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks || timeout_ms < 0) return ARCTOPK_EINVAL;
    *out = nullptr;
    const Rccl* r = nullptr;
    int e = rccl_load(rccl_path, &r);
    if (e) return e;
    DeviceGuard dg(device);
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != device) return (int)hipErrorInvalidDevice;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t c = nullptr;
    const bool nb = timeout_ms > 0 && r->nonblocking();
    if (nb) {
        // non-blocking creation, polled against the deadline: a rank that never joins makes
        // this fail with ARCTOPK_ETIMEOUT instead of blocking forever
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        ncclResult_t st = r->comm_init_rank_config(&c, nranks, uid, rank, &cfg);
        const int64_t t0 = now_ms();
        while (st == ncclInProgress || (st == ncclSuccess && c)) {
            ncclResult_t a = ncclSuccess;
            if (r->get_async_error(c, &a) != ncclSuccess) {
                st = ncclInternalError;
                break;
            }
            if (a != ncclInProgress) {
                st = a;
                break;
            }
            if (now_ms() - t0 > timeout_ms) {
                (void)r->comm_abort(c);
                return ARCTOPK_ETIMEOUT;
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        if (st != ncclSuccess) {
            if (c) (void)r->comm_abort(c);
            return rccl_status(st);
        }
    } else {
        e = rccl_status(r->comm_init_rank(&c, nranks, uid, rank));
        if (e) return e;
    }
    arctopk_comm* m = new (std::nothrow) arctopk_comm;
    if (!m) {
        (void)(r->comm_abort ? r->comm_abort(c) : r->comm_destroy(c));
        return ARCTOPK_EINVAL;
    }
    m->kind = arctopk_comm::RCCL;
    m->nranks = nranks;
    m->rank = rank;
    m->device = device;
    m->nccl = c;
    m->rccl = r;
    m->nonblocking = nb;
    m->timeout_ms = nb ? timeout_ms : 0;
    if (m->timeout_ms > 0) Watchdog::get().add(m);
    *out = m;
    return 0;
}

extern "C" int arctopk_comm_init_rccl(const char* rccl_path, const void* id, int32_t nranks, int32_t rank,
                                      int32_t device, arctopk_comm** out) {
    return arctopk_comm_init_rccl_timeout(rccl_path, id, nranks, rank, device, 0, out);
}

extern "C" int arctopk_comm_init_callback(arctopk_allreduce_fn fn, void* ctx, int32_t nranks, int32_t rank,
                                          arctopk_comm** out) {
    if (!fn || !out || nranks < 1 || rank < 0 || rank >= nranks) return ARCTOPK_EINVAL;
    arctopk_comm* m = new (std::nothrow) arctopk_comm;
    if (!m) return ARCTOPK_EINVAL;
    m->kind = arctopk_comm::CALLBACK;
    m->nranks = nranks;
    m->rank = rank;
    m->fn = fn;
    m->ctx = ctx;
    *out = m;
    return 0;
}

extern "C" int arctopk_comm_init_wire(int32_t emul_ranks, double busbw_gbs, double latency_us, int32_t blocks,
                                      int32_t device, arctopk_comm** out) {
    if (!out || emul_ranks < 1 || !(busbw_gbs > 0.0) || latency_us < 0.0 || blocks < 1 || blocks > 1024)
        return ARCTOPK_EINVAL;
    arctopk_comm* m = new (std::nothrow) arctopk_comm;
    if (!m) return ARCTOPK_EINVAL;
    m->kind = arctopk_comm::WIRE;
    m->nranks = 1;  // results of a one-rank all-reduce; the wire's cost of emul_ranks
    m->device = device;
    m->wire = arctopk::WireParams{emul_ranks, busbw_gbs, latency_us, blocks};
    *out = m;
    return 0;
}

extern "C" int arctopk_comm_status(const arctopk_comm* c) { return c ? c->err.load() : ARCTOPK_EINVAL; }

extern "C" int arctopk_comm_abort(arctopk_comm* c) {
    if (!c) return ARCTOPK_EINVAL;
    std::lock_guard<std::mutex> lc(c->mu);
    abort_locked(c, ARCTOPK_EABORTED);
    return 0;
}

extern "C" int arctopk_comm_destroy(arctopk_comm* c) {
    if (!c) return 0;
    int e = 0;
    if (c->kind == arctopk_comm::RCCL) {
        if (c->timeout_ms > 0) Watchdog::get().remove(c);
        std::lock_guard<std::mutex> lc(c->mu);
        if (c->nccl) {
            const Rccl* R = c->rccl;
            // a non-blocking communicator is finalized first and polled until its pending
            // operations have flushed (bounded by its timeout: past it, abort), then destroyed
            if (c->nonblocking && R->comm_finalize) {
                ncclResult_t st = R->comm_finalize(c->nccl);
                const int64_t t_end = now_ms() + (c->timeout_ms > 0 ? c->timeout_ms : 60000);
                while (st == ncclInProgress || st == ncclSuccess) {
                    ncclResult_t a = ncclSuccess;
                    if (R->get_async_error(c->nccl, &a) != ncclSuccess) a = ncclInternalError;
                    if (a != ncclInProgress) {
                        st = a;
                        break;
                    }
                    if (now_ms() > t_end) {
                        st = ncclInProgress;
                        break;
                    }
                    std::this_thread::sleep_for(std::chrono::milliseconds(1));
                }
                if (st != ncclSuccess) {
                    (void)R->comm_abort(c->nccl);
                    c->nccl = nullptr;
                    e = st == ncclInProgress ? ARCTOPK_ETIMEOUT : rccl_status(st);
                }
            }
            if (c->nccl) {
                const ncclResult_t r = R->comm_destroy(c->nccl);
                e = (r == ncclInProgress) ? 0 : rccl_status(r);
                c->nccl = nullptr;
            }
        }
    }
    if (c->wire_ev) (void)hipEventDestroy(c->wire_ev);
    delete c;
    return e;
}

extern "C" int arctopk_comm_size(const arctopk_comm* c) { return c ? c->nranks : -ARCTOPK_EINVAL; }

// SUM all-reduce in place, stream-ordered (the reference's dist.all_reduce, :58, :280)
extern "C" int arctopk_comm_allreduce(arctopk_comm* c, void* buf, int64_t count, int32_t dtype, void* stream) {
    if (!c || (!buf && count) || count < 0) return ARCTOPK_EINVAL;
    if (dtype != ARCTOPK_F32 && dtype != ARCTOPK_BF16) return ARCTOPK_EDTYPE;
    if (int f = comm_failed(c)) return f;
    if (count == 0) return 0;
    if (c->kind == arctopk_comm::CALLBACK) return c->fn(c->ctx, buf, count, dtype, stream);
    if (c->kind == arctopk_comm::WIRE) {
        std::lock_guard<std::mutex> lc(c->mu);
        hipStream_t st = (hipStream_t)stream;
        if (!c->wire_ev) {
            const hipError_t he = hipEventCreateWithFlags(&c->wire_ev, hipEventDisableTiming);
            if (he != hipSuccess) return (int)he;
        }
        if (c->wire_used && c->wire_last != st) {
            const hipError_t he = hipStreamWaitEvent(st, c->wire_ev, 0);
            if (he != hipSuccess) return (int)he;
        }
        const int e = arctopk::wire_allreduce(c->wire, buf, count * (dtype == ARCTOPK_BF16 ? 2 : 4), st, c->wire_ev);
        if (!e) {
            c->wire_last = st;
            c->wire_used = true;
        }
        return e;
    }
    std::unique_lock<std::mutex> lc(c->mu);
    if (!c->nccl) return c->err.load() ? c->err.load() : ARCTOPK_EABORTED;
    ncclResult_t r = c->rccl->all_reduce(buf, buf, (size_t)count, dtype == ARCTOPK_BF16 ? ncclBfloat16 : ncclFloat32,
                                         ncclSum, c->nccl, (hipStream_t)stream);
    if (r == ncclInProgress && c->nonblocking) {
        // non-blocking communicator: the call returns while RCCL still sets up (its first
        // collective connects the ranks); wait for that on the host, against the deadline
        const int64_t t0 = now_ms();
        for (;;) {
            ncclResult_t a = ncclSuccess;
            if (c->rccl->get_async_error(c->nccl, &a) != ncclSuccess) a = ncclInternalError;
            if (a != ncclInProgress) {
                r = a;
                break;
            }
            if (now_ms() - t0 > c->timeout_ms) {
                lc.unlock();
                Watchdog::get().fail_all(ARCTOPK_ETIMEOUT);
                return ARCTOPK_ETIMEOUT;
            }
            lc.unlock();
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
            lc.lock();
            if (!c->nccl) return c->err.load() ? c->err.load() : ARCTOPK_EABORTED;
        }
    }
    if (r != ncclSuccess) {
        const int st = rccl_status(r);
        lc.unlock();
        if (c->timeout_ms > 0) Watchdog::get().fail_all(st);
        return st;
    }
    return 0;
}


namespace {

// Diagnostics: host time of the exchange step's parts (ARCTOPK_HOST_TIMING=1 in the
// environment at the first step; read and reset by arctopk_diag_host_times)
constexpr int kHtParts = 8;  // entry, encode, sketch all-reduce, select, pack, packed all-reduce, finish, decode
std::atomic<int64_t> g_ht_ns[kHtParts];
std::atomic<int64_t> g_ht_calls{0};
bool ht_on() {
    static const bool on = [] {
        const char* e = std::getenv("ARCTOPK_HOST_TIMING");
        return e && e[0] == '1';
    }();
    return on;
}
struct HostTimer {
    bool on = ht_on();
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(int part) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        g_ht_ns[part].fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(n - t).count(),
                                std::memory_order_relaxed);
        t = n;
    }
};

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

namespace {
// a deferred pack (world size 1) that no encode launch took: its own launch
int pack_now(arctopk_plan* p, void* stream) {
    if (!p->x_pack) return 0;
    const int e = arctopk_pack(p, p->x_bucket, p->x_err, p->x_ef, p->b_rowlist, p->b_slotmap, p->b_packed, stream);
    if (!e) p->x_pack = 0;
    return e;
}
}  // namespace

namespace {
// `to` waits for everything enqueued on `from` so far (plan p's join event)
int join_stream(arctopk_plan* p, hipStream_t from, hipStream_t to) {
    if (from == to) return 0;
    if (int e = ensure_event(&p->x_ev_join, hipEventDisableTiming | hipEventReleaseToDevice)) return e;
    hipError_t he = hipEventRecord((hipEvent_t)p->x_ev_join, from);
    if (he == hipSuccess) he = hipStreamWaitEvent(to, (hipEvent_t)p->x_ev_join, 0);
    return (int)he;
}
// the stream a deferred step's remaining work goes on: its select stream, else the caller's
inline hipStream_t x_stream_of(const arctopk_plan* p, hipStream_t caller) {
    return p->x_stream ? (hipStream_t)p->x_stream : caller;
}
}  // namespace

namespace {
// a trailing step enqueued on its own (no step carried it): encode + select on `st`, then a
// deferred world-size-1 step like any other (its decode: the fused finalize, x_fin 1)
int trail_run(arctopk_plan* c, hipStream_t st) {
    const void* V = c->x_t_V ? c->x_t_V : c->b_V;
    int e = arctopk::encode_keyed(c, c->x_t_bucket, c->x_t_err, c->x_t_ef, c->x_t_err_in, V, c->b_sketch, st);
    if (!e) e = arctopk::select_draw_keyed(c, c->b_sketch, 1, c->b_rowlist, c->b_slotmap, nullptr, 0, nullptr, true, st);
    if (e) return e;
    c->x_trail = 0;
    c->x_deferred = 2;
    c->x_fin = 1;
    c->x_bucket = c->x_t_bucket;
    c->x_err = c->x_t_err;
    c->x_gerr = c->x_t_gerr;
    c->x_ef = c->x_t_ef;
    c->x_ws = 1;
    c->x_stream = nullptr;
    return 0;
}
}  // namespace

extern "C" int arctopk_exchange_trail(arctopk_plan* p, void* bucket, void* err, void* gerr, int32_t ef,
                                      int32_t err_in, int32_t draw, uint64_t seed, const void* V, void* stream) {
    if (!p || !bucket || !p->b_sketch || (ef != ARCTOPK_EF_NONE && ef != ARCTOPK_EF14)) return ARCTOPK_EINVAL;
    // only a plan another step's launches can carry: single-block selects, short-row / 1-D tiles
    if (p->n_large_batches > 0 || p->n_small == 0 || p->n_split || p->any_keyed)
        return ARCTOPK_EINVAL;
    if (ef == ARCTOPK_EF14 && !err) return ARCTOPK_EINVAL;
    if (p->x_trail || p->x_deferred) return ARCTOPK_EINVAL;  // the caller finishes a plan's step first
    if (!V) V = p->b_V;
    if (draw && p->info.v_len > 0) {
        if (int e = arctopk_draw_projections(p, seed, const_cast<void*>(V), stream)) return e;
    }
    p->x_trail = 1;
    p->x_t_bucket = bucket;
    p->x_t_err = err;
    p->x_t_gerr = gerr;
    p->x_t_V = V;
    p->x_t_ef = ef;
    p->x_t_err_in = err_in;
    return 0;
}

extern "C" int arctopk_exchange_finish(arctopk_plan* p, void* stream, void* const* marks) {
    if (!p) return ARCTOPK_EINVAL;
    if (p->x_trail) {
        if (int e = trail_run(p, (hipStream_t)stream)) return e;
    }
    if (!p->x_deferred) return 0;
    hipStream_t cs = (hipStream_t)stream;
    // where the step's select and pack ran (its select stream, or the caller's); `stream` then
    // waits for the decode
    hipStream_t st = x_stream_of(p, cs);
    int e = pack_now(p, st);
    if (!e) e = wait_ar(p, st);
    if (!e) e = mark(marks, ARCTOPK_MARK_PACKED_AR, st);
    if (!e) e = arctopk::decode_signal(p, p->b_packed, p->b_slotmap, p->x_ws, p->x_ef, p->x_gerr, p->x_bucket, st, nullptr);
    if (!e) e = mark(marks, ARCTOPK_MARK_DECODE, st);
    if (!e) e = join_stream(p, st, cs);
    if (!e) {
        p->x_deferred = p->x_fin = 0;
        p->x_stream = nullptr;
    }
    return e;
}

extern "C" int arctopk_exchange_step(arctopk_plan* p, void* bucket, void* err, void* gerr, int32_t ef,
                                     int32_t err_in, int32_t draw, uint64_t seed, const arctopk_plan* next,
                                     uint64_t next_seed, arctopk_comm* sketch_comm, arctopk_comm* packed_comm,
                                     void* stream, void* ar_stream, int32_t defer, arctopk_plan* ride,
                                     void* const* ride_marks, arctopk_plan* const* finish,
                                     void* const* const* finish_marks, int32_t nfinish, const void* V,
                                     void* const* marks, void* sel_stream, arctopk_plan* trail) {
    if (!p || !bucket || !p->b_sketch || !sketch_comm != !packed_comm || nfinish < 0 || (nfinish && !finish))
        return ARCTOPK_EINVAL;
    if (trail && (trail == p || !trail->x_trail)) return ARCTOPK_EINVAL;
    // a select stream takes the select, pack and decodes off the caller's stream (not with markers:
    // the marker pass times the phases in one stream's order); its packed all-reduce must then go
    // on the all-reduce stream (a communicator's collectives stay on one stream each), and it draws
    // no projections for the next call (that call's encode on the caller's stream would wait for it)
    const bool side = sel_stream && sel_stream != stream && !marks;
    if (side && ((packed_comm && (!ar_stream || ar_stream == stream || ar_stream == sel_stream)) || next))
        return ARCTOPK_EINVAL;
    if (sketch_comm && sketch_comm->nranks != packed_comm->nranks) return ARCTOPK_EINVAL;
    if (next && (!next->b_sketch || next->dtype != p->dtype || next->device != p->device)) return ARCTOPK_EINVAL;
    // deferring with a collective needs the all-reduce stream (the decode waits for its event)
    if (defer && packed_comm && (!ar_stream || ar_stream == stream)) return ARCTOPK_EINVAL;
    if (ride && (ride == p || !ride->x_deferred)) return ARCTOPK_EINVAL;
    // a communicator that failed (watchdog timeout, RCCL error, abort) takes no more work
    if (int f = comm_failed(sketch_comm)) return f;
    if (int f = comm_failed(packed_comm)) return f;
    const int ws = packed_comm ? packed_comm->nranks : 1;
    hipStream_t st = (hipStream_t)stream, as = (hipStream_t)ar_stream;
    hipStream_t ss = side ? (hipStream_t)sel_stream : st;  // the select, pack and decodes
    HostTimer ht;
    if (ht.on) g_ht_calls.fetch_add(1, std::memory_order_relaxed);
    // this bucket's own deferred decode, if a caller never finished it (the hook always does)
    int e = arctopk_exchange_finish(p, stream, nullptr);
    // the trailing step: carried by this step's encode and compact launches when both plans
    // qualify, else enqueued on its own now
    arctopk_plan* carry = nullptr;
    if (!e && trail) {
        constexpr int64_t big_rows = ARCTOPK_SEL_BIG_ROWS;
        const bool fits = !sketch_comm && !marks && trail->device == p->device && trail->dtype == p->dtype &&
                          trail->r == p->r && p->r == 4 && trail->x_t_ef == ef && trail->x_t_err_in == err_in &&
                          ef != ARCTOPK_EF21 && p->n_large_batches > 0 && p->n_split == 0 &&
                          trail->n_large_batches == 0 && trail->n_small > 0 &&
                          trail->n_split == 0 && !trail->any_keyed && trail->small_lds <= big_rows * 4 + 16 &&
                          trail->small_lds <= 48 * 1024 && trail->x_t_bucket != bucket &&
                          (!err || trail->x_t_err != err);
        if (fits) carry = trail;
        else e = trail_run(trail, st);
    }
    p->x_carry = carry;
    struct CarryReset {  // no early return leaves the carry set on the plan
        arctopk_plan* p;
        ~CarryReset() { p->x_carry = nullptr; }
    } carry_reset{p};
    // a step with markers times its own encode: the ride's deferred pack goes first, unmarked
    if (!e && marks && ride) e = pack_now(ride, stream);
    if (!e) e = mark(marks, ARCTOPK_MARK_START, st);
    if (!V) V = p->b_V;
    if (!e && draw && p->info.v_len > 0) e = arctopk_draw_projections(p, seed, const_cast<void*>(V), stream);
    if (!e) e = mark(marks, ARCTOPK_MARK_DRAW, st);
    ht.lap(0);
    // world size 1 (no communicators): the sketch is not all-reduced, so the multi-block select
    // items' encode writes their energy keys directly (keys mode)
    const bool keyed = !sketch_comm;
    // with a select stream at world size 1 the encode's last kernel completes x_ev_enc itself (its
    // stop event), so the caller's stream carries no marker packet; with collectives the event
    // follows the sketch all-reduce (a marker after it, below)
    void* enc_done = nullptr;
    if (!e && side && keyed) {
        if ((e = ensure_event(&p->x_ev_enc, 0))) return e;
        enc_done = p->x_ev_enc;
    }
    // the ride's deferred pack (world size 1) runs as the first blocks of this encode launch when
    // it can: same EF mode and dtype, other buffers (a bucket hooked twice in a row reads the
    // residual the pack rewrites: then the pack goes first, in its own launch)
    if (!e && ride && ride->x_pack) {
        const bool fits = keyed && ride->x_ef == ef && ride->dtype == p->dtype && ride->x_bucket != bucket &&
                          (!err || ride->x_err != err);
        int prode = 0;
        if (fits) {
            e = arctopk::encode_keyed(p, bucket, err, ef, err_in, V, p->b_sketch, stream, ride, ride->x_bucket,
                                      ride->x_err, &prode, enc_done);
            if (!e && prode) ride->x_pack = 0;
            if (!e) e = pack_now(ride, stream);  // (not taken: nothing of this call's touches it)
        } else {
            e = pack_now(ride, stream);
            if (!e) e = keyed ? arctopk::encode_keyed(p, bucket, err, ef, err_in, V, p->b_sketch, stream, nullptr,
                                                      nullptr, nullptr, nullptr, enc_done)
                              : arctopk_encode(p, bucket, err, ef, err_in, V, p->b_sketch, stream);
        }
    } else if (!e) {
        e = keyed ? arctopk::encode_keyed(p, bucket, err, ef, err_in, V, p->b_sketch, stream, nullptr, nullptr,
                                          nullptr, nullptr, enc_done)
                  : arctopk_encode(p, bucket, err, ef, err_in, V, p->b_sketch, stream);
    }
    if (!e) e = mark(marks, ARCTOPK_MARK_ENCODE, st);
    ht.lap(1);
    // one all-reduce for every tensor's sketch (the reference: one per tensor, :33, :58, :88)
    if (!e && sketch_comm) e = arctopk_comm_allreduce(sketch_comm, p->b_sketch, p->info.sketch_len, p->dtype, stream);
    if (!e) e = mark(marks, ARCTOPK_MARK_SKETCH_AR, st);
    if (e) return e;
    // The select stream takes over after the encode and the sketch all-reduce: the latency-bound
    // select chain (and the decode riding in it) overlaps the caller's next encode instead of
    // delaying it (select streams)
    if (side) {
        hipError_t he = hipSuccess;
        if (!enc_done) {  // (with collectives: after the sketch all-reduce)
            if ((e = ensure_event(&p->x_ev_enc, 0))) return e;
            he = hipEventRecord((hipEvent_t)p->x_ev_enc, st);
        }
        if (he == hipSuccess) he = hipStreamWaitEvent(ss, (hipEvent_t)p->x_ev_enc, 0);
        if (he != hipSuccess) return (int)he;
    }
    ht.lap(2);
    // a ride whose step ran on another select stream is not ordered before this one: finished on
    // its own stream instead (the caller's stream then waits for it)
    if (ride && ride->x_stream && ride->x_stream != (void*)ss) {
        if ((e = arctopk_exchange_finish(ride, stream, ride_marks))) return e;
        ride = nullptr;
    }
    // the select, with an earlier bucket's deferred decode riding in the same launch when
    // both fit (the select's latency hides behind the decode's stream)
    int rode = 0;
    if (ride) {
        if ((e = wait_ar(ride, ss)) || (e = mark(ride_marks, ARCTOPK_MARK_PACKED_AR, ss))) return e;
        e = arctopk::select_ride(p, p->b_sketch, ws, p->b_rowlist, p->b_slotmap, next, next_seed,
                                 next ? next->b_V : nullptr, ride, ride->x_ws, ride->x_ef, ride->x_gerr,
                                 ride->x_bucket, &rode, ss, keyed);
        if (!e && rode) {
            ride->x_deferred = ride->x_fin = 0;
            ride->x_stream = nullptr;
            e = mark(ride_marks, ARCTOPK_MARK_DECODE, ss);
        }
        if (!e && !rode) {  // a separate decode launch after the select
            e = arctopk::decode_signal(ride, ride->b_packed, ride->b_slotmap, ride->x_ws, ride->x_ef, ride->x_gerr,
                                       ride->x_bucket, ss, nullptr);
            if (!e) {
                ride->x_deferred = ride->x_fin = 0;
                ride->x_stream = nullptr;
            }
            if (!e) e = mark(ride_marks, ARCTOPK_MARK_DECODE, ss);
        }
    } else {
        e = arctopk::select_draw_keyed(p, p->b_sketch, ws, p->b_rowlist, p->b_slotmap, next, next_seed,
                                       next ? next->b_V : nullptr, keyed, ss);
    }
    p->x_carry = nullptr;
    if (!e && carry) {  // the trailing step was encoded and selected in this step's launches
        carry->x_trail = 0;
        carry->x_deferred = 2;
        carry->x_fin = 1;
        carry->x_bucket = carry->x_t_bucket;
        carry->x_err = carry->x_t_err;
        carry->x_gerr = carry->x_t_gerr;
        carry->x_ef = carry->x_t_ef;
        carry->x_ws = 1;
        carry->x_stream = side ? (void*)ss : nullptr;
    }
    if (!e) e = mark(marks, ARCTOPK_MARK_SELECT, st);
    if (e) return e;
    ht.lap(3);
    // with collectives the pack kernel completes x_ev_packed itself (no marker packet on the
    // caller's stream, where one idles the GPU several us): the all-reduce stream waits for it,
    // and the watchdog sees the sketch all-reduce before it complete
    // the packed all-reduce goes on the all-reduce stream whenever the caller gave one: a
    // deferred step's, and the backward's last step's too (its decode then waits for it on the
    // caller's stream, while the earlier steps' decodes run beside it on the wire); inline only
    // without that stream or with markers (the marker pass times the phases in stream order)
    const bool async_ar = packed_comm && ar_stream && ar_stream != stream && (defer || !marks);
    if (packed_comm) {
        if ((e = ensure_event(&p->x_ev_packed, 0)) ||
            (e = ensure_event(&p->x_ev_ar, hipEventDisableTiming | hipEventReleaseToDevice)))
            return e;
        e = arctopk::pack_signal(p, bucket, err, ef, p->b_rowlist, p->b_slotmap, p->b_packed, ss,
                                 p->x_ev_packed);
        if (!e) Watchdog::get().watch(sketch_comm, p->x_ev_packed);
        // The backward's last step: its decode comes after its own packed all-reduce, the end of
        // the wire's work.  EF14 / noef: the bucket is dead once packed (EF14 packs the residual,
        // noef the bucket itself, both read by the pack before this), so it is zeroed now, while
        // the packed values are on the wire, and the decode after the wire writes only the
        // selected rows (x_fin 3): the same bytes, most of them moved off the drain.  EF21's
        // decode writes gE to the unselected elements and keeps the whole-bucket decode.
        const size_t esz = p->dtype == ARCTOPK_BF16 ? 2 : 4;
        if (!e && ARCTOPK_ZERO_AHEAD && !defer && async_ar && ef != ARCTOPK_EF21 && p->n_dec > 0 &&
            (int64_t)(p->info.numel * esz) >= (int64_t)ARCTOPK_ZERO_AHEAD_MIN_BYTES) {
            const hipError_t he = hipMemsetAsync(bucket, 0, (size_t)p->info.numel * esz, ss);
            if (he != hipSuccess) return (int)he;
            p->x_fin = 3;
        }
    } else if (!marks && ef != ARCTOPK_EF21) {
        // world size 1 (EF14 / noef): the all-reduce is the identity, so no packed buffer is
        // needed -- the decode (riding in a later select launch, or inline below) takes the
        // selected rows from E / the bucket itself and zeroes the rest (finalize_chunk)
        p->x_fin = 1;
        p->x_err = err;
    } else if (defer && !marks && !side) {
        // world size 1, deferred (EF21): nothing reads the packed values before the next call's
        // select (the decode rides there), so the pack rides in the next call's encode launch
        // (not with a select stream: that encode, on the caller's stream, would wait for this select)
        p->x_pack = 1;
        p->x_err = err;
    } else {
        e = arctopk_pack(p, bucket, err, ef, p->b_rowlist, p->b_slotmap, p->b_packed, ss);
    }
    if (!e) e = mark(marks, ARCTOPK_MARK_PACK, st);
    if (e) return e;
    ht.lap(4);
    if (async_ar) {  // the index-free all-reduce of the packed values (:280) on its own stream
        hipError_t he = hipStreamWaitEvent(as, (hipEvent_t)p->x_ev_packed, 0);
        if (he != hipSuccess) return (int)he;
        if ((e = arctopk_comm_allreduce(packed_comm, p->b_packed, p->info.packed_len, p->dtype, as))) return e;
        he = hipEventRecord((hipEvent_t)p->x_ev_ar, as);
        if (he != hipSuccess) return (int)he;
        Watchdog::get().watch(packed_comm, p->x_ev_ar);
    }
    ht.lap(5);
    // the backward's last step (no deferral): the last deferred decode it finishes shares one
    // launch with its own decode, after its own packed all-reduce (unless markers were asked for)
    arctopk_plan* pair = nullptr;
    if (!defer && !async_ar && nfinish > 0 && finish[nfinish - 1] && finish[nfinish - 1] != p &&
        finish[nfinish - 1]->x_deferred && !(finish_marks && finish_marks[nfinish - 1]) && !marks &&
        x_stream_of(finish[nfinish - 1], st) == ss)
        pair = finish[nfinish - 1];
    // earlier buckets' deferred decodes the caller wants done now (in its order)
    for (int32_t i = 0; i < nfinish && !e; ++i)
        if (finish[i] && finish[i] != p && finish[i] != pair)
            e = arctopk_exchange_finish(finish[i], stream, finish_marks ? finish_marks[i] : nullptr);
    if (e) return e;
    ht.lap(6);
    if (defer) {
        p->x_deferred = async_ar ? 1 : 2;
        p->x_bucket = bucket;
        p->x_gerr = gerr;
        p->x_ef = ef;
        p->x_ws = ws;
        p->x_stream = side ? (void*)ss : nullptr;
        return 0;
    }
    if (async_ar) {  // this step's own packed all-reduce, on the all-reduce stream
        if ((e = (int)hipStreamWaitEvent(ss, (hipEvent_t)p->x_ev_ar, 0))) return e;
    } else if (packed_comm) {
        e = arctopk_comm_allreduce(packed_comm, p->b_packed, p->info.packed_len, p->dtype, ss);
    }
    if (!e) e = mark(marks, ARCTOPK_MARK_PACKED_AR, st);
    if (e) return e;
    if (pair) {
        if (packed_comm && (e = ensure_event(&p->x_ev_dec, hipEventDisableTiming | hipEventReleaseToDevice))) return e;
        if ((e = pack_now(pair, ss)) || (e = wait_ar(pair, ss))) return e;
        e = arctopk::decode_pair(pair, pair->x_ws, pair->x_ef, pair->x_gerr, pair->x_bucket, p, ws, ef, gerr, bucket,
                                 ss, packed_comm ? p->x_ev_dec : nullptr);
        if (!e) {
            pair->x_deferred = pair->x_fin = 0;
            pair->x_stream = nullptr;
            p->x_fin = 0;
            if (packed_comm) Watchdog::get().watch(packed_comm, p->x_ev_dec);
            e = join_stream(p, ss, st);  // the caller's stream sees the bucket decoded
            ht.lap(7);
            return e;
        }
        if (e != ARCTOPK_EINVAL) return e;
        // the pair does not qualify (dtype, EF class, LDS): one by one
        if ((e = arctopk_exchange_finish(pair, ss, nullptr))) return e;
    }
    if (packed_comm) {  // the decode kernel completes x_ev_dec: the inline all-reduce is watched too
        if ((e = ensure_event(&p->x_ev_dec, hipEventDisableTiming | hipEventReleaseToDevice))) return e;
        e = arctopk::decode_signal(p, p->b_packed, p->b_slotmap, ws, ef, gerr, bucket, ss, p->x_ev_dec);
        if (!e) Watchdog::get().watch(packed_comm, p->x_ev_dec);
        p->x_fin = 0;
    } else {
        e = arctopk::decode_signal(p, p->b_packed, p->b_slotmap, ws, ef, gerr, bucket, ss, nullptr);
        p->x_fin = 0;
    }
    if (!e) e = mark(marks, ARCTOPK_MARK_DECODE, st);
    if (!e) e = join_stream(p, ss, st);  // the caller's stream sees the bucket decoded
    ht.lap(7);
    return e;
}

// Diagnostics (include/arctopk.h, diagnostics section): host ns spent in the exchange step's parts since the
// last read (ARCTOPK_HOST_TIMING=1), summed over `*calls` steps; resets the sums.
extern "C" int arctopk_diag_host_times(int64_t* ns, int32_t n, int64_t* calls) {
    if (!ns || n < 0 || !calls) return ARCTOPK_EINVAL;
    for (int i = 0; i < n && i < kHtParts; ++i) ns[i] = g_ht_ns[i].exchange(0);
    *calls = g_ht_calls.exchange(0);
    return 0;
}
