/*
 * arctopk.h -- C ABI of libarctopk.so, the MI355X (gfx950) ARC-TopK / TopK /
 * RandK gradient-bucket codec.
 *
 * Boundary.  The reference (Aris-ma/AllreduceTopK) is pure Python: its hot path
 * is the DDP comm hook `group_topk_hook(state, bucket)`
 * (comm_hooks/group_topk_hook_no_reshape.py:190-297) plus the TopK/RandK hook
 * `sparse_hook_sync` (comm_hooks/sparse_hook.py:163-304), and all arithmetic in
 * them is torch aten ops.  This library replaces exactly those aten op sequences
 * with stream-ordered HIP kernels; the collectives stay with the caller
 * (torch.distributed / RCCL), so the drop-in Python hooks in
 * allreducetopk_amd/comm_hooks/ call, per bucket:
 *
 *     arctopk_encode  -> all_reduce(sketch) -> arctopk_select -> arctopk_pack
 *                     -> all_reduce(packed) -> arctopk_decode
 *
 * Conventions.
 *  - Every entry point returns 0 on success or a nonzero status (a hipError_t
 *    value, or one of the ARCTOPK_E* codes below).  Nothing throws across the ABI.
 *  - Device pointers are plain element pointers into device memory; `stream` is
 *    a hipStream_t passed as void*.  Compute entry points only enqueue work on
 *    `stream`: no host synchronisation, no allocation (graph-capturable).
 *  - A plan owns its device tables and a select workspace; calls that share a
 *    plan must be ordered on one stream.
 *  - Element types: ARCTOPK_F32 (every BASELINE config's bucket) and ARCTOPK_BF16
 *    (the Llama driver's default dtype).  Bucket-typed buffers are passed as void*.
 *    The TopK / RandK entry points are fp32 only.
 */
#ifndef ARCTOPK_H
#define ARCTOPK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes besides hipError_t */
#define ARCTOPK_OK 0
#define ARCTOPK_EINVAL 1001     /* bad argument (null pointer, ratio out of (0,1], r out of range) */
#define ARCTOPK_ERESHAPE 1002   /* ND tensor numel not divisible by m = 2*t^2 (ref :76 raises) */
#define ARCTOPK_EDTYPE 1003     /* unsupported element type */
#define ARCTOPK_EEMPTY 1004     /* empty tensor: torch.topk(k=1) on 0 elements raises */
#define ARCTOPK_ENOCOMM 1005    /* the RCCL library could not be loaded / lacks entry points */
#define ARCTOPK_ETIMEOUT 1006   /* a communicator's collective (or its creation) outlived the
                                   process group's timeout; the communicator was aborted */
#define ARCTOPK_EABORTED 1007   /* the communicator was aborted (by arctopk_comm_abort, or after
                                   an error of another communicator of this process) */
#define ARCTOPK_ECOMM 1100      /* RCCL error: ARCTOPK_ECOMM + ncclResult_t */

/* error-feedback modes (ref GroupTopKState.use_error_feedback, :149, :224-250) */
#define ARCTOPK_EF_NONE 0
#define ARCTOPK_EF14 1
#define ARCTOPK_EF21 2

/* element types of a bucket (and of its sketch, projections and packed values, which
 * the reference keeps in the bucket's dtype: group_topk_hook_no_reshape.py:49, :263) */
#define ARCTOPK_F32 0
#define ARCTOPK_BF16 1   /* bfloat16 storage; arithmetic in fp32, each value the reference
                            rounds to bf16 rounded the same way (round-to-nearest-even) */

/* segment kinds */
#define ARCTOPK_SEG_RAW 0     /* 1-D tensor: the "sketch" is the tensor itself (ref :19-41) */
#define ARCTOPK_SEG_SKETCH 1  /* 2-D [n,m] or ND reshaped to [d/m, m], m = 2*t^2 (ref :44-102) */

typedef struct arctopk_plan arctopk_plan;

/* Totals of a plan, for sizing the caller's buffers. */
typedef struct {
    int64_t numel;       /* bucket elements (bucket.buffer().numel())                  */
    int64_t sketch_len;  /* floats of the concatenated sketch: sum n*r (SKETCH) + d (RAW) */
    int64_t v_len;       /* floats of the concatenated projections: sum m*r over SKETCH   */
    int64_t packed_len;  /* floats of the packed buffer: every segment's k_rows*m values,
                            each segment starting 16-B aligned (<= 3 pad floats between)  */
    int64_t sel_rows;    /* sum of selected rows (length of the row list)                 */
    int64_t rows_total;  /* sum n (length of the slot map)                                */
    int32_t nseg;        /* gradient views in the bucket                                  */
    int32_t r;           /* sketch rank                                                   */
    int64_t values_len;  /* sum_k: selected elements (ref values_memory length, :261-263)  */
} arctopk_plan_info;

/* Per-segment geometry (for the host-side mirror and tests). */
typedef struct {
    int64_t offset;      /* element offset in the bucket                 */
    int64_t n, m;        /* rows, columns (m = 1 for RAW)                 */
    int64_t k_rows;      /* selected rows: max(1, int(n * ratio))  (ref cal_k :173-187) */
    int64_t sketch_off;  /* float offset in the sketch buffer            */
    int64_t v_off;       /* float offset in the projection buffer (-1: RAW) */
    int64_t packed_off;  /* element offset in the packed buffer          */
    int64_t row_off;     /* offset in the slot map (global row index)    */
    int64_t sel_off;     /* offset in the selected-row list              */
    int32_t kind;        /* ARCTOPK_SEG_RAW / ARCTOPK_SEG_SKETCH          */
    int32_t pad;
} arctopk_segment;

/*
 * Build the plan of one bucket layout.  `dims` holds the shapes of
 * bucket.gradients() concatenated, `ndims[i]` the rank of tensor i.  Geometry and
 * k follow the reference: 1-D -> RAW; 2-D -> [shape0, shape1]; ND -> [d/m, m]
 * with m = 2*shape[-1]^2 (group_topk_hook_no_reshape.py:16-102, cal_k :173-187).
 * Replaces: the per-call Python loop over bucket.gradients() (:111-129, :259).
 */
int arctopk_plan_create(const int64_t* dims, const int32_t* ndims, int32_t ntensors, int32_t r,
                        double compress_ratio, int32_t dtype, int32_t device, arctopk_plan** out);
int arctopk_plan_destroy(arctopk_plan* plan);
/* Host-only: the geometry a plan would have (no device memory touched); segs_out may be NULL. */
int arctopk_plan_describe(const int64_t* dims, const int32_t* ndims, int32_t ntensors, int32_t r,
                          double compress_ratio, arctopk_segment* segs_out, arctopk_plan_info* info);
int arctopk_plan_query(const arctopk_plan* plan, arctopk_plan_info* info);
/*
 * A plan over the consecutive segments [seg_begin, seg_end) of `parent` (a group of the bucket's
 * tensors): the exchange pipeline's unit below a bucket.  Geometry, k and
 * projections (the parent's Philox offsets) are the parent's; every offset is relative to the
 * group's first segment, so bind the group to the parent's buffers at those segment's offsets
 * (sketch_off, row_off, row_off, packed_off, first SKETCH v_off) and pass bucket / residual
 * pointers at its element offset.  ARCTOPK_EINVAL when the group's base offsets are not
 * multiples of 8 elements (sketch, packed, bucket, V) and 4 (slot map), which keeps every vector
 * path of the kernels aligned as in the parent.  Destroy with arctopk_plan_destroy.
 * Replaces: nothing in the reference (its per-tensor sketch all-reduce, :33, :58, :88, is the
 * finest grain; the group is a run of those tensors).
 */
int arctopk_plan_group(const arctopk_plan* parent, int32_t seg_begin, int32_t seg_end,
                       arctopk_plan** out);

int arctopk_plan_segment(const arctopk_plan* plan, int32_t i, arctopk_segment* seg);

/*
 * K1 encode.  EF pre-apply fused with the rank-r sketch of every tensor.
 *   ef = NONE : X = G
 *   ef = EF14 : X = G + E (err_in = 1) or X = G (first call, err_in = 0); writes E := X
 *   ef = EF21 : X = G - E (nothing written but the sketch)
 * sketch[SKETCH seg] = X.view(n,m) @ V  ([n][r] row-major); sketch[RAW seg] = X.
 * `V` is the concatenation of each SKETCH tensor's [m][r] projection in bucket order.
 * Replaces: input_tensor.add_(error, alpha=+-1) (:227, :234), tensor @ V (:53, :83),
 *           P = P_local.clone() (:31, :56, :86).
 */
int arctopk_encode(const arctopk_plan* plan, const void* grad, void* err, int32_t ef,
                   int32_t err_in, const void* V, void* sketch, void* stream);

/*
 * K2 select.  From the all-reduced sketch: P /= world_size, row energy
 * sum_j P[row][j]^2 (sequential j, as torch.sum over dim 1 for r <= 4) or P^2
 * (RAW), top-k_rows rows per segment.  Ties at the k-th energy: lowest rows
 * first.  Writes the selected rows ascending (rowlist[sel_off ..]) and, for every
 * row, its packed slot or -1 (slotmap[row_off + row]).
 * Replaces: P /= ws; norms = sum(P**2, 1); torch.topk(norms, k, sorted=False);
 *           row*m + arange(m) index materialisation (:34-38, :59-66, :89-96).
 */
int arctopk_select(const arctopk_plan* plan, const void* sketch, int32_t world_size,
                   int32_t* rowlist, int32_t* slotmap, void* stream);

/*
 * arctopk_select, and in the same launch (its trailing blocks, which run beside the
 * latency-bound select blocks) the device projections of the NEXT call: V_next =
 * arctopk_draw_projections(next, next_seed).  The caller predicts the next call (plan and
 * seed) and keeps V_next only when that call's seed matches; otherwise it draws again.
 * `next` must have `plan`'s dtype and device; `next` = NULL is arctopk_select.
 * Removes the draw launch (and its kernel boundary) from the next call's critical path.
 */
int arctopk_select_draw(const arctopk_plan* plan, const void* sketch, int32_t world_size,
                        int32_t* rowlist, int32_t* slotmap, const arctopk_plan* next,
                        uint64_t next_seed, void* next_V, void* stream);

/*
 * Phase markers of a step (arctopk_step / arctopk_exchange_step): `marks` is NULL or an array
 * of ARCTOPK_NMARKS hipEvent_t handles; every non-NULL entry is recorded at that point (for
 * per-phase timing; each record between two kernels idles the GPU a few microseconds).
 * PACKED_AR and DECODE are recorded on the stream that runs them (the exchange stream when
 * there is one).
 */
#define ARCTOPK_MARK_START 0      /* before the projection draw                       */
#define ARCTOPK_MARK_DRAW 1       /* after the draw, before the encode                */
#define ARCTOPK_MARK_ENCODE 2
#define ARCTOPK_MARK_SKETCH_AR 3  /* exchange step only                               */
#define ARCTOPK_MARK_SELECT 4
#define ARCTOPK_MARK_PACK 5
#define ARCTOPK_MARK_PACKED_AR 6  /* exchange step only                               */
#define ARCTOPK_MARK_DECODE 7
#define ARCTOPK_NMARKS 8

/*
 * One-call step at world size 1, where both all-reduces of the hook are identities
 * (group_topk_hook_no_reshape.py:264, :280): [draw V for `seed` when draw != 0] -> encode
 * -> select (+ the next call's projections: next / next_seed, as arctopk_select_draw) ->
 * pack -> decode into `bucket`, on the buffers bound to the plan by arctopk_plan_bind (the
 * sketch, row list, slot map, packed values and projection buffer the phase entry points
 * take as arguments).  One foreign-function call per hook call instead of one per phase.
 */
int arctopk_plan_bind(arctopk_plan* plan, void* sketch, int32_t* rowlist, int32_t* slotmap,
                      void* packed, void* V);
int arctopk_step(const arctopk_plan* plan, void* bucket, void* err, void* gerr, int32_t ef,
                 int32_t err_in, int32_t draw, uint64_t seed, const arctopk_plan* next,
                 uint64_t next_seed, void* stream, void* const* marks);

/* ---- the exchange: collectives of the hook (group_topk_hook_no_reshape.py:58, :280) ---- */
/*
 * A communicator for the hook's SUM all-reduces: an RCCL communicator owned by this library
 * (RCCL loaded at run time from `rccl_path`, normally the librccl.so torch itself loaded, so
 * the process holds one RCCL), or a callback (`fn(ctx, buf, count, dtype, stream)` must
 * all-reduce `count` elements at `buf` in place, ordered on `stream`; returns 0 or nonzero).
 * Creating an RCCL communicator is collective: every rank calls arctopk_comm_init_rccl with
 * the id rank 0 obtained from arctopk_comm_unique_id (128 bytes), and it blocks until all have.
 */
typedef struct arctopk_comm arctopk_comm;
typedef int (*arctopk_allreduce_fn)(void* ctx, void* buf, int64_t count, int32_t dtype, void* stream);
int arctopk_comm_unique_id(const char* rccl_path, void* id_out);
int arctopk_comm_init_rccl(const char* rccl_path, const void* id, int32_t nranks, int32_t rank,
                           int32_t device, arctopk_comm** out);
/*
 * Failure detection (the reference's collectives run on ProcessGroupNCCL, whose watchdog turns
 * a hung or failed collective into an error after the group's timeout: cifar10/run_cifar10.py:
 * 55-58).  arctopk_comm_init_rccl_timeout creates the communicator non-blocking
 * (ncclCommInitRankConfig, blocking = 0) and gives up after `timeout_ms` (aborting it:
 * ARCTOPK_ETIMEOUT) when a rank never joins.  With timeout_ms > 0 a watchdog thread of the
 * library then polls ncclCommGetAsyncError and the completion of every collective the
 * exchange step issued on the communicator; an asynchronous RCCL error, or a collective still
 * pending `timeout_ms` after it was enqueued, aborts EVERY RCCL communicator of the library
 * (the GPU kernels of an aborted communicator exit) and leaves the error sticky:
 * arctopk_comm_status returns it, and every later exchange step on the communicator returns
 * it instead of enqueueing work.  Work already queued behind the failed collective (the decode,
 * the caller's copy-back and optimizer step) would then run on partially reduced buffers, so,
 * as ProcessGroupNCCL's async error handling does by default, the watchdog ends the process
 * instead of aborting (stderr message, exit status 1).  ARCTOPK_ASYNC_ERROR_HANDLING (else torch's
 * TORCH_NCCL_ASYNC_ERROR_HANDLING) = 0 or 2 keeps it alive: the error is then raised by the
 * next exchange step.  arctopk_comm_init_rccl = timeout 0: blocking creation, no watchdog.  The
 * device current on the calling thread is left unchanged.
 */
int arctopk_comm_init_rccl_timeout(const char* rccl_path, const void* id, int32_t nranks, int32_t rank,
                                   int32_t device, int64_t timeout_ms, arctopk_comm** out);
int arctopk_comm_status(const arctopk_comm* comm);
int arctopk_comm_abort(arctopk_comm* comm);
int arctopk_comm_init_callback(arctopk_allreduce_fn fn, void* ctx, int32_t nranks, int32_t rank,
                               arctopk_comm** out);
/*
 * Measurement only: an "emulated wire" communicator of world size 1 (results are those of a
 * one-rank all-reduce: the buffer is left unchanged) whose all-reduce costs what an
 * `emul_ranks`-rank ring all-reduce costs the local GPU: a kernel of `blocks` workgroups
 * (RCCL's CU footprint) that reads and rewrites 2 (R - 1) / R of the buffer's bytes in HBM,
 * paced to take at least latency_us + 2 (R - 1) / R * bytes / busbw_gbs.  Lets one GPU measure
 * the exchange step beside an N-rank wire.
 */
int arctopk_comm_init_wire(int32_t emul_ranks, double busbw_gbs, double latency_us, int32_t blocks,
                           int32_t device, arctopk_comm** out);
/* Destroy a communicator.  An RCCL communicator created non-blocking is finalized first
 * (ncclCommFinalize, polled until its pending operations have flushed, at most its timeout;
 * past it, or on an error, it is aborted and ARCTOPK_ETIMEOUT / the RCCL error is returned),
 * then destroyed. */
int arctopk_comm_destroy(arctopk_comm* comm);
int arctopk_comm_size(const arctopk_comm* comm);
/* in-place SUM all-reduce of `count` elements (ARCTOPK_F32 / ARCTOPK_BF16), stream-ordered */
int arctopk_comm_allreduce(arctopk_comm* comm, void* buf, int64_t count, int32_t dtype, void* stream);

/*
 * One bucket call of the hook, collectives included, in one host call.  World size = the
 * communicators' size (both NULL: world size 1, no collectives issued).  On `stream`:
 *   [draw] -> encode -> all_reduce(sketch, sketch_comm) -> select (+ next V)
 *          -> pack -> the `finish` steps' deferred decodes -> [all_reduce(packed) -> decode]
 * defer = 1: this step's decode is deferred to arctopk_exchange_finish(plan, ...) (or to a
 *   later step's `ride` / `finish`); with communicators its packed all-reduce runs on
 *   `ar_stream` after the pack kernel, which completes the event that stream waits for (no
 *   marker packet on `stream`), so the caller's stream encodes the next bucket while these
 *   packed values are on the wire.  defer = 0: the decode follows on `stream`; given an
 *   `ar_stream` (and no markers), the packed all-reduce runs there too and `stream` waits for
 *   it just before the decode, so the `finish` steps' decodes run beside it on the wire;
 *   otherwise the all-reduce is inline on `stream`.
 *   Without communicators (world size 1) and markers the all-reduces are identities: for EF14 /
 *   noef no packed values are formed at all -- the decode (deferred or inline) takes the
 *   selected rows from the residual / the bucket and zeroes the rest, the same bits as pack then
 *   decode; for EF21, defer = 1 defers the pack as well, to the first blocks of the
 *   next step's encode launch (that step's `ride`; same EF mode and dtype, other bucket and
 *   residual buffers) or arctopk_exchange_finish.  Until the decode the plan's packed buffer and
 *   the residual's selected rows are not final.  CONTRACT at world size 1 with defer = 1: the
 *   deferred decode (and EF21's deferred pack) READS `bucket` and `err` -- the selected rows
 *   are taken from them when it runs, not when this step is enqueued -- so a caller must leave
 *   the bucket and residual (and gerr) untouched on every stream until that decode has been
 *   enqueued (by arctopk_exchange_finish or a later step's `ride` / `finish`); the DDP hook does
 *   (the Reducer reads a bucket only after its Future completes, which flushes the decode).
 * ride: an earlier step's deferred decode, run inside this step's select launch (extra blocks of
 *   the single-block select launch, or of the multi-block select's last, fused write launch: the
 *   select's latency then hides behind the decode's HBM stream), else right after the select;
 *   ride_marks are that step's markers.
 * finish[0 .. nfinish): earlier deferred steps decoded after this pack, in order.
 * `V`: the projections to encode with (NULL: the plan's bound projection buffer, drawn there
 * for `seed` when draw != 0).  `marks`: see ARCTOPK_MARK_*.
 * sel_stream (NULL: `stream`): a SELECT STREAM.  The draw, the encode and the sketch all-reduce
 *   stay on `stream`; the select (+ ride), the pack, the `finish` decodes and this step's own
 *   decode go on sel_stream after an event on the encode, so the latency-bound select chain runs
 *   beside the caller's next encode.  A deferred step remembers its select stream: its decode
 *   (arctopk_exchange_finish, or a later step's `ride`) goes there, and the finishing stream then
 *   waits for it; a ride from another select stream is finished on its own instead of riding.
 *   A non-deferred step leaves `stream` waiting for its decode.  With a select stream: `next`
 *   must be NULL (the next call draws its own projections), markers disable it, and with
 *   communicators `ar_stream` must be a third stream (ARCTOPK_EINVAL otherwise).
 * trail (NULL: none): a step recorded by arctopk_exchange_trail.  World size 1 without markers,
 *   when both plans qualify (same dtype, r = 4, EF mode and err_in; EF14 / noef; the trail's tensors
 *   all single-block selects and no column-split encode, this plan's with a multi-block
 *   select), the trail's encode tiles run as extra blocks of this step's encode launch and its
 *   selects as extra blocks of this step's first compact launch; otherwise it is enqueued on its
 *   own first.  Either way it leaves this call as a deferred step (its decode: a later `ride` /
 *   `finish` / arctopk_exchange_finish, like a defer = 1 step's).
 * Replaces: the whole of group_topk_hook's compressed path (:254-290) given the seed.
 */
int arctopk_exchange_step(arctopk_plan* plan, void* bucket, void* err, void* gerr, int32_t ef,
                          int32_t err_in, int32_t draw, uint64_t seed, const arctopk_plan* next,
                          uint64_t next_seed, arctopk_comm* sketch_comm, arctopk_comm* packed_comm,
                          void* stream, void* ar_stream, int32_t defer, arctopk_plan* ride,
                          void* const* ride_marks, arctopk_plan* const* finish,
                          void* const* const* finish_marks, int32_t nfinish, const void* V,
                          void* const* marks, void* sel_stream, arctopk_plan* trail);
/*
 * A TRAILING step (world size 1, EF14 / noef, a deferring caller): the call is recorded on the
 * plan and nothing is enqueued but the projection draw (draw != 0: on `stream`, now).  The next
 * arctopk_exchange_step given it as `trail` carries its encode and select in its own launches
 * (a small bucket then costs no launch of its own); arctopk_exchange_finish enqueues a trailing
 * step that no step carried, then decodes it.  The CONTRACT of a deferred step holds from this
 * call on (bucket, err, gerr untouched until the decode is enqueued).
 */
int arctopk_exchange_trail(arctopk_plan* plan, void* bucket, void* err, void* gerr, int32_t ef,
                           int32_t err_in, int32_t draw, uint64_t seed, const void* V, void* stream);
/* The deferred decode of `plan`'s last deferred exchange step (no-op if none): after that step's
 * packed all-reduce (and, at world size 1, its deferred pack), on the step's select stream if it
 * had one (then `stream` waits for it), else on `stream`.  A trailing step is enqueued first. */
int arctopk_exchange_finish(arctopk_plan* plan, void* stream, void* const* marks);

/*
 * K2 variant for tests/bit-exact checks: the per-row energy keys only
 * (float bits of the energy the reference feeds torch.topk), keys[row_off + row].
 */
int arctopk_row_energy(const arctopk_plan* plan, const void* sketch, int32_t world_size,
                       float* energy, void* stream);

/*
 * K3 pack.  Gather the selected rows into the packed buffer (segment order,
 * ascending rows) and update the local residual.  `rowlist` and `slotmap` are
 * arctopk_select's outputs (rows of 1 or 2 elements are packed by a stream over the
 * slot map, longer rows by gathering the row list):
 *   NONE : packed = G[sel]
 *   EF14 : packed = E[sel] (E holds X after encode); E[sel] = 0
 *   EF21 : D = G[sel] - E[sel]; packed = D; E[sel] = E[sel] + D
 * Replaces: tensor[topk_indices] gathers (:70-71, :101-102), values_memory /
 * indices_memory packing (:116-117), EF14 tensor.view(-1)[indices] = 0 (:124),
 * EF21 zero_/index_put (:126-128) and the residual persistence (:270-275).
 */
int arctopk_pack(const arctopk_plan* plan, const void* grad, void* err, int32_t ef,
                 const int32_t* rowlist, const int32_t* slotmap, void* packed, void* stream);

/*
 * K4 decode.  From the all-reduced packed values:
 *   NONE/EF14 : out = scatter(packed / world_size) into zeros
 *   EF21      : out = gE + scatter(packed / world_size); gE[sel] = out[sel]
 * `out` may alias the bucket (it is the bucket in the hook).  `packed` and `slotmap` are all
 * it reads of the selection: any slot map of arctopk_select's format (per row its slot within
 * the segment, ascending with the row, or -1) and packed values laid out as arctopk_pack
 * writes them, whatever ran on the plan before (the short-row chunks derive their packed
 * ranges from the slot map given, in one extra launch).
 * Replaces: values_memory.div_(ws) (:281), input_tensor.zero_() (:284), the
 * per-tensor index_put scatter (:131-141) and gE.add_/input.copy_ (:288-290).
 */
int arctopk_decode(const arctopk_plan* plan, const void* packed, const int32_t* slotmap,
                   int32_t world_size, int32_t ef, void* gerr, void* out, void* stream);

/*
 * Segment-range forms of K3/K4 (segments [seg_begin, seg_end) only), so a caller can
 * pipeline the packed all-reduce: pack group g, start its collective, pack g+1, ...
 * and decode each group once its collective has completed.  Packed data of the
 * segments in [b, e) occupy packed[seg(b).packed_off, seg(e-1).packed_off + k(e-1)).
 */
int arctopk_pack_segments(const arctopk_plan* plan, int32_t seg_begin, int32_t seg_end,
                          const void* grad, void* err, int32_t ef, const int32_t* rowlist,
                          const int32_t* slotmap, void* packed, void* stream);
int arctopk_decode_segments(const arctopk_plan* plan, int32_t seg_begin, int32_t seg_end,
                            const void* packed, const int32_t* slotmap, int32_t world_size,
                            int32_t ef, void* gerr, void* out, void* stream);

/* ---- TopK / RandK baselines (comm_hooks/sparse_hook.py, sparse_hook_c4.py) ---------- */
/*
 * Bucket-typed buffers (x, vals, E, out, gerr) are of element type `dtype` (ARCTOPK_F32 or
 * ARCTOPK_BF16); bf16 arithmetic rounds after every add / divide, as the reference's torch
 * ops on bf16 tensors do.  Tensors of a bucket are described by host arrays of `ntensors` entries:
 * offsets[i] (element offset in the bucket), numels[i], ks[i] (= max(1, int(numel*ratio)),
 * sparse_hook.py:77-78) and k_off[i] (offset of tensor i's k entries in the packed
 * idx/vals buffers).  Up to ARCTOPK_SPARSE_MAX_BATCH tensors go into one launch; more
 * are processed in batches.
 */
#define ARCTOPK_SPARSE_MAX_BATCH 64

/*
 * Bytes of `workspace` that arctopk_topk_select needs for these tensor sizes (fixed
 * tables plus a candidate list of ~n/8 per tensor of a launch batch), or
 * -ARCTOPK_EINVAL for bad arguments.
 */
int64_t arctopk_sparse_workspace_bytes(int32_t ntensors, const int64_t* numels);

/*
 * Exact element top-k of |x| per tensor by multi-block radix select; ties at the
 * k-th |x|: lowest index first.  Writes each tensor's k indices ascending as int32
 * (idx[k_off[i] ..]) and the values x[idx] (vals[k_off[i] ..]).
 * Replaces: torch.topk(tensor.abs(), k, sorted=False), .to(int32), tensor[indices]
 * (sparse_hook.py:26-28, :97-98).  zero_selected = 1: x (non-const here) is also written
 * back with its selected elements zeroed, in the same pass (EF14's `tensor[indices] = 0`,
 * :104, when x is the residual E after arctopk_ef14_fold).
 */
int arctopk_topk_select(const void* x, int32_t ntensors, const int64_t* offsets,
                        const int64_t* numels, const int64_t* ks, const int64_t* k_off,
                        int32_t* idx, void* vals, void* workspace, int32_t dtype,
                        int32_t zero_selected, void* stream);

/*
 * RandK, device-side index source (the performance mode; the parity mode draws torch.randperm
 * on the host, sparse_hook.py:20): tensor i's k indices are those of its k largest keys
 * key(j) = rk(s_i, j), a keyed bijection of the index j (two xorshift-multiply rounds; s_i =
 * splitmix64(seed + 0x9E3779B97F4A7C15 * (i + 1)) truncated to 32 bits), so the keys are
 * distinct and the subset is a uniformly random k-subset of [0, numel_i).  They are selected by
 * the same exact multi-block radix select as arctopk_topk_select and written ASCENDING
 * (idx[k_off[i] ..]), so every later pass streams the tensor in order.  x != NULL: also
 * vals = x[offsets[i] + idx] and (zero_selected) x written back with those entries zeroed in
 * the same pass (EF14's residual, sparse_hook.py:104, x = E after arctopk_ef14_fold); x = NULL:
 * indices only (offsets / vals NULL, zero_selected 0).  workspace: arctopk_sparse_workspace_bytes.
 * Replaces: torch.randperm(numel, device=...)[:k] + tensor[indices] (sparse_hook.py:20-22).
 */
int arctopk_randk_select(const void* x, int32_t ntensors, const int64_t* offsets,
                         const int64_t* numels, const int64_t* ks, const int64_t* k_off,
                         uint64_t seed, int32_t* idx, void* vals, void* workspace, int32_t dtype,
                         int32_t zero_selected, void* stream);
/*
 * arctopk_topk_select on x = E with EF14 applied in the select's first pass (fp32 only, every
 * tensor 16-B aligned with numel % 4 == 0; ARCTOPK_EINVAL otherwise, and nothing is enqueued):
 * that pass streams g (the bucket) and E, writes E := g + E (err_in; else E := g, the first call)
 * -- tensor.add_(E) (sparse_hook.py:205) -- and histograms it; the later passes select, gather and
 * (:104) zero E as arctopk_topk_select(E, ..., zero_selected = 1) does.  g is not written.
 * Replaces arctopk_ef14_fold followed by that select: one pass over the bucket and the residual
 * fewer.
 */
int arctopk_topk_select_ef14(const void* g, void* E, int32_t err_in, int32_t ntensors,
                             const int64_t* offsets, const int64_t* numels, const int64_t* ks,
                             const int64_t* k_off, int32_t* idx, void* vals, void* workspace,
                             int32_t dtype, void* stream);
/*
 * The same RandK draw with EF14 applied in the select's write pass (the hash keys never read the
 * data, so the passes before it do not either): v = g + E (err_in; else v = g, the first call),
 * rounded to the dtype as tensor.add_(E) is (sparse_hook.py:205), vals = v[idx], and E := v with
 * the selected elements zeroed (:104).  g (the bucket) is not written.  Replaces arctopk_ef14_fold
 * followed by arctopk_randk_select(E, ..., zero_selected = 1): one pass over the bucket and the
 * residual instead of two.
 */
int arctopk_randk_select_ef14(const void* g, void* E, int32_t err_in, int32_t ntensors,
                              const int64_t* offsets, const int64_t* numels, const int64_t* ks,
                              const int64_t* k_off, uint64_t seed, int32_t* idx, void* vals,
                              void* workspace, int32_t dtype, void* stream);

/* Gather vals[k_off[i] + j] = x[offsets[i] + idx[k_off[i] + j]]  (sparse_hook.py:22). */
int arctopk_sparse_gather(const void* x, int32_t ntensors, const int64_t* offsets,
                          const int64_t* ks, const int64_t* k_off, const int32_t* idx,
                          void* vals, int32_t dtype, void* stream);

/*
 * Residual persistence at the selected entries (sparse_hook.py:103-109, :257-267):
 *   EF14 : E[off + idx] = 0        (E already holds x = G + E_prev, see arctopk_ef_apply)
 *   EF21 : E[off + idx] = E + decay * vals, one rounding (E.add_(C(G - E), alpha=error_decay),
 *          :265; C(.) is zero elsewhere; decay = 1 is the default state)
 */
int arctopk_sparse_residual(void* E, int32_t ntensors, const int64_t* offsets,
                            const int64_t* ks, const int64_t* k_off, const int32_t* idx,
                            const void* vals, int32_t ef, float decay, int32_t dtype, void* stream);

/*
 * Decode into `out` (every element written):
 *   accumulate = 0 (RandK): out = 0; out[off + idx[j]] = vals[j] / world_size     (:273-278)
 *   accumulate = 2 (RandK, each tensor's idx ascending: arctopk_randk_select): the same, as one
 *                           pass of whole chunks (zeros and values composed in LDS)
 *   accumulate = 1 (TopK) : out = 0; for rank q = 0..nranks-1 in order:
 *                           out[off + idx_q[j]] += vals_q[j]; then out /= world_size (:285-292)
 * `vals`/`idx` hold nranks consecutive payloads of packed_len entries each.
 * EF21 (gerr != NULL): gE = gE + decay * out (one rounding: gE.add_(out, alpha=error_decay));
 * out = gE (:295-297).
 */
int arctopk_sparse_decode(void* out, int64_t numel, int32_t ntensors, const int64_t* offsets,
                          const int64_t* ks, const int64_t* k_off, int64_t packed_len,
                          const int32_t* idx, const void* vals, int32_t nranks,
                          int32_t world_size, int32_t accumulate, void* gerr, float decay,
                          int32_t dtype, void* stream);

/*
 * EF pre-apply on a whole bucket, one pass (ARC-TopK fuses this into arctopk_encode):
 *   EF14 : x = x + E (err_in = 1) or x unchanged (first call); then E = x
 *   EF21 : x = x - E
 * Replaces: input_tensor.add_(error_dict[b], alpha=+-1) (sparse_hook.py:205, :212) and the
 * full-bucket E.copy_(input_tensor) of EF14 (:258).
 */
int arctopk_ef_apply(void* x, void* E, int64_t numel, int32_t ef, int32_t err_in, int32_t dtype,
                     void* stream);

/*
 * EF14 fold for the sparse hooks: E := x + E (err_in = 1) or E := x (first call); x is not
 * written.  The caller then selects / gathers from E (which holds the pre-compression
 * bucket) and decodes into x.  Replaces input_tensor.add_(E) (sparse_hook.py:205) and the
 * full-bucket E.copy_(input_tensor) (:258).  With arctopk_topk_select(..., zero_selected=1)
 * on E, the EF14 residual `E[indices] = 0` (:104) is done in the select's last pass.
 */
int arctopk_ef14_fold(const void* x, void* E, int64_t numel, int32_t err_in, int32_t dtype,
                      void* stream);

/*
 * Device projections of one bucket call: for every SKETCH segment in bucket order,
 * V[v_off ..] = torch.randn(m, r, device=dev, dtype) as drawn by the reference on the GPU
 * right after torch.manual_seed(seed) (group_topk_hook_no_reshape.py:49, :79, :255):
 * torch's Philox4x32-10 normal_ kernel (hiprand) reproduced element by element, bit for bit.
 * Stream-ordered, one launch.  arctopk_plan_philox_advance: the device generator's Philox
 * offset after those draws (what torch.manual_seed + the reference's draws leave behind).
 */
int arctopk_draw_projections(const arctopk_plan* plan, uint64_t seed, void* V, void* stream);
int arctopk_plan_philox_advance(const arctopk_plan* plan, uint64_t* advance);

/*
 * Host-only (no GPU): `total` (a multiple of 16) consecutive values of the reference's
 * bf16 projection stream -- torch.randn(..., dtype=bfloat16) on CPU after
 * torch.manual_seed(seed) (group_topk_hook_no_reshape.py:49, :79, :255) -- as bf16 bit
 * patterns.  Valid when every tensor's m*r is a multiple of 16 (no tail recompute).
 * Replaces torch's scalar BFloat16 normal_fill (~8x slower) in the projection prefetch.
 */
int arctopk_draw_bf16_normal(uint64_t seed, int64_t total, uint16_t* out);

/*
 * Host-only (no GPU): one bucket call's projections -- for each of `ntensors` tensors in
 * bucket order, sizes[t] = m_t * r values of torch.randn(m_t, r, dtype) on CPU, all drawn
 * from ONE generator stream after torch.manual_seed(seed) (group_topk_hook_no_reshape.py:49,
 * :79, :255) -- concatenated into `out` (dtype ARCTOPK_F32: float, ARCTOPK_BF16: bf16 bit
 * patterns).  Replaces the reference's per-tensor torch.randn calls (one torch dispatch and
 * Python round trip each) with one call that runs without the GIL.
 */
int arctopk_draw_normal(uint64_t seed, int32_t dtype, int32_t ntensors, const int64_t* sizes,
                        void* out);

/*
 * Host-only: a pool of native threads drawing projections ahead (arctopk_draw_normal into
 * caller-owned buffers that must stay alive until the draw is waited or polled complete).
 * submit returns a ticket (> 0) or -status; wait blocks until that draw is done and returns
 * its status; poll returns 1 when done, -status if the draw failed (ticket then forgotten
 * either way), 0 if still pending.
 * destroy drops queued draws and joins the threads (running draws finish).
 */
int arctopk_draw_pool_create(int32_t nthreads, void** pool);
int arctopk_draw_pool_destroy(void* pool);
int64_t arctopk_draw_submit(void* pool, uint64_t seed, int32_t dtype, int32_t ntensors,
                            const int64_t* sizes, void* out);
int arctopk_draw_wait(void* pool, int64_t ticket);
int arctopk_draw_poll(void* pool, int64_t ticket);

/* Stream-ordered host -> device copy (hipMemcpyAsync), for the projection ring. */
int arctopk_memcpy_h2d_async(void* dst, const void* src, int64_t bytes, void* stream);

/*
 * Device-scope stream events for the hook's own intra-device ordering (projection copy ->
 * encode, encode -> reuse of a projection slot).  torch's events release to system scope:
 * recording one between two kernels writes back the L2 and leaves the GPU idle for several
 * microseconds; these use hipEventReleaseToDevice | hipEventDisableTiming.  No reference
 * counterpart (the reference is synchronous).
 *   query: 0 = complete, 1 = not yet, < 0 / other = HIP error.
 */
int arctopk_event_create(void** event);
int arctopk_event_destroy(void* event);
int arctopk_event_record(void* event, void* stream);
int arctopk_event_wait(void* stream, void* event);
int arctopk_event_query(void* event);
/* Timing variant (hipEventReleaseToDevice, timing enabled) for per-kernel durations in
 * bench.py: a torch event between two kernels writes back the L2 to system scope, which
 * adds several microseconds to the interval it brackets; these measure what the kernel
 * trace measures.  elapsed: milliseconds between two completed records. */
int arctopk_event_create_timed(void** event);
int arctopk_event_elapsed_ms(float* ms, void* start, void* end);

/* Test entry point: the kernels' fp32 -> bf16 rounding (RNE, NaN -> 0x7FC0) of n device
 * values, to check it against c10::BFloat16 on the host. */
int arctopk_round_bf16(const float* in, uint16_t* out, int64_t n, void* stream);

/* Diagnostics (not part of the codec): with ARCTOPK_HOST_TIMING=1 in the environment at the
 * first exchange step, the host nanoseconds each part of arctopk_exchange_step took, summed over
 * the steps since the last read -- ns[0 .. min(n, 8)) = entry, encode, sketch all-reduce, select,
 * pack, packed all-reduce, finish, decode; *calls = steps summed -- and the sums are reset.
 * All zero when the variable is unset.  (bench.py --host-timing breakdowns) */
int arctopk_diag_host_times(int64_t* ns, int32_t n, int64_t* calls);

/* library build identification (for smoke tests) */
const char* arctopk_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ARCTOPK_H */
