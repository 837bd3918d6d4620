"""ARC-TopK DDP comm hook on MI355X -- drop-in for the reference's
comm_hooks/group_topk_hook_no_reshape.py (``GroupTopKState`` :143-171,
``cal_k`` :173-187, ``group_topk_hook`` :190-297).

Per bucket call the codec runs as four HIP kernels of libarctopk.so with two
RCCL all-reduces in between, all enqueued on the caller's current stream with
no host synchronisation:

    encode  (EF pre-apply + rank-r sketch of every tensor, one HBM pass)
    all_reduce(sketch)            one call per bucket (the reference: one per tensor)
    select  (mean sketch -> row energy -> exact top-k rows)
    pack    (gather selected rows, EF14/EF21 residual update)
    all_reduce(packed values)     index-free: every rank selected the same rows
    decode  (mean of the selected rows into the bucket, EF21 global residual)

Semantics kept from the reference: same state attributes (``iter``,
``error_dict``, ``global_error_dict``, ``rng``, ``comm_bits_this_round`` ...),
same warm-up and EF21-init paths, the same seed draw and global reseed (the
global generators are left exactly where the reference's leave them), the same
projections V (``state.projections``: "device" = the reference's
torch.randn(..., device=tensor.device) Philox stream, drawn by a HIP kernel;
"host" = torch's CPU generator stream, as when the reference runs on CPU), the
same k per tensor, the same output bucket and residuals.  Selected rows are identical to the reference's
except where two rows' sketch energies are equal within fp32 rounding of the
sketch (the GPU sums G.V in a different order than CPU sgemm); exact ties at
the k-th energy are resolved lowest-row-first.  Buckets may be float32 or
bfloat16 (every value the reference rounds to bf16 is rounded the same way).

At world size 1 the hook returns an already completed Future holding the bucket,
as the reference does (:294-297).  At world size > 1 (``async_exchange``) the
packed all-reduce and the decode run off the caller's stream and the Future is
device-aware: ``wait()`` makes the waiting stream wait for the decode, as DDP's
finalize does, so the next bucket's encode overlaps this bucket's exchange.
"""

import collections
import logging
import os
import time
import weakref
from typing import Dict, List, Tuple

import torch
import torch.distributed as dist

from allreducetopk_amd import _native as N
from allreducetopk_amd import exchange as X
from allreducetopk_amd.comm_hooks import default_hooks
from allreducetopk_amd.comm_hooks.projections import SYNC_MAX_VALUES, ProjectionSource
from allreducetopk_amd.comm_hooks.utils import HookState, dtype_bits, tensor_bits

logger = logging.getLogger(__name__)

__all__ = ["GroupTopKState", "cal_k", "group_topk_hook", "BucketPlan"]


def _geometry(shape) -> Tuple[int, int, int]:
    """(kind, n, m) as the reference reads a gradient (:19, :44-46, :73-76)."""
    shape = tuple(int(s) for s in shape)
    d = 1
    for s in shape:
        d *= s
    if len(shape) == 1:
        return N.SEG_RAW, d, 1
    if len(shape) == 2:
        return N.SEG_SKETCH, shape[0], shape[1]
    t = shape[-1]
    m = 2 * t * t
    return N.SEG_SKETCH, d // m if m else 0, m


def group_runs(segs, numel: int, esz: int, target_bytes: int):
    """[(seg_begin, seg_end), ...]: the bucket's segments cut into runs of about
    `target_bytes` each (at most one cut per segment boundary), or None when fewer than two
    runs result.  A run may start only at a segment whose offsets keep the kernels' vector
    alignment (arctopk_plan_group: bucket, sketch, packed and V offsets multiples of 8
    elements, slot map of 4); each cut is the valid boundary nearest to an equal share."""
    ng = min(len(segs), -(-numel * esz // max(1, int(target_bytes))))
    if ng < 2:
        return None

    # arctopk_plan_group (plan.hip) checks the V offset of the run's first SKETCH segment, which
    # need not be the run's first segment (DDP's reverse order puts biases and norms first): the
    # V offset a run starting at i is bound to is that of the first SKETCH segment at or after i
    next_v = [0] * (len(segs) + 1)
    for i in range(len(segs) - 1, -1, -1):
        next_v[i] = int(segs[i].v_off) if segs[i].kind == N.SEG_SKETCH else next_v[i + 1]

    def ok(i):
        s = segs[i]
        return (s.offset % 8 == 0 and s.sketch_off % 8 == 0 and s.packed_off % 8 == 0
                and s.row_off % 4 == 0 and next_v[i] % 8 == 0)

    cuts = [0]
    for j in range(1, ng):
        goal = numel * j // ng
        best = None
        for i in range(cuts[-1] + 1, len(segs)):
            if ok(i) and (best is None or abs(segs[i].offset - goal) < abs(segs[best].offset - goal)):
                best = i
        if best is not None:
            cuts.append(best)
    cuts.append(len(segs))
    runs = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if a < b]
    return runs if len(runs) >= 2 else None


class BucketPlan:
    """Native plan + persistent device buffers of one bucket layout."""

    def __init__(self, shapes: List[Tuple[int, ...]], r: int, ratio: float, dtype, device):
        if dtype not in N.DTYPE_CODE:
            raise TypeError(f"ARC-TopK HIP codec supports float32 and bfloat16 buckets, got {dtype}")
        L = N.lib()
        dims: List[int] = []
        nd: List[int] = []
        for s in shapes:
            dims.extend(int(d) for d in s)
            nd.append(len(s))
        self.shapes = shapes
        self.r = r
        self.ratio = ratio
        self.device = torch.device(device)
        handle = N.c_void_p()
        st = L.arctopk_plan_create((N.c_int64 * max(1, len(dims)))(*dims), (N.c_int32 * len(nd))(*nd),
                                   len(nd), r, float(ratio), N.DTYPE_CODE[dtype], self.device.index or 0,
                                   N.ctypes.byref(handle))
        N.check(st, f"arctopk_plan_create(shapes={shapes}, r={r}, ratio={ratio})")
        self.handle = handle
        info = N.PlanInfo()
        N.check(L.arctopk_plan_query(handle, N.ctypes.byref(info)), "arctopk_plan_query")
        self.info = info
        self.segments = []
        for i in range(info.nseg):
            seg = N.Segment()
            N.check(L.arctopk_plan_segment(handle, i, N.ctypes.byref(seg)), "arctopk_plan_segment")
            self.segments.append(seg)
        self.ms = tuple(int(s.m) for s in self.segments if s.kind == N.SEG_SKETCH)
        dev = self.device
        # sketch, packed values and projections live in the bucket dtype, as in the reference
        # (group_topk_hook_no_reshape.py:49, :53, :263)
        self.dtype = dtype
        self.sketch = torch.empty(max(1, info.sketch_len), dtype=dtype, device=dev)
        # zero-filled: the <= 3 alignment pad floats between segments ride the
        # all-reduce as zeros and are never decoded
        self.packed = torch.zeros(max(1, info.packed_len), dtype=dtype, device=dev)
        self.rowlist = torch.empty(max(1, info.sel_rows), dtype=torch.int32, device=dev)
        self.slotmap = torch.empty(max(1, info.rows_total), dtype=torch.int32, device=dev)
        # projections: device slots filled by H2D copies on a side stream, so the copy for a
        # call overlaps the kernels before it.  A slot is reused (least recently used first)
        # only once the host knows its last reader complete; otherwise another slot is
        # added: the copy stream never waits for the caller's stream (such a wait makes
        # hipMemcpyAsync block the host until that stream drains, starving the GPU).
        # Completion is tracked by a checkpoint event every V_CHECK_EVERY calls, not per
        # call: any event recorded between two kernels idles the GPU ~6 us.
        self.V_ring = [torch.empty(max(1, info.v_len), dtype=dtype, device=dev)
                       for _ in range(self.V_RING)]
        self._v_call = [0] * self.V_RING      # plan call whose encode last read slot i (0: none)
        self._v_ready = [None] * self.V_RING  # event after slot i's H2D copy
        self._v_streams = [None] * self.V_RING
        self._v_order = collections.deque(range(self.V_RING))  # least recently used first
        self._ncalls = 0                      # encodes that read a ring slot
        self._checks = collections.deque()    # (call number, DeviceEvent after its encode)
        self._done_upto = 0                   # every such encode up to this call is complete
        self._ev_free = []                    # completed checkpoint events, for reuse
        self.v_waits = 0                      # calls whose encode had to wait for its copy
        self.prestaged = None    # (seed, ring slot) of the next call's V, copied a call early
        # device projections: the seed whose V_ring[0] draw is already enqueued (drawn by the
        # previous call's select launch), and the stream of V_ring[0]'s last writer / reader
        self.v_drawn = None
        self.v_stream = None
        self.comm_registered = None  # the exchange communicator this plan's buffers are known to
        # the device generator's Philox offset after the reference's per-tensor
        # torch.randn(m, r, device=...) draws of one call (see _reseed_global)
        adv = N.c_uint64()
        N.check(L.arctopk_plan_philox_advance(handle, N.ctypes.byref(adv)), "arctopk_plan_philox_advance")
        self.philox_advance = int(adv.value)
        # the buffers arctopk_step (one native call per world-size-1 step) works on
        N.check(L.arctopk_plan_bind(handle, self.sketch.data_ptr(), self.rowlist.data_ptr(),
                                    self.slotmap.data_ptr(), self.packed.data_ptr(),
                                    self.V_ring[0].data_ptr()), "arctopk_plan_bind")
        bits = dtype_bits(dtype)
        # bits_sum of one call: sketch P + selected values per tensor (:32, :57, :70, :119)
        self.bits_sum = sum(((s.n if s.kind == N.SEG_RAW else s.n * r) + s.k_rows * s.m) * bits
                            for s in self.segments)

    V_RING = 4        # projection slots allocated up front per bucket
    V_RING_MAX = 32   # ... and at most (then the copy stream waits for the oldest reader)
    V_CHECK_EVERY = 8  # calls per slot-reuse checkpoint event

    def _checkpoint(self, stream):
        ev = self._ev_free.pop() if self._ev_free else N.DeviceEvent()
        ev.record(stream.cuda_stream)
        self._checks.append((self._ncalls, ev))
        return ev

    def _known_done(self, call: int) -> bool:
        while self._checks and self._checks[0][1].query():
            c, ev = self._checks.popleft()
            self._done_upto = c
            self._ev_free.append(ev)
        return call <= self._done_upto

    def _take_v_slot(self, copy_stream, stream) -> int:
        order = self._v_order
        i = order[0]
        last = self._v_call[i]
        if last and not self._known_done(last):  # LRU slot may still be read
            if len(self.V_ring) < self.V_RING_MAX:
                i = len(self.V_ring)
                self.V_ring.append(torch.empty_like(self.V_ring[0]))
                self._v_call.append(0)
                self._v_ready.append(None)
                self._v_streams.append(None)
                order.append(i)  # most recently used
                return i
            ev = next((e for c, e in self._checks if c >= last), None)
            if ev is None:  # read after the last checkpoint: record one now
                ev = self._checkpoint(stream)
            ev.wait(copy_stream.cuda_stream)
        order.rotate(-1)
        self._v_call[i] = 0
        return i

    def stage_projection(self, host: torch.Tensor, copy_stream, stream):
        """Copy this call's projections `host` (pinned) into the next ring slot on
        `copy_stream`; `stream` waits for the copy.  Returns (slot index, device buffer);
        slot -1: copied in order on `stream` itself (no ring bookkeeping)."""
        if copy_stream is stream:  # in order on the caller's stream: no cross-stream events
            buf = self.V_ring[0]
            N.check(N.lib().arctopk_memcpy_h2d_async(buf.data_ptr(), host.data_ptr(),
                                                     int(self.info.v_len) * buf.element_size(),
                                                     stream.cuda_stream), "arctopk_memcpy_h2d_async")
            return -1, buf
        i = self.copy_projection(host, copy_stream, stream)
        return i, self.await_projection(i, stream)

    def copy_projection(self, host: torch.Tensor, copy_stream, stream) -> int:
        """Issue the H2D copy of `host` into a free ring slot on `copy_stream`; returns the
        slot.  The copy may be issued a call early (see `group_topk_hook`'s pre-staging);
        `stream` is the caller's stream (the encodes that read the ring)."""
        i = self._take_v_slot(copy_stream, stream)
        buf = self.V_ring[i]
        _ht("stage_pre")
        if self._v_streams[i] is not copy_stream:  # allocator: the slot is also used there
            buf.record_stream(copy_stream)
            self._v_streams[i] = copy_stream
        N.check(N.lib().arctopk_memcpy_h2d_async(buf.data_ptr(), host.data_ptr(),
                                                 int(self.info.v_len) * buf.element_size(),
                                                 copy_stream.cuda_stream), "arctopk_memcpy_h2d_async")
        if self._v_ready[i] is None:
            self._v_ready[i] = torch.cuda.Event()
        self._v_ready[i].record(copy_stream)
        return i

    def await_projection(self, i: int, stream) -> torch.Tensor:
        """Order `stream` after slot i's copy.  A copy the host already sees complete needs
        no stream wait (a wait packet between two kernels idles the GPU)."""
        if not self._v_ready[i].query():
            stream.wait_event(self._v_ready[i])
            self.v_waits += 1
        return self.V_ring[i]

    def projection_consumed(self, i: int, stream) -> None:
        """The encode just enqueued on `stream` reads slot i."""
        self._ncalls += 1
        self._v_call[i] = self._ncalls
        if self._ncalls % self.V_CHECK_EVERY == 0:
            self._checkpoint(stream)

    @property
    def sketch_view(self):
        return self.sketch[:self.info.sketch_len]

    def packed_values(self) -> torch.Tensor:
        """The selected values in the reference's values_memory layout (segments back to
        back, no alignment pads) -- for inspection and tests."""
        return torch.cat([self.packed[int(s.packed_off):int(s.packed_off + s.k_rows * s.m)]
                          for s in self.segments])

    @property
    def packed_view(self):
        return self.packed[:self.info.packed_len]

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and N is not None and N._lib is not None:
            try:
                N._lib.arctopk_plan_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None

    # ---- the four codec phases (each enqueues on `stream`) --------------------
    def encode(self, grad, err, ef: int, err_in: bool, V, stream: int):
        N.check(N.lib().arctopk_encode(self.handle, grad.data_ptr(), N.ptr(err), ef, int(err_in),
                                       V.data_ptr(), self.sketch.data_ptr(), stream),
                "arctopk_encode")

    def select(self, world_size: int, stream: int, next_plan=None, next_seed: int = 0):
        """Select; with `next_plan`, its projections for `next_seed` are drawn into its
        V_ring[0] by the same launch (arctopk_select_draw)."""
        if next_plan is None:
            N.check(N.lib().arctopk_select(self.handle, self.sketch.data_ptr(), world_size,
                                           self.rowlist.data_ptr(), self.slotmap.data_ptr(), stream),
                    "arctopk_select")
            return
        N.check(N.lib().arctopk_select_draw(self.handle, self.sketch.data_ptr(), world_size,
                                            self.rowlist.data_ptr(), self.slotmap.data_ptr(),
                                            next_plan.handle, next_seed,
                                            next_plan.V_ring[0].data_ptr(), stream),
                "arctopk_select_draw")

    def pack(self, grad, err, ef: int, stream: int):
        N.check(N.lib().arctopk_pack(self.handle, N.ptr(grad), N.ptr(err), ef,
                                     self.rowlist.data_ptr(), self.slotmap.data_ptr(),
                                     self.packed.data_ptr(), stream), "arctopk_pack")

    def decode(self, world_size: int, ef: int, gerr, out, stream: int):
        N.check(N.lib().arctopk_decode(self.handle, self.packed.data_ptr(), self.slotmap.data_ptr(),
                                       world_size, ef, N.ptr(gerr), out.data_ptr(), stream),
                "arctopk_decode")

    def row_energy(self, world_size: int, out, stream: int):
        N.check(N.lib().arctopk_row_energy(self.handle, self.sketch.data_ptr(), world_size,
                                           out.data_ptr(), stream), "arctopk_row_energy")

    def groups(self, target_bytes: int):
        """The bucket cut into runs of consecutive tensors of about `target_bytes` each (the
        exchange pipeline's unit), as GroupPlans bound to this plan's
        buffers; None when the bucket yields fewer than two (one tensor, or a small bucket).
        Cuts fall only where every buffer offset keeps the kernels' alignment."""
        key = int(target_bytes)
        cache = self.__dict__.setdefault("_groups", {})
        if key in cache:
            return cache[key]
        esz = torch.empty(0, dtype=self.dtype).element_size()
        runs = group_runs(self.segments, int(self.info.numel), esz, key)
        out = [GroupPlan(self, a, b) for a, b in runs] if runs else None
        cache[key] = out
        return out


class GroupPlan:
    """A run of consecutive tensors [seg_begin, seg_end) of a bucket plan (arctopk_plan_group):
    its own native plan, bound to the parent's buffers at the run's offsets, so its sketch,
    row list, slot map, packed values and projections are slices of the parent's.  The exchange
    step runs it as it runs a bucket."""

    def __init__(self, parent: BucketPlan, seg_begin: int, seg_end: int):
        L = N.lib()
        handle = N.c_void_p()
        N.check(L.arctopk_plan_group(parent.handle, seg_begin, seg_end, N.ctypes.byref(handle)),
                f"arctopk_plan_group({seg_begin}, {seg_end})")
        self.handle = handle
        # a weak reference: the parent caches its groups, and a strong one back would make a
        # replaced bucket plan (DDP's bucket rebuild) wait for the cyclic GC to free its device
        # buffers and native plans; the views below keep the buffers' storage alive
        self.parent = weakref.ref(parent)
        self.seg_begin, self.seg_end = seg_begin, seg_end
        info = N.PlanInfo()
        N.check(L.arctopk_plan_query(handle, N.ctypes.byref(info)), "arctopk_plan_query")
        self.info = info
        self.dtype, self.device, self.r = parent.dtype, parent.device, parent.r
        s0 = parent.segments[seg_begin]
        self.offset = int(s0.offset)  # first bucket element of the run
        vb = next((int(s.v_off) for s in parent.segments[seg_begin:seg_end] if s.kind == N.SEG_SKETCH), 0)
        self.v_off = vb
        self.sketch = parent.sketch[int(s0.sketch_off):int(s0.sketch_off) + max(1, info.sketch_len)]
        self.packed = parent.packed[int(s0.packed_off):int(s0.packed_off) + max(1, info.packed_len)]
        self.rowlist = parent.rowlist[int(s0.sel_off):]
        self.slotmap = parent.slotmap[int(s0.row_off):]
        self.V = parent.V_ring[0][vb:]
        N.check(L.arctopk_plan_bind(handle, self.sketch.data_ptr(), self.rowlist.data_ptr(),
                                    self.slotmap.data_ptr(), self.packed.data_ptr(), self.V.data_ptr()),
                "arctopk_plan_bind")
        self.v_drawn = None
        self.v_stream = None
        self.comm_registered = None

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and N is not None and N._lib is not None:
            try:
                N._lib.arctopk_plan_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None


class GroupTopKState(HookState):
    """State of the ARC-TopK hook (reference :143-171; same constructor)."""

    def __init__(self, process_group: dist.ProcessGroup, r: int = 4, compress_ratio: float = 0.08,
                 start_compress_iter: int = 2, use_error_feedback="noef", seed=0, error_decay=1.0):
        super().__init__(process_group)
        self.r = r
        self.compress_ratio = compress_ratio
        self.iter = 0
        self.start_compress_iter = start_compress_iter
        self.seed = seed
        self.use_error_feedback = use_error_feedback
        self.error_dict: Dict[int, torch.Tensor] = {}
        self.global_error_dict: Dict[int, torch.Tensor] = {}
        self.error_decay = error_decay
        # the projection-seed generator (reference :165-166) -- see the `rng` property
        self._rng = torch.Generator()
        self._rng.manual_seed(seed)
        self._rng_lag = 0          # seeds handed out but not yet drawn from _rng
        self._rng_strict = False   # True once _rng was exposed: draw from it every call
        # MI355X codec state (not in the reference)
        self._plans: Dict[int, Tuple[tuple, BucketPlan]] = {}
        self._proj = ProjectionSource(r)
        # optional phase timing: a list that receives one dict of HIP events for every
        # `phase_event_every`-th call (HIP events on the hook's stream); `hook_events` receives
        # the light samples of every `hook_event_every`-th other call: only start, after the
        # V draw, after encode and the decode end (each marker idles the GPU a few us)
        self.phase_events = None
        self.phase_event_every = 1
        self.hook_events = None
        self.hook_event_every = 0
        self.prestage_hits = 0  # calls whose projections were copied during the previous call
        self._ev_calls = 0
        # measurement option (not in the reference): model a NIC-staged exchange by moving
        # the packed payload device -> pinned host -> device around the all-reduce
        self.host_staged = False
        self._host_buf = None
        # The exchange (not in the reference, which blocks on every collective): at world size
        # > 1 each call is ONE native step that issues the kernels and both all-reduces
        # (arctopk_exchange_step); with `async_exchange` the packed all-reduce and the decode
        # run on an exchange stream, so the next bucket's encode overlaps this bucket's time on
        # the wire, and the returned Future is device-aware (wait() orders the waiter's stream
        # after the decode).  `force_exchange` runs that same path at world size 1 (over a
        # one-rank communicator): the code path of every N > 1 rank, measurable on one GPU.
        self.async_exchange = True
        self.force_exchange = os.environ.get("ARCTOPK_FORCE_EXCHANGE", "0") == "1"
        # projection H2D on a copy stream (event-ordered) or in order on the caller's stream
        self.v_copy_side_stream = os.environ.get("ARCTOPK_V_COPY", "side") != "main"
        self._copy_streams: Dict[int, torch.cuda.Stream] = {}
        self._ar_streams: Dict[int, torch.cuda.Stream] = {}   # packed all-reduces
        self._side_streams: Dict[int, torch.cuda.Stream] = {}  # host-staged copies
        # Deferred decodes: a step's decode runs inside a later call (in
        # that call's select launch, whose latency it hides; or, with collectives, once the
        # packed all-reduce on the exchange stream is done), and the backward's last bucket
        # finishes them all.  The Future of a deferred step completes only when its decode is
        # enqueued (a later hook call), so deferral needs a caller that waits on no bucket's
        # Future before the backward's last hook call -- DDP's Reducer (finalize, after every
        # bucket).  None (default): defer for DDP's own buckets (dist.GradBucket, or a state
        # registered by register_comm_hook_for_ddp_model); True: always (callers that wait like
        # DDP: bench.py); False: never (every Future complete on return).
        # FIFO of (plan, its Future, its markers, bucket tensor, stream, residuals kept alive).
        self.defer_decode = None
        self._x_pend: List[tuple] = []
        # measurement only: emulated-wire communicators (exchange.Comm.wire parameters, e.g.
        # dict(ranks=8, busbw_gbs=350)) instead of real ones; with force_exchange at world
        # size 1 the step then runs beside the local cost of an N-rank ring
        self.emulate_wire = None
        # Sketch all-reduces on a communicator of their own ("separate") or on the packed
        # values' communicator ("shared": a sketch then queues behind the previous bucket's
        # packed all-reduce).  DESIGN.md section 6 discusses the two-communicator ordering.
        self.sketch_comm = os.environ.get("ARCTOPK_SKETCH_COMM", "separate")
        if self.sketch_comm not in ("separate", "shared"):
            raise ValueError("ARCTOPK_SKETCH_COMM must be 'separate' or 'shared'")
        self._comms = None  # (group, device, sketch Comm, packed Comm), see init_exchange_comms
        # The exchange pipeline below a bucket: "auto" runs a bucket as
        # groups of consecutive tensors of about `group_bytes` when its all-reduce would leave
        # the wire idle (the first bucket after the pipeline drained, the backward's last);
        # "all": every bucket; "off": whole buckets.  Results are the same bits either way.
        self.exchange_groups = os.environ.get("ARCTOPK_EXCHANGE_GROUPS", "auto")
        if self.exchange_groups not in ("auto", "all", "off"):
            raise ValueError("ARCTOPK_EXCHANGE_GROUPS must be 'auto', 'all' or 'off'")
        self.group_bytes = int(float(os.environ.get("ARCTOPK_GROUP_MIB", "128")) * (1 << 20))
        # Select streams: the encode (and sketch all-reduce) stay on the
        # caller's stream, and the latency-bound select chain, the pack and the decodes of a
        # deferred bucket run on one of two high-priority side streams (alternating), so they
        # overlap the next buckets' encodes and each other.  Each hand-over costs a cross-queue
        # dependency (~12 us measured) and the backward's last two decodes no longer pair, so
        # "auto" uses them only where the overlap pays: buckets of at most `select_stream_bytes`
        # (a large bucket's encode and decode stream at HBM speed) in a backward whose previous
        # pass had at least `select_stream_min_buckets` such buckets (ResNet-50's DDP buckets:
        # +11 %; ResNet-18's two: -15 %).  "on": every bucket; "off": the
        # caller's stream only.  Results are the same bits either way.
        self.select_streams = os.environ.get("ARCTOPK_SELECT_STREAMS", "auto")
        if self.select_streams not in ("auto", "on", "off"):
            raise ValueError("ARCTOPK_SELECT_STREAMS must be 'auto', 'on' or 'off'")
        self.select_stream_bytes = int(float(os.environ.get("ARCTOPK_SELECT_STREAM_MIB", "64")) * (1 << 20))
        self.select_stream_min_buckets = int(os.environ.get("ARCTOPK_SELECT_STREAM_MIN_BUCKETS", "4"))
        # Trailing steps: at world size 1, a bucket of at most
        # `trail_bytes` whose tensors all take single-block selects (ResNet-18's and ResNet-50's
        # first DDP buckets: the fc layer and a few BatchNorm vectors) enqueues nothing; the next
        # bucket's encode and compact launches carry its encode tiles and selects, so it costs no
        # launch of its own.  0 disables.  Results are the same bits either way.
        self.trail_bytes = int(float(os.environ.get("ARCTOPK_TRAIL_MIB", "2")) * (1 << 20))
        self._trail = None  # the pending entry (in _x_pend) of a recorded trailing step
        self.trail_calls = 0
        self._sel_streams: Dict[int, List[torch.cuda.Stream]] = {}
        self._sel_turn = 0
        self._sel_small = 0        # select-stream-sized buckets hooked so far in this backward
        self._sel_small_last = 0   # ... in the previous backward
        # The plan of a bucket is found by its buffer's identity (no gradients() walk per
        # call).  DDP rebuilds its buckets once, after the first iteration, and the caching
        # allocator may hand a rebuilt bucket the same block: for the first
        # `layout_check_iters` iterations after compression starts every call re-checks
        # the gradient shapes against its plan.
        self.layout_check_iters = 3
        self._first_compressed_iter = None
        # Where V comes from.  "device" (default): drawn on the bucket's GPU by
        # arctopk_draw_projections, bit-identical to the reference's own
        # torch.randn(m, r, device=tensor.device) after torch.manual_seed(seed) -- what the
        # reference computes when it runs on GPUs, as every BASELINE config does.  "host":
        # the CPU generator's stream (the reference run on CPU, which is how this container's
        # golden vectors were produced), drawn natively ahead of time and copied to the GPU.
        self.projections = os.environ.get("ARCTOPK_PROJECTIONS", "device")
        if self.projections not in ("device", "host"):
            raise ValueError("projections must be 'device' or 'host'")
        # device projections drawn a call early: each select launch also draws the
        # predicted next call's V (next bucket in the observed order, next seed of the rng)
        # in its trailing blocks, beside the latency-bound select; the next call uses it
        # only if its seed is the predicted one, else draws its own.  Takes the draw
        # launch off the critical path.
        self.predraw = os.environ.get("ARCTOPK_PREDRAW", "1") != "0"
        self.predraw_hits = 0
        self._succ: Dict[int, int] = {}  # bucket -> the bucket that followed it last time
        self._last_b = None

    @property
    def rng(self) -> torch.Generator:
        """The projection-seed generator (reference :165-166, drawn once per compressed call
        at :254).  The hook takes its seeds from a batched look-ahead clone and draws the
        same values from this generator lazily: any access here first brings it to the exact
        position, and from then on every call draws from it directly (the caller may keep
        the reference and reseed it)."""
        self._sync_rng()
        self._rng_strict = True
        return self._rng

    @rng.setter
    def rng(self, g: torch.Generator) -> None:
        self._rng = g
        self._rng_lag = 0
        self._rng_strict = True
        self._proj.reset()

    def _sync_rng(self) -> None:
        if self._rng_lag:  # one randint of n = n randints of 1, in order
            torch.randint(0, 1_000_000_000, (self._rng_lag,), generator=self._rng)
            self._rng_lag = 0

    def _checkpoint_rng(self) -> torch.Generator:
        """The generator at its exact position, for state_dict / load_state_dict (which
        do not expose it to the caller)."""
        self._sync_rng()
        return self._rng

    def _next_seed(self) -> int:
        """This call's projection seed: the next value of rng's randint(0, 1e9) sequence."""
        p = self._proj
        if self._rng_strict:
            return p.consume_seed(self._rng)
        if p._lookahead is None:
            self._sync_rng()
            p._sync_lookahead(self._rng)
        seed = p._peek_seeds(1)[0]
        p._future_seeds.popleft()
        self._rng_lag += 1
        return seed

    def init_exchange_comms(self, device=None) -> None:
        """Create the exchange's communicators now: collective over the ranks of the hook's
        group (RCCL communicators block until every rank has called this).
        register_comm_hook_for_ddp_model calls it on every rank; otherwise the hook does it
        at its first compressed call (every rank reaches that call at the same point of the
        same backward).  The constructor itself is not collective."""
        if self._comms is not None:
            return
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("init_exchange_comms needs an initialised process group")
        group = self.process_group if self.process_group is not None else dist.group.WORLD
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        device = torch.device(device)
        wire = self.emulate_wire
        if wire is not None and group.size() != 1:
            raise RuntimeError("emulate_wire models the wire on one GPU: world size must be 1")
        sk, pk = X.make_comms(group, device, self.sketch_comm, wire=wire)
        self._comms = (group, device, sk, pk)

    def reset_exchange_comms(self) -> None:
        """Drop the exchange communicators (after finishing deferred decodes); the next
        compressed call makes new ones (e.g. after switching emulate_wire)."""
        self.flush_exchange()
        self._comms = None

    def _raise_if_comm_failed(self) -> None:
        """RuntimeError when a communicator of the exchange failed (watchdog timeout, RCCL
        error, abort): the reference's collectives raise from the hook in that case."""
        if self._comms is not None:
            for c in (self._comms[2], self._comms[3]):
                c.raise_if_failed()

    def flush_exchange(self, upto=None) -> None:
        """Enqueue deferred decodes in call order (each on the stream of its call) and
        complete their Futures: all of them, or up to and including `upto`'s.  The hook does
        this itself in later calls; a Python wait()/value() on such a Future does it too."""
        while self._x_pend:
            e_ = self._x_pend.pop(0)
            plan, fut, marks, t, sid, _keep = e_
            if e_ is self._trail:  # (a trailing step: enqueued, then decoded, by the finish)
                self._trail = None
            N.check(N.lib().arctopk_exchange_finish(plan.handle, sid, marks), "arctopk_exchange_finish")
            if fut is None:  # a group of a bucket: its last group's entry holds the Future
                continue
            fut.set_result(t)
            if fut is upto:
                break
        self._raise_if_comm_failed()

    def state_dict(self) -> dict:
        self.flush_exchange()  # the deferred decode writes gE (EF21)
        return super().state_dict()

    def load_state_dict(self, sd: dict, device=None) -> None:
        # a pending decode writes into the residuals being replaced
        self.flush_exchange()
        super().load_state_dict(sd, device)

    def _exchange_comms(self, group, dev):
        if self._comms is None:
            logger.info("ARC-TopK: creating the exchange communicators at the first compressed call")
            self.init_exchange_comms(dev)
        g, d, sk, pk = self._comms
        if g is not group or d != dev:
            raise RuntimeError("the exchange communicators were made for another group or device")
        return sk, pk

    def _side_stream(self, table: Dict[int, "torch.cuda.Stream"], device,
                     priority: int = 0) -> "torch.cuda.Stream":
        idx = torch.device(device).index or 0
        s = table.get(idx)
        if s is None:
            s = torch.cuda.Stream(device=device, priority=priority)
            table[idx] = s
        return s

    def _select_stream(self, device) -> "torch.cuda.Stream":
        """The next of the device's two select streams (high priority: their latency-bound
        launches are dispatched ahead of the caller's queued encode blocks)."""
        idx = torch.device(device).index or 0
        pair = self._sel_streams.get(idx)
        if pair is None:
            pair = [torch.cuda.Stream(device=device, priority=XSTREAM_PRIORITY) for _ in range(2)]
            self._sel_streams[idx] = pair
        self._sel_turn ^= 1
        return pair[self._sel_turn]

    def _after_load(self) -> None:
        # prefetched projections were keyed on seeds of the old rng position
        self._proj.reset()

    def _plan_for(self, bucket, buf=None) -> BucketPlan:
        if buf is None:
            buf = bucket.buffer()
        if _LIB[0] is None:
            _LIB[0] = N.lib()
        if self._first_compressed_iter is None:
            self._first_compressed_iter = self.iter
        # fast path: the bucket's flat buffer is the one this plan was built for (DDP keeps a
        # bucket's buffer across iterations; its one-time rebuild falls in the check window)
        ident = (buf.data_ptr(), buf.numel(), buf.dtype, self.r, float(self.compress_ratio))
        hit = self._plans.get(bucket.index())
        if (hit is not None and hit[2] == ident
                and self.iter >= self._first_compressed_iter + self.layout_check_iters):
            return hit[1]
        grads = bucket.gradients()
        shapes = [tuple(g.shape) for g in grads]
        key = (tuple(shapes), buf.dtype, buf.device, self.r, float(self.compress_ratio))
        if hit is not None and hit[0] == key:
            self._plans[bucket.index()] = (key, hit[1], ident)
            return hit[1]
        _check_bucket_layout(buf, grads)
        plan = BucketPlan(shapes, self.r, self.compress_ratio, buf.dtype, buf.device)
        self._plans[bucket.index()] = (key, plan, ident)
        return plan

    def _note_call(self, b: int) -> None:
        """Record the observed bucket order (the bucket that followed the previous call's);
        the predictions below follow the latest observation, so a changed order (a DDP
        bucket rebuild) costs one misprediction per bucket."""
        if self._last_b is not None and self._last_b != b:
            self._succ[self._last_b] = b
        self._last_b = b

    def _next_plan(self, b: int):
        """The plan of the bucket predicted to come after bucket b."""
        nb = self._succ.get(b)
        ent = None if nb is None else self._plans.get(nb)
        return None if ent is None else ent[1]

    def _upcoming_ms(self, bucket) -> List[Tuple[int, ...]]:
        """Column lists of the next calls, following the observed bucket order."""
        b = bucket.index()
        out = []
        for _ in range(self._proj.depth):
            b = self._succ.get(b)
            ent = None if b is None else self._plans.get(b)
            if ent is None:
                break
            out.append(ent[1].ms)
        return out


def _prestage_next(state, bucket, dtype, dev) -> None:
    """Issue the H2D copy of the NEXT call's projections now, if its prefetched draw is
    already complete.  The next call is predicted as for the prefetch (bucket order
    repeats) with the seed the rng will yield; a wrong prediction is simply not used (the
    next call compares seeds).  Copying a call early lets that call skip its stream wait
    on the copy (`BucketPlan.await_projection`)."""
    nplan = state._next_plan(bucket.index())
    if nplan is None:
        return
    if not nplan.info.v_len or nplan.dtype != dtype or nplan.device != dev:
        return
    seed = state._proj.peek_next_seed()
    if seed is None:
        return
    slot = state._proj.try_get(seed, nplan.ms, dtype)
    if slot is None:
        if sum(nplan.ms) * nplan.r >= SYNC_MAX_VALUES:  # prefetched draw not done: at its call
            return
        slot = state._proj.get(seed, nplan.ms, dtype)  # small: drawn here instead of next call
    cs = state._side_stream(state._copy_streams, dev, COPY_PRIORITY)
    i = nplan.copy_projection(slot.host, cs, torch.cuda.current_stream(dev))
    state._proj.release(slot, cs)
    nplan.prestaged = (seed, i)


# light samples alternate between a marker after the decode (the device timeline between
# two of them, several calls apart, gives the hook's device time per call) and the encode
# kernel alone (after the V draw .. after encode)
_LIGHT_MARKS = (frozenset(("decode",)), frozenset(("draw", "encode")))
# the markers each path records (ARCTOPK_MARK_* of arctopk_step / arctopk_exchange_step)
_STEP_MARKS = frozenset(("start", "draw", "encode", "select", "pack", "decode"))
_EXCHANGE_MARKS = frozenset(N.MARKS)
_PHASE_MARKS = ("start", "draw", "encode", "sketch_allreduce", "select", "pack", "h2d",
                "packed_allreduce", "decode")


def _phase_marks(state, names=_PHASE_MARKS):
    """This call's timing markers (bench sampling, state.phase_events / hook_events): a dict
    name -> timed device event, or None.  Each marker between two kernels idles the GPU a
    few us, so only every `phase_event_every`-th call gets the full set and every
    `hook_event_every`-th other call a light set (_LIGHT_MARKS)."""
    if state.phase_events is None and state.hook_events is None:
        return None
    state._ev_calls += 1
    c = state._ev_calls - 1
    if state.phase_events is not None and c % state.phase_event_every == 0:
        evs = {n: N.DeviceEvent(timing=True) for n in names}
        state.phase_events.append(evs)
        return evs
    if state.hook_events is not None and state.hook_event_every and c % state.hook_event_every == 0:
        light = _LIGHT_MARKS[(c // state.hook_event_every) % 2]
        evs = {n: N.DeviceEvent(timing=True) for n in names if n in light}
        evs["_call"] = c
        state.hook_events.append(evs)
        return evs
    return None


def _call_marks(state, names):
    """The ARCTOPK_MARK_* event array a native step records, or None."""
    evs = _phase_marks(state, names)
    if evs is None:
        return None
    arr = (N.c_void_p * N.NMARKS)()
    for n, e in evs.items():
        if n != "_call":
            arr[N.MARKS[n]] = e.handle
    return arr


class ExchangeFuture(torch.futures.Future):
    """The Future of an overlapped exchange step, whose decode is deferred to the next hook
    call.  It completes once that decode is enqueued on the caller's
    stream (the reference's completed-Future semantics from then on).  wait() / value() from
    Python enqueue the decode first, so a caller that waits before its next hook call never
    blocks; DDP waits (from C++) only in its finalize, after the backward's last bucket,
    whose call runs inline and leaves nothing deferred."""

    def wait(self):
        if not self.done():
            self._arctopk_state.flush_exchange(upto=self)
        return super().wait()

    def value(self):
        if not self.done():
            self._arctopk_state.flush_exchange(upto=self)
        return super().value()


def _order_after_exchange(state, dev) -> None:
    """Before a collective on the torch process group (warm-up, EF21 init, phase path): the
    deferred decode is enqueued (its stream then follows the last packed all-reduce), so
    collectives of this library's communicators and of torch's are never in flight together."""
    state.flush_exchange()


def _host_projections(state, plan, bucket, seed, dtype, dev, stream):
    """The "host" projection source: V from the CPU generator's stream (drawn natively,
    ahead of time) copied to a device slot on a side stream.  Returns (ring slot, V)."""
    vslot, V = -1, plan.V_ring[0]
    pre, plan.prestaged = plan.prestaged, None
    if pre is not None and pre[0] == seed and state.v_copy_side_stream:
        # copied during the previous call: usually complete by now, so no stream wait
        vslot, V = pre[1], plan.await_projection(pre[1], stream)
        state.prestage_hits += 1
        _ht("prestaged")
    else:
        slot = state._proj.get(seed, plan.ms, dtype)
        _ht("proj_get")
        if plan.info.v_len:  # 512 KiB pinned H2D at headline, on a side stream, ahead of encode
            cs = state._side_stream(state._copy_streams, dev, COPY_PRIORITY) if state.v_copy_side_stream else stream
            vslot, V = plan.stage_projection(slot.host, cs, stream)
            _ht("stage_copy")
            state._proj.release(slot, cs)  # refilled only after this copy completed
        else:
            state._proj.release(slot)
    _ht("stage_v")
    state._proj.prefetch(state._upcoming_ms(bucket), dtype)
    _ht("prefetch")
    if state.v_copy_side_stream:
        _prestage_next(state, bucket, dtype, dev)
        _ht("prestage_next")
    return vslot, V


def _claim_projections(state, plan, seed: int, sid: int, dev) -> bool:
    """Device projections of this call: True when V must be drawn now, False when the
    previous call's select launch already drew it for this seed (or there is no V).
    V_ring[0] is written and read on the caller's stream only; when the caller's stream
    changed since its last user (raw handle `sid` differs), that stream may be gone by now,
    so the device is synchronised once instead of waiting on a stored handle."""
    if not plan.info.v_len:
        return False
    if plan.v_stream is not None and plan.v_stream != sid:
        torch.cuda.synchronize(dev)
    plan.v_stream = sid
    pre, plan.v_drawn = plan.v_drawn, None
    if pre == seed:
        state.predraw_hits += 1
        return False
    return True


def _predraw_target(state, b: int, dtype, dev, sid: int):
    """(plan, seed) whose projections this call's select launch draws in advance: the
    predicted next bucket's plan and the rng's next seed, or (None, 0)."""
    if not state.predraw:
        return None, 0
    nplan = state._next_plan(b)
    if (nplan is None or not nplan.info.v_len or nplan.dtype != dtype or nplan.device != dev
            or (nplan.v_stream is not None and nplan.v_stream != sid)):
        return None, 0
    nseed = state._proj.peek_next_seed()
    return (nplan, nseed) if nseed is not None else (None, 0)


_RESEED_FAST = None
_LIB = [None]


def _current_raw_stream(device_index: int) -> int:
    """The caller's current HIP stream on the device, as a raw handle (no Stream object)."""
    return torch._C._cuda_getCurrentRawStream(device_index)

# optional host-time breakdown of the hook (diagnostics; ARCTOPK_HOST_TIMING=1)
# Priority of the projection copy stream.  HIP maps a process's streams onto a few HW
# queues (4 on MI355X); a normal-priority copy stream can share one with the caller's
# stream, and its completion marker then waits behind the queued kernels, so the encode
# always had to wait for the copy (~17 us idle per call).  A high-priority stream gets a
# queue of its own: the copy is seen complete a call later and no wait is needed.
COPY_PRIORITY = -1
# The exchange streams run the packed all-reduce and the decode beside the next bucket's
# encode: high priority, so RCCL's blocks are dispatched ahead of the encode's queued blocks.
XSTREAM_PRIORITY = -1
HOST_TIMES = {} if os.environ.get("ARCTOPK_HOST_TIMING") == "1" else None
_ht_last = [0.0]


def _ht(name=None):
    if HOST_TIMES is None:
        return
    t = time.perf_counter()
    if name is not None:
        HOST_TIMES[name] = HOST_TIMES.get(name, 0.0) + (t - _ht_last[0])
    _ht_last[0] = t


def _reseed_global(seed: int, device_index: int = 0, advance: int = 0) -> None:
    """``torch.manual_seed(seed)`` (ref :255) and the reference's projection draws'
    effect on the device generator, without their per-call cost.

    torch.manual_seed reseeds the CPU generator and every CUDA device's default
    generator (plus MPS/XPU/custom devices, absent on ROCm builds).  When only CPU and
    CUDA exist this does exactly that; otherwise it defers to torch.manual_seed.  The
    reference then draws ``torch.randn(m, r, device=tensor.device)`` per 2-D/ND tensor
    (:49, :79), which moves that device generator's Philox offset by `advance` (summed
    per draw, BucketPlan.philox_advance); the codec draws V from the CPU stream instead
    (DESIGN.md deviation 3), so the offset is set directly: afterwards the global
    generators stand exactly where the reference leaves them.
    """
    global _RESEED_FAST
    if _RESEED_FAST is None:
        fast = (torch.cuda.is_available() and not torch.backends.mps.is_available()
                and not (hasattr(torch, "xpu") and torch.xpu.is_available())
                and torch._C._get_privateuse1_backend_name() == "privateuseone")
        _RESEED_FAST = [torch.cuda.default_generators[i] for i in range(torch.cuda.device_count())] \
            if fast else False
    if _RESEED_FAST is False or not torch.cuda.is_initialized():
        torch.manual_seed(seed)
        if advance and torch.cuda.is_initialized():
            torch.cuda.default_generators[device_index].set_offset(advance)
        return
    for g in _RESEED_FAST:
        g.manual_seed(seed)
    torch.default_generator.manual_seed(seed)
    if advance:
        _RESEED_FAST[device_index].set_offset(advance)


def cal_k(state, tensor) -> int:
    """Selected elements of one tensor (reference :173-187)."""
    kind, n, m = _geometry(tensor.shape)
    return max(1, int(n * state.compress_ratio)) * m


def _bucket_plan_of(p):
    """The bucket plan a pending exchange entry belongs to (a GroupPlan's parent)."""
    return p.parent() if isinstance(p, GroupPlan) else p


def _check_bucket_layout(buf: torch.Tensor, grads) -> None:
    if not buf.is_cuda:
        raise RuntimeError("ARC-TopK HIP codec needs the bucket on a GPU (got CPU tensor); "
                           "the CPU reference algorithm lives in oracle/ (tests only)")
    if buf.dim() != 1 or not buf.is_contiguous():
        raise RuntimeError("bucket buffer must be a contiguous 1-D tensor")
    esz = buf.element_size()
    off = 0
    for g in grads:
        if not g.is_contiguous():
            raise RuntimeError("bucket gradient views must be contiguous (view(-1) in the reference)")
        if (g.data_ptr() - buf.data_ptr()) // esz != off:
            raise RuntimeError("bucket gradient views must tile the buffer in order")
        off += g.numel()
    if off != buf.numel():
        raise RuntimeError("bucket gradient views do not cover the buffer")


def _residual_on(table: Dict[int, torch.Tensor], b: int, bucket: torch.Tensor,
                 name: str) -> torch.Tensor:
    """The residual of bucket b, checked before its pointer reaches a kernel: same numel and
    dtype as the bucket (else RuntimeError, as the reference's add_ raises), contiguous, on
    the bucket's device (a checkpoint loaded with map_location='cpu' or onto another rank's
    device is moved there once and kept)."""
    t = table[b]
    if t.numel() != bucket.numel():
        raise RuntimeError(f"bucket {b} changed size ({t.numel()} -> {bucket.numel()}) after its "
                           f"residual ({name}) was created")
    if t.dtype != bucket.dtype:
        raise RuntimeError(f"{name}[{b}] is {t.dtype} but the bucket is {bucket.dtype}")
    if t.device != bucket.device or not t.is_contiguous():
        t = t.to(bucket.device).contiguous()
        table[b] = t
    return t


def _stage_through_host(state: GroupTopKState, pv: torch.Tensor, stream, dev,
                        chunks: int = 8) -> None:
    """Move the packed payload device -> pinned host -> device as a NIC-staged exchange
    would, in `chunks` pieces: D2H of piece i+1 runs while piece i goes back H2D (PCIe is
    full duplex), so the pair costs about one direction plus one piece.  `stream` waits
    for the last piece."""
    n = pv.numel()
    if state._host_buf is None or state._host_buf.numel() < n:
        state._host_buf = torch.empty(n, dtype=pv.dtype, pin_memory=True)
    hb = state._host_buf[:n]
    d2h = state._side_stream(state._copy_streams, dev, COPY_PRIORITY)
    h2d = state._side_stream(state._side_streams, dev)
    d2h.wait_stream(stream)
    h2d.wait_stream(stream)
    step = max(1, -(-n // chunks))
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        with torch.cuda.stream(d2h):
            hb[lo:hi].copy_(pv[lo:hi], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(d2h)
        h2d.wait_event(ev)
        with torch.cuda.stream(h2d):
            pv[lo:hi].copy_(hb[lo:hi], non_blocking=True)
    stream.wait_stream(h2d)
    stream.wait_stream(d2h)


def group_topk_hook(state: GroupTopKState, bucket: dist.GradBucket
                    ) -> torch.futures.Future[torch.Tensor]:
    state.maybe_accumulate_momentum_on_bucket(bucket)
    group = state.process_group if state.process_group is not None else dist.group.WORLD
    world_size = group.size()
    input_tensor = bucket.buffer()

    # warm-up: dense all-reduce for the first start_compress_iter iterations (:213-215)
    if state.iter < state.start_compress_iter:
        if state._x_pend:
            _order_after_exchange(state, input_tensor.device)
        state.maybe_increase_iter(bucket)
        return default_hooks._allreduce_fut(group, input_tensor, state)

    b = bucket.index()
    total = input_tensor.shape[0]
    ef_name = state.use_error_feedback
    ef = N.EF_CODE.get(ef_name)
    if ef is None:
        raise ValueError(f"use_error_feedback must be noef/ef14/ef21, got {ef_name!r}")
    err = gerr = None
    err_in = True
    if ef == N.EF14:
        if b not in state.error_dict:
            logger.info("A zero tensor of length %s that represents local error is created.", total)
            state.error_dict[b] = torch.zeros(total, device=input_tensor.device,
                                              dtype=input_tensor.dtype)
            err_in = False  # first call: the residual is not added (:228-230)
        err = state.error_dict[b]
    elif ef == N.EF21:
        if b not in state.error_dict:  # E_0 = grad; all-reduce grad; gE_0 = mean (:236-250)
            logger.info("A tensor of length %s that represents local/global error is created.", total)
            state.error_dict[b] = torch.clone(input_tensor).detach()
            state.comm_bits_this_round += tensor_bits(input_tensor)
            if state._x_pend:
                _order_after_exchange(state, input_tensor.device)
            dist.all_reduce(input_tensor, group=group, async_op=False)
            input_tensor.div_(world_size)
            state.global_error_dict[b] = torch.clone(input_tensor).detach()
            state.maybe_increase_iter(bucket)
            fut = torch.futures.Future()
            fut.set_result(input_tensor)
            return fut
        err = state.error_dict[b]
        gerr = state.global_error_dict[b]
    if err is not None:
        err = _residual_on(state.error_dict, b, input_tensor, "error_dict")
        if gerr is not None:
            gerr = _residual_on(state.global_error_dict, b, input_tensor, "global_error_dict")

    # per-call projection seed, and the reference's global reseed side effect (:254-255)
    _ht()
    device_v = state.projections == "device"
    seed = state._next_seed()  # (:254), from a batched look-ahead of the sequence
    plan = state._plan_for(bucket, input_tensor)
    dev = input_tensor.device
    dix = dev.index or 0
    # host projections model the reference on CPU, whose draws move the CPU generator, not
    # the device one: the generator-position guarantee covers device projections
    _reseed_global(seed, dix, plan.philox_advance if device_v else 0)
    state._note_call(b)
    _ht("seed+plan")

    sid = _current_raw_stream(dix)
    dtype = input_tensor.dtype
    L = _LIB[0]
    if not state.host_staged:
        # ONE native call per bucket (arctopk_exchange_step): the kernels, the collectives at
        # world size > 1 (or with force_exchange: the N > 1 code path over one-rank
        # communicators), and earlier buckets' deferred decodes
        comms = world_size > 1 or state.force_exchange or state.emulate_wire is not None
        sk = pk = None
        if comms:
            sk, pk = state._exchange_comms(group, dev)  # (a failed communicator: the step returns its status)
            if plan.comm_registered is not pk:
                sk.register(plan.sketch)
                pk.register(plan.packed)
                plan.comm_registered = pk
        vslot, vptr, draw, nplan, nseed = -1, None, False, None, 0
        if device_v:
            draw = _claim_projections(state, plan, seed, sid, dev)
            nplan, nseed = _predraw_target(state, b, dtype, dev, sid)
        else:
            vslot, V = _host_projections(state, plan, bucket, seed, dtype, dev, torch.cuda.current_stream(dev))
            vptr = V.data_ptr()
        # deferred except for the last bucket of a backward (nothing follows it), which then
        # finishes every earlier deferred decode: nothing is left in flight when it returns
        dd = state.defer_decode
        if dd is None:  # DDP's own buckets (or a DDP-registered state): Futures waited at finalize
            dd = isinstance(bucket, dist.GradBucket) or getattr(state, "_ddp_registered", False)
        defer = dd and state.async_exchange and not bucket.is_last()
        pend = state._x_pend
        marks = _call_marks(state, _EXCHANGE_MARKS)
        # The exchange pipeline below a bucket: with collectives, a bucket
        # may run as groups of consecutive tensors, each group its own encode -> sketch
        # all-reduce -> select -> pack -> packed all-reduce on the exchange stream, so the wire
        # starts on the first group while later ones are encoded.  Selection is per tensor and
        # both all-reduces are elementwise: the results are the bucket's bits.  Each group pays
        # one collective latency, so "auto" groups only the buckets whose all-reduce would
        # otherwise leave the wire idle: the first after the pipeline drained (nothing in flight)
        # and the backward's last (its decode is the drain).
        # a small bucket of single-block selects, with a bucket after it in this backward: a
        # trailing step, carried by the next step's launches (arctopk_exchange_trail)
        # (not in a backward that runs on select streams: there the small bucket's select already
        # overlaps the next encode, and carrying its row tiles costs the carrier's lean encode
        # kernel its occupancy -- ResNet-50 DDP measured 380 -> 335 GB/s)
        sel_backward = state.select_streams == "on" or (
            state.select_streams == "auto" and state._sel_small_last >= state.select_stream_min_buckets)
        if (not comms and defer and marks is None and device_v and state.trail_bytes > 0
                and ef != N.EF21 and state._trail is None and not sel_backward
                and total * input_tensor.element_size() <= state.trail_bytes):
            rc = L.arctopk_exchange_trail(plan.handle, input_tensor.data_ptr(), N.ptr(err), N.ptr(gerr), ef,
                                          int(err_in), int(draw), seed, None, sid)
            if rc == 0:
                fut = ExchangeFuture()
                fut._arctopk_state = state
                state._trail = (plan, fut, None, input_tensor, sid, (err, gerr))
                pend.append(state._trail)
                state.trail_calls += 1
                state._sel_small += int(total * input_tensor.element_size() <= state.select_stream_bytes)
                state.comm_bits_this_round += 2 * (world_size - 1) * plan.bits_sum  # (:278)
                state.maybe_increase_iter(bucket)
                _ht("trail")
                return fut
            if rc != N.EINVAL:
                N.check(rc, "arctopk_exchange_trail")
        trail = state._trail
        if trail is not None and (trail[4] != sid or trail[0] is plan):
            state.flush_exchange()  # another stream, or the same bucket again: enqueued on its own
            trail = None
        if trail is not None:  # not a ride candidate of this call: carried (or enqueued) by it
            pend.remove(trail)
            state._trail = None
        units = None
        if (comms and state.async_exchange and marks is None and state.exchange_groups != "off"
                and (state.exchange_groups == "all" or not pend or bucket.is_last())):
            units = plan.groups(state.group_bytes)
        grouped = units is not None
        if not grouped:
            units = (plan,)
        # finish first: a caller that skipped buckets, or one whose stream changed since a
        # pending step (its decode is enqueued on that step's own stream)
        if any(_bucket_plan_of(e_[0]) is plan or e_[4] != sid for e_ in pend):
            state.flush_exchange()
        ars = None
        if comms:
            ars = state._side_stream(state._ar_streams, dev, XSTREAM_PRIORITY)
            if pk.kind == "callback" and ars.cuda_stream not in pk._streams:
                pk.known_stream(ars)
        # a select stream for this bucket (whole buckets of deferring callers, no markers)
        small = total * input_tensor.element_size() <= state.select_stream_bytes
        state._sel_small += int(small)
        if bucket.is_last():
            state._sel_small_last, state._sel_small = state._sel_small, 0
        side = None
        if (state.select_streams != "off" and not grouped and marks is None and dd
                and (not comms or ars is not None)
                and (state.select_streams == "on"
                     or (small and state._sel_small_last >= state.select_stream_min_buckets))):
            side = state._select_stream(dev)
            nplan, nseed = None, 0  # the select does not draw the next call's V (that encode would wait)
        # the decode riding in this call's select launch: the previous bucket's without
        # collectives, the one before it with them (its all-reduce has had a whole call to
        # finish, so the select is not held back waiting for it) or with select streams (the
        # same stream's previous bucket: the streams alternate)
        depth = 2 if (comms or side is not None) else 1
        if defer:
            fut = ExchangeFuture()
            fut._arctopk_state = state
        else:
            fut = torch.futures.Future()
        esz = input_tensor.element_size()
        x_p, e_p, g_p = input_tensor.data_ptr(), N.ptr(err), N.ptr(gerr)
        nu = len(units)
        for ui, u in enumerate(units):
            last_u = ui == nu - 1
            u_defer = defer if last_u else True  # a group's decode is finished by a later one
            if grouped:
                if u.comm_registered is not pk:
                    sk.register(u.sketch)
                    pk.register(u.packed)
                    u.comm_registered = pk
                off = u.offset * esz
                u_x, u_e, u_g = x_p + off, (e_p + off if e_p else None), (g_p + off if g_p else None)
                if device_v:  # V drawn by group 0 and then by each group's select for the next
                    u_draw = int(draw and ui == 0)
                    u_next, u_nseed = (units[ui + 1], seed) if (draw and not last_u) else (None, 0)
                    u_vptr = None
                else:
                    u_draw, u_next, u_nseed = 0, None, 0
                    u_vptr = vptr + u.v_off * esz
                if last_u:
                    u_next, u_nseed = nplan, nseed
            else:
                u_x, u_e, u_g, u_draw, u_next, u_nseed, u_vptr = x_p, e_p, g_p, draw, nplan, nseed, vptr
            ride = pend.pop(0) if len(pend) >= depth else None
            u_trail = None
            if trail is not None and ui == 0:  # deferred once this step returns
                pend.append(trail)
                u_trail = trail[0].handle
            fin = pend[:] if not u_defer else []
            if not u_defer:
                pend.clear()
            nf = len(fin)
            if nf:
                fin_plans = (N.c_void_p * nf)(*[e_[0].handle for e_ in fin])
                fin_marks = (N.c_void_p * nf)(*[N.ctypes.cast(e_[2], N.c_void_p).value if e_[2] is not None
                                                else None for e_ in fin])
            else:  # (most calls: no ctypes arrays built per call)
                fin_plans = fin_marks = None
            _ht("prep")
            st_ = L.arctopk_exchange_step(u.handle, u_x, u_e, u_g, ef, int(err_in), int(u_draw), seed,
                                          u_next.handle if u_next is not None else None, u_nseed,
                                          sk.handle if comms else None, pk.handle if comms else None, sid,
                                          ars.cuda_stream if ars is not None else None,
                                          int(u_defer), ride[0].handle if ride is not None else None,
                                          ride[2] if ride is not None else None, fin_plans, fin_marks, nf,
                                          u_vptr, marks, side.cuda_stream if side is not None else None,
                                          u_trail)
            if st_:
                if comms:
                    for c in (sk, pk):
                        c.check(st_, "arctopk_exchange_step")
                N.check(st_, "arctopk_exchange_step")
            for e_ in ([ride] if ride is not None else []) + fin:  # their decodes are enqueued now
                if e_[1] is not None:
                    e_[1].set_result(e_[3])
            if u_defer:
                pend.append((u, fut if last_u else None, marks, input_tensor, sid, (err, gerr)))
        if nplan is not None:
            nplan.v_drawn, nplan.v_stream = nseed, sid
        if vslot >= 0:
            plan.projection_consumed(vslot, torch.cuda.current_stream(dev))
        _ht("native_step")
        state.comm_bits_this_round += 2 * (world_size - 1) * plan.bits_sum  # (:278)
        state.maybe_increase_iter(bucket)
        if not defer:
            fut.set_result(input_tensor)
        _ht("tail")
        return fut

    # host-staged measurement mode (packed payload through pinned host memory, NIC model):
    # phase by phase on the caller's stream
    if state._x_pend:
        state.flush_exchange()
    stream = torch.cuda.current_stream(dev)
    vslot, V = -1, plan.V_ring[0]
    if not device_v:
        vslot, V = _host_projections(state, plan, bucket, seed, dtype, dev, stream)
    evs = _phase_marks(state)

    def mark(name):
        if evs is not None and name in evs:
            evs[name].record(sid)

    mark("start")
    if device_v and _claim_projections(state, plan, seed, sid, dev):
        N.check(L.arctopk_draw_projections(plan.handle, seed, V.data_ptr(), sid), "arctopk_draw_projections")
    mark("draw")
    plan.encode(input_tensor, err, ef, err_in, V, sid)
    if vslot >= 0:
        plan.projection_consumed(vslot, stream)
    mark("encode")
    if world_size > 1:
        _order_after_exchange(state, dev)
        dist.all_reduce(plan.sketch_view, group=group, async_op=False)
    mark("sketch_allreduce")
    nplan, nseed = _predraw_target(state, b, dtype, dev, sid) if device_v else (None, 0)
    plan.select(world_size, sid, nplan, nseed)
    if nplan is not None:
        nplan.v_drawn, nplan.v_stream = nseed, sid
    mark("select")
    state.comm_bits_this_round += 2 * (world_size - 1) * plan.bits_sum
    plan.pack(input_tensor, err, ef, sid)
    mark("pack")
    if state.host_staged:  # D2H to a pinned "NIC buffer" and back (NIC model)
        _stage_through_host(state, plan.packed_view, stream, dev)
        mark("h2d")
    if world_size > 1:
        dist.all_reduce(plan.packed_view, group=group, async_op=False)
    mark("packed_allreduce")
    plan.decode(world_size, ef, gerr, input_tensor, sid)
    mark("decode")
    _ht("decode")

    state.maybe_increase_iter(bucket)
    fut = torch.futures.Future()
    fut.set_result(input_tensor)
    _ht("tail")
    return fut
