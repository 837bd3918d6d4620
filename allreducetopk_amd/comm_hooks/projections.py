"""Source of the per-call Gaussian projections V of ARC-TopK.

Reference semantics (comm_hooks/group_topk_hook_no_reshape.py:254-255, :49, :79):
per bucket call a seed is drawn from ``state.rng`` (a CPU generator), the global
RNG is reseeded with it, and ``torch.randn(m, r)`` is drawn once per 2-D/ND
tensor in bucket order.  V is drawn here from torch's CPU generator stream (mt19937 +
torch's normal transform), so the projections -- and therefore the selected rows --
are those of the reference on CPU bit for bit.

One native call (libarctopk's ``arctopk_draw_normal``, projection.cpp) draws a whole
bucket's V without the GIL; it restates torch's CPU ``normal_`` (vectorised 16-blocks
with the tail recompute, the scalar Box-Muller path with its cached sample for tensors
of < 16 values).  It is checked against torch itself once per process and dtype
(:func:`native_ok`); should they ever differ (a torch build whose kernel uses other math
routines) the projections fall back to per-tensor torch draws -- the same values, slower.

Drawing V for a 16 x [2048, 2048] bucket still costs ~1 ms of host time, more than the
whole GPU codec.  V depends only on (seed, column counts), and the seed sequence is
deterministic, so a small thread pool draws the projections of the *next* calls while
the current one runs (``depth`` calls ahead); buckets with few projection values are
drawn synchronously (cheaper than a hand-off to a thread).  A miss (first call, changed
bucket order) draws synchronously; hits and misses return the same values.
"""
from __future__ import annotations

import collections
import ctypes
import logging
import os
import threading
from typing import Dict, Optional, Sequence, Tuple

import torch

logger = logging.getLogger(__name__)

SYNC_MAX_VALUES = 4096  # projection values drawn on the caller's thread instead of prefetched


def _sizes(ms: Sequence[int], r: int):
    return (ctypes.c_int64 * max(1, len(ms)))(*[int(m) * r for m in ms])


def _draw_native(seed: int, sizes, ntensors: int, dtype: torch.dtype, out: torch.Tensor) -> None:
    from allreducetopk_amd import _native as N
    N.check(N.lib().arctopk_draw_normal(int(seed), N.DTYPE_CODE[dtype], ntensors, sizes,
                                        out.data_ptr()), "arctopk_draw_normal")


_NATIVE_OK: Dict[torch.dtype, bool] = {}
_NATIVE_LOCK = threading.Lock()
# sizes covering both torch paths: < 16 values (scalar, with the cached second sample
# carried across tensors, odd counts), 16-multiples, and tails that are recomputed
_CHECK_SIZES = (8, 3, 72, 16, 5, 4101, 12, 8192, 7, 36, 1, 600)


def native_ok(dtype: torch.dtype) -> bool:
    """Whether the native draw equals torch's CPU randn stream here (checked once)."""
    ok = _NATIVE_OK.get(dtype)
    if ok is not None:
        return ok
    with _NATIVE_LOCK:
        ok = _NATIVE_OK.get(dtype)
        if ok is None:
            seed = 440527571
            g = torch.Generator().manual_seed(seed)
            ref = torch.cat([torch.randn(n, dtype=dtype, generator=g) for n in _CHECK_SIZES])
            got = torch.empty_like(ref)
            _draw_native(seed, (ctypes.c_int64 * len(_CHECK_SIZES))(*_CHECK_SIZES),
                         len(_CHECK_SIZES), dtype, got)
            iv = torch.int16 if dtype == torch.bfloat16 else torch.int32
            ok = bool(torch.equal(got.view(iv), ref.view(iv)))
            if not ok:
                logger.warning("native %s projection draw differs from this torch build's CPU "
                               "randn; using per-tensor torch draws", dtype)
            _NATIVE_OK[dtype] = ok
    return ok


def draw_bf16_into(seed: int, out: torch.Tensor) -> None:
    """Fill the contiguous bf16 CPU tensor `out` (numel % 16 == 0) with the stream."""
    from allreducetopk_amd import _native as N
    N.check(N.lib().arctopk_draw_bf16_normal(int(seed), out.numel(), out.data_ptr()),
            "arctopk_draw_bf16_normal")


def _fill_plan(host: torch.Tensor, ms: Sequence[int], r: int, dtype: torch.dtype):
    """Views of `host` that one torch generator pass fills in the reference's stream order
    (the fallback when the native draw is not usable).

    Consecutive tensors whose m*r is a multiple of 16 share ONE view: torch's CPU normal
    fill draws all uniforms in stream order and transforms them in independent 16-value
    blocks, so one fill of the concatenation is bit-identical to per-tensor calls
    (tests/test_host_logic.py checks it); other tensors get their own [m, r] view, as the
    reference's per-tensor ``torch.randn(m, r)``.  ``Tensor.normal_`` on a view draws
    exactly what ``torch.randn`` of that shape draws, at a third of the Python overhead.
    """
    views = []
    fast = dtype == torch.float32
    off = run_start = run_len = 0
    for m in ms:
        n = int(m) * r
        if fast and n >= 16 and n % 16 == 0:
            if run_len == 0:
                run_start = off
            run_len += n
        else:
            if run_len:
                views.append(host[run_start:run_start + run_len])
                run_len = 0
            views.append(host[off:off + n].view(int(m), r))
        off += n
    if run_len:
        views.append(host[run_start:run_start + run_len])
    return views


def _torch_fill(seed: int, views) -> None:
    g = torch.Generator().manual_seed(int(seed))
    for v in views:
        v.normal_(generator=g)


def draw_host(seed: int, ms: Sequence[int], r: int, dtype: torch.dtype, pin: bool) -> torch.Tensor:
    """Concatenated [m_i][r] projections for one call, on the host (pinned if asked)."""
    total = sum(int(m) * r for m in ms)
    host = torch.empty(max(total, 1), dtype=dtype, pin_memory=pin)
    if total and native_ok(dtype):
        _draw_native(seed, _sizes(ms, r), len(ms), dtype, host)
    else:
        _torch_fill(seed, _fill_plan(host, ms, r, dtype))
    return host


class Slot:
    """A reusable pinned host buffer for one column list."""

    __slots__ = ("key", "host", "total", "sizes", "n", "dtype", "views", "event", "pending")

    def __init__(self, key, ms, r, dtype, pin):
        self.key = key
        self.total = sum(int(m) * r for m in ms)
        self.host = torch.empty(max(self.total, 1), dtype=dtype, pin_memory=pin)
        self.sizes = _sizes(ms, r)
        self.n = len(ms)
        self.dtype = dtype
        self.views = None if native_ok(dtype) else _fill_plan(self.host, ms, r, dtype)
        self.event = None      # reused event: recorded after an async copy out of `host`
        self.pending = False   # ... and that copy may still be running

    def copy_done(self) -> bool:
        """Whether the last H2D copy out of this buffer has completed (non-blocking)."""
        if self.pending and self.event.query():
            self.pending = False
        return not self.pending

    def fill(self, seed: int):
        """Draw on the calling thread."""
        if self.pending:  # the previous H2D copy from this buffer must be done
            self.event.synchronize()
            self.pending = False
        if not self.total:
            return self
        if self.views is None:
            _draw_native(seed, self.sizes, self.n, self.dtype, self.host)
        else:
            _torch_fill(seed, self.views)
        return self


class ProjectionSource:
    """Per-state projection provider with look-ahead prefetch into pooled pinned slots.

    ``get`` returns a filled :class:`Slot`; the caller copies ``slot.host`` to the device
    and hands the slot back with :meth:`release` (recording the copy's stream, so the
    buffer is refilled only after that copy completed).  Prefetched draws run on
    libarctopk's native thread pool (``arctopk_draw_submit`` / ``_wait``): no Python
    thread competes with the hook's thread for the GIL.
    """

    def __init__(self, r: int, depth: int = 8,
                 workers: int = int(os.environ.get("ARCTOPK_DRAW_THREADS", "4"))):
        self.r = r
        self.depth = depth
        self._pool = None  # native draw pool handle, created on first prefetch
        self._workers = workers
        self._pending: Dict[Tuple, Tuple[int, Slot]] = {}  # (seed, ms, dtype) -> (ticket, slot)
        self._stale: list = []  # (ticket, slot) of predictions that did not come true
        self._free: Dict[Tuple, list] = collections.defaultdict(list)
        self._lookahead: Optional[torch.Generator] = None
        self._future_seeds: collections.deque = collections.deque()
        self.hits = 0
        self.misses = 0

    # -- seed look-ahead -----------------------------------------------------
    def _sync_lookahead(self, rng: torch.Generator):
        """Prepare a clone of ``rng`` positioned where ``rng`` is now."""
        self._lookahead = torch.Generator()
        self._lookahead.set_state(rng.get_state())
        self._future_seeds.clear()

    PEEK_BATCH = 16  # seeds drawn per look-ahead refill (one randint of 16 = 16 of 1, in order)

    def _peek_seeds(self, n: int):
        if len(self._future_seeds) < n:
            self._future_seeds.extend(torch.randint(
                0, 1_000_000_000, (max(n - len(self._future_seeds), self.PEEK_BATCH),),
                generator=self._lookahead).tolist())
        if n == 1:
            return [self._future_seeds[0]]
        return list(self._future_seeds)[:n]

    def consume_seed(self, rng: torch.Generator) -> int:
        """Draw the call's seed from ``rng`` exactly as the reference (:254)."""
        seed = int(torch.randint(0, 1_000_000_000, (1,), generator=rng).item())
        if self._lookahead is None:
            self._sync_lookahead(rng)
        elif self._peek_seeds(1)[0] == seed:
            self._future_seeds.popleft()
        else:  # someone else drew from rng: resynchronise
            self._sync_lookahead(rng)
        return seed

    # -- slots --------------------------------------------------------------
    def _slot(self, ms: Tuple[int, ...], dtype: torch.dtype) -> Slot:
        """A free slot whose last H2D copy has completed, or a new one."""
        key = (tuple(ms), dtype)
        free = self._free[key]
        for i in range(len(free) - 1, -1, -1):
            if free[i].copy_done():
                return free.pop(i)
        return Slot(key, ms, self.r, dtype, pin=torch.cuda.is_available())

    def release(self, slot: Slot, stream=None):
        """Return a slot; with `stream`, after the work enqueued on it so far (the copy)."""
        if stream is not None:
            if slot.event is None:
                slot.event = torch.cuda.Event()
            slot.event.record(stream)
            slot.pending = True
        self._free[slot.key].append(slot)

    # -- drawing ------------------------------------------------------------
    def _native_pool(self):
        if self._pool is None:
            from allreducetopk_amd import _native as N
            h = ctypes.c_void_p()
            N.check(N.lib().arctopk_draw_pool_create(self._workers, ctypes.byref(h)),
                    "arctopk_draw_pool_create")
            self._pool = h.value
        return self._pool

    def get(self, seed: int, ms: Tuple[int, ...], dtype: torch.dtype) -> Slot:
        ent = self._pending.pop((seed, ms, dtype), None)
        if ent is not None:
            from allreducetopk_amd import _native as N
            ticket, slot = ent
            N.check(N.lib().arctopk_draw_wait(self._pool, ticket), "arctopk_draw_wait")
            self.hits += 1
            return slot
        self.misses += 1
        return self._slot(ms, dtype).fill(seed)

    def try_get(self, seed: int, ms: Tuple[int, ...], dtype: torch.dtype) -> Optional[Slot]:
        """The prefetched draw for (seed, ms, dtype) if it has already completed, else None
        (non-blocking; used to stage the next call's projections a call early)."""
        key = (seed, tuple(ms), dtype)
        ent = self._pending.get(key)
        if ent is None:
            return None
        from allreducetopk_amd import _native as N
        st = N.lib().arctopk_draw_poll(self._pool, ent[0])
        if st == 0:
            return None
        del self._pending[key]
        if st < 0:
            self._free[ent[1].key].append(ent[1])
            N.check(-st, "arctopk_draw_submit (prefetched draw)")
        self.hits += 1
        return ent[1]

    def peek_next_seed(self) -> Optional[int]:
        """The seed the next call will draw (None before the first call)."""
        if self._lookahead is None:
            return None
        return self._peek_seeds(1)[0]

    def _reap_stale(self):
        from allreducetopk_amd import _native as N
        keep = []
        for ticket, slot in self._stale:
            if N.lib().arctopk_draw_poll(self._pool, ticket) != 0:  # done (or failed)
                self.release(slot)
            else:
                keep.append((ticket, slot))
        self._stale = keep

    def prefetch(self, upcoming_ms: Sequence[Tuple[int, ...]], dtype: torch.dtype):
        """Schedule the projections of the next ``len(upcoming_ms)`` calls."""
        if self.depth <= 0 or not upcoming_ms or not native_ok(dtype):
            return  # (torch fallback draws: synchronously in get())
        from allreducetopk_amd import _native as N
        if self._stale:
            self._reap_stale()
        seeds = self._peek_seeds(min(self.depth, len(upcoming_ms)))
        live = set()
        for seed, ms in zip(seeds, upcoming_ms):
            if sum(ms) * self.r < SYNC_MAX_VALUES:  # drawn by get() on the caller's thread
                continue
            key = (seed, ms, dtype)
            live.add(key)
            if key not in self._pending:
                slot = self._slot(ms, dtype)
                ticket = N.lib().arctopk_draw_submit(self._native_pool(), int(seed),
                                                     N.DTYPE_CODE[dtype], slot.n, slot.sizes,
                                                     slot.host.data_ptr())
                if ticket < 0:
                    N.check(-ticket, "arctopk_draw_submit")
                self._pending[key] = (ticket, slot)
        for key in [k for k in self._pending if k not in live]:  # stale predictions
            self._stale.append(self._pending.pop(key))

    def reset(self):
        """Forget the seed look-ahead and pending draws (the rng was repositioned)."""
        self._stale.extend(self._pending.values())
        self._pending.clear()
        self._lookahead = None
        self._future_seeds.clear()

    def close(self):
        """Stop the native pool (queued draws are dropped, running ones finish)."""
        pool, self._pool = self._pool, None
        if pool is not None:
            from allreducetopk_amd import _native as N
            if N._lib is not None:
                N._lib.arctopk_draw_pool_destroy(pool)
        self._pending.clear()
        self._stale.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass
