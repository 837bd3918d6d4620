"""Source of the per-call Gaussian projections V of ARC-TopK.

Reference semantics (comm_hooks/group_topk_hook_no_reshape.py:254-255, :49, :79):
per bucket call a seed is drawn from ``state.rng`` (a CPU generator), the global
RNG is reseeded with it, and ``torch.randn(m, r)`` is drawn once per 2-D/ND
tensor in bucket order.  V is drawn here with torch's CPU generator (mt19937 +
torch's normal transform): a private ``torch.Generator`` seeded with the same
seed yields exactly that stream, so the projections -- and therefore the
selected rows -- are those of the reference on CPU bit for bit.

Drawing V for a 16 x [2048, 2048] bucket costs ~0.5 ms of host time, more than
the whole GPU codec.  V depends only on (seed, column counts), and the seed
sequence is deterministic, so a small thread pool draws the projections of the
*next* calls while the current one runs (``depth`` calls ahead).  A miss (first
call, changed bucket order) draws synchronously; hits and misses return the
same values.
"""
from __future__ import annotations

import collections
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Optional, Sequence, Tuple

import torch


# ---- bf16 projections -----------------------------------------------------------------
# torch's CPU normal_ on a bf16 tensor (the reference's torch.randn(m, r, dtype=bfloat16))
# runs a scalar BFloat16 loop, ~8x slower than the fp32 path and slower than the device
# codec.  For every tensor with m*r a multiple of 16 the values are a table function of
# 8-bit mt19937 uniforms; libarctopk's host routine arctopk_draw_bf16_normal computes them
# bit-identically (projection.cpp; tests/test_host_logic.py pins it against torch) and,
# called through ctypes, without holding the GIL.


def bf16_fast_ok(ms: Sequence[int], r: int) -> bool:
    """Every tensor's draw is whole 16-blocks (no tail recompute, no scalar path)."""
    return all(int(m) * r >= 16 and (int(m) * r) % 16 == 0 for m in ms)


def draw_bf16_into(seed: int, out: torch.Tensor) -> None:
    """Fill the contiguous bf16 CPU tensor `out` (numel % 16 == 0) with the stream."""
    from allreducetopk_amd import _native as N
    N.check(N.lib().arctopk_draw_bf16_normal(int(seed), out.numel(), out.data_ptr()),
            "arctopk_draw_bf16_normal")


def _fill_plan(host: torch.Tensor, ms: Sequence[int], r: int, dtype: torch.dtype):
    """Views of `host` that one generator pass fills in the reference's stream order.

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


def draw_host(seed: int, ms: Sequence[int], r: int, dtype: torch.dtype, pin: bool) -> torch.Tensor:
    """Concatenated [m_i][r] projections for one call, on the host (pinned if asked)."""
    total = sum(int(m) * r for m in ms)
    host = torch.empty(max(total, 1), dtype=dtype, pin_memory=pin)
    if dtype == torch.bfloat16 and total and bf16_fast_ok(ms, r):
        draw_bf16_into(seed, host[:total])
        return host
    g = torch.Generator().manual_seed(int(seed))
    for v in _fill_plan(host, ms, r, dtype):
        v.normal_(generator=g)
    return host


class Slot:
    """A reusable pinned host buffer for one column list, with its fill views."""

    __slots__ = ("key", "host", "views", "event", "pending", "fast")

    def __init__(self, key, ms, r, dtype, pin):
        self.key = key
        total = sum(int(m) * r for m in ms)
        self.host = torch.empty(max(total, 1), dtype=dtype, pin_memory=pin)
        self.views = _fill_plan(self.host, ms, r, dtype)
        # bf16: the native table-driven draw (bit-identical to torch's normal_)
        self.fast = self.host[:total] if dtype == torch.bfloat16 and total and bf16_fast_ok(ms, r) else None
        self.event = None      # reused event: recorded after an async copy out of `host`
        self.pending = False   # ... and that copy may still be running

    def fill(self, seed: int):
        if self.pending:  # the previous H2D copy from this buffer must be done
            self.event.synchronize()
            self.pending = False
        if self.fast is not None:
            draw_bf16_into(seed, self.fast)
            return self
        g = torch.Generator().manual_seed(int(seed))
        for v in self.views:
            v.normal_(generator=g)
        return self


class ProjectionSource:
    """Per-state projection provider with look-ahead prefetch into pooled pinned slots.

    ``get`` returns a filled :class:`Slot`; the caller copies ``slot.host`` to the device
    and hands the slot back with :meth:`release` (recording the copy's stream, so the
    buffer is refilled only after that copy completed).
    """

    def __init__(self, r: int, depth: int = 8, workers: int = 8):
        self.r = r
        self.depth = depth
        self._pool: Optional[ThreadPoolExecutor] = None
        self._workers = workers
        self._pending: Dict[Tuple, object] = {}
        self._free: Dict[Tuple, list] = collections.defaultdict(list)
        self._lock = threading.Lock()
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

    def _peek_seeds(self, n: int):
        while len(self._future_seeds) < n:
            s = int(torch.randint(0, 1_000_000_000, (1,), generator=self._lookahead).item())
            self._future_seeds.append(s)
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
        key = (tuple(ms), dtype)
        with self._lock:
            free = self._free[key]
            if free:
                return free.pop()
        return Slot(key, ms, self.r, dtype, pin=torch.cuda.is_available())

    def release(self, slot: Slot, stream=None):
        """Return a slot; with `stream`, after the work enqueued on it so far (the copy)."""
        if stream is not None:
            if slot.event is None:
                slot.event = torch.cuda.Event()
            slot.event.record(stream)
            slot.pending = True
        with self._lock:
            self._free[slot.key].append(slot)

    # -- drawing ------------------------------------------------------------
    def get(self, seed: int, ms: Tuple[int, ...], dtype: torch.dtype) -> Slot:
        key = (seed, ms, dtype)
        with self._lock:
            fut = self._pending.pop(key, None)
        if fut is not None:
            self.hits += 1
            return fut.result()
        self.misses += 1
        return self._slot(ms, dtype).fill(seed)

    def prefetch(self, upcoming_ms: Sequence[Tuple[int, ...]], dtype: torch.dtype):
        """Schedule the projections of the next ``len(upcoming_ms)`` calls."""
        if self.depth <= 0 or not upcoming_ms:
            return
        if self._pool is None:
            self._pool = ThreadPoolExecutor(max_workers=self._workers,
                                            thread_name_prefix="arctopk-proj")
        seeds = self._peek_seeds(min(self.depth, len(upcoming_ms)))
        stale = []
        with self._lock:
            live = set()
            for seed, ms in zip(seeds, upcoming_ms):
                key = (seed, ms, dtype)
                live.add(key)
                if key not in self._pending:
                    self._pending[key] = self._pool.submit(
                        lambda sd=seed, m_=ms: self._slot(m_, dtype).fill(sd))
            for key in [k for k in self._pending if k not in live]:  # stale predictions
                stale.append(self._pending.pop(key))
        for fut in stale:  # recycle their slots once drawn
            fut.add_done_callback(lambda f: self.release(f.result()) if not f.cancelled()
                                  and f.exception() is None else None)

    def reset(self):
        """Forget the seed look-ahead and pending draws (the rng was repositioned)."""
        with self._lock:
            self._pending.clear()
        self._lookahead = None
        self._future_seeds.clear()

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=False, cancel_futures=True)
            self._pool = None
