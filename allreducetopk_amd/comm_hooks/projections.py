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


def draw_host(seed: int, ms: Sequence[int], r: int, dtype: torch.dtype, pin: bool) -> torch.Tensor:
    """Concatenated [m_i][r] projections for one call, on the host (pinned if asked).

    Consecutive tensors whose m*r is a multiple of 16 are drawn by ONE randn call:
    torch's CPU normal fill draws all uniforms in stream order and transforms them in
    independent 16-value blocks, so the concatenation is bit-identical to per-tensor
    calls (tests/test_host_logic.py checks it); other tensors get their own call,
    exactly as the reference's per-tensor ``torch.randn(m, r)``.
    """
    total = sum(int(m) * r for m in ms)
    host = torch.empty(max(total, 1), dtype=dtype, pin_memory=pin)
    g = torch.Generator().manual_seed(int(seed))
    fast = dtype == torch.float32
    off = 0
    run_start = run_len = 0
    for m in ms:
        n = int(m) * r
        if fast and n >= 16 and n % 16 == 0:
            if run_len == 0:
                run_start = off
            run_len += n
        else:
            if run_len:
                torch.randn(run_len, generator=g, dtype=dtype, out=host[run_start:run_start + run_len])
                run_len = 0
            torch.randn(int(m), r, generator=g, dtype=dtype, out=host[off:off + n].view(int(m), r))
        off += n
    if run_len:
        torch.randn(run_len, generator=g, dtype=dtype, out=host[run_start:run_start + run_len])
    return host


class ProjectionSource:
    """Per-state projection provider with look-ahead prefetch."""

    def __init__(self, r: int, depth: int = 8, workers: int = 8):
        self.r = r
        self.depth = depth
        self._pool: Optional[ThreadPoolExecutor] = None
        self._workers = workers
        self._pending: Dict[Tuple, object] = {}
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

    # -- drawing ------------------------------------------------------------
    def get(self, seed: int, ms: Tuple[int, ...], dtype: torch.dtype) -> torch.Tensor:
        key = (seed, ms, dtype)
        with self._lock:
            fut = self._pending.pop(key, None)
        if fut is not None:
            self.hits += 1
            return fut.result()
        self.misses += 1
        return draw_host(seed, ms, self.r, dtype, pin=torch.cuda.is_available())

    def prefetch(self, upcoming_ms: Sequence[Tuple[int, ...]], dtype: torch.dtype):
        """Schedule the projections of the next ``len(upcoming_ms)`` calls."""
        if self.depth <= 0 or not upcoming_ms:
            return
        if self._pool is None:
            self._pool = ThreadPoolExecutor(max_workers=self._workers,
                                            thread_name_prefix="arctopk-proj")
        seeds = self._peek_seeds(min(self.depth, len(upcoming_ms)))
        pin = torch.cuda.is_available()
        with self._lock:
            live = set()
            for seed, ms in zip(seeds, upcoming_ms):
                key = (seed, ms, dtype)
                live.add(key)
                if key not in self._pending:
                    self._pending[key] = self._pool.submit(draw_host, seed, ms, self.r, dtype, pin)
            for key in [k for k in self._pending if k not in live]:  # stale predictions
                self._pending.pop(key)

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
