"""A duck-typed stand-in for ``torch.distributed.GradBucket``.

``dist.GradBucket`` has no Python constructor, but the comm hooks of the
reference only call ``buffer()``, ``gradients()``, ``index()``, ``is_last()``
and ``parameters()`` on it (reference comm_hooks/group_topk_hook_no_reshape.py:
193-197, :208-209, :222; comm_hooks/utils.py:60, :71).  ``SyntheticBucket``
offers exactly that surface so a hook can be driven without DDP (bench.py,
tests, the golden-vector generator).

As in DDP's Reducer, ``gradients()`` are contiguous shaped *views* into the
flat ``buffer()`` in bucket order, so a hook that mutates the buffer in place
mutates the gradients too.
"""
from __future__ import annotations

from typing import List, Sequence

import torch


def bucket_numel(shapes: Sequence[Sequence[int]]) -> int:
    total = 0
    for s in shapes:
        n = 1
        for d in s:
            n *= int(d)
        total += n
    return total


class SyntheticBucket:
    """Flat gradient buffer + shaped views, with the GradBucket call surface."""

    def __init__(self, buffer: torch.Tensor, shapes: Sequence[Sequence[int]],
                 index: int = 0, is_last: bool = True, parameters=None):
        if buffer.dim() != 1 or not buffer.is_contiguous():
            raise ValueError("bucket buffer must be a contiguous 1-D tensor")
        if bucket_numel(shapes) != buffer.numel():
            raise ValueError("shapes do not cover the bucket buffer")
        self._buffer = buffer
        self._shapes = [tuple(int(d) for d in s) for s in shapes]
        self._index = int(index)
        self._is_last = bool(is_last)
        self._grads: List[torch.Tensor] = []
        off = 0
        for s in self._shapes:
            n = bucket_numel([s])
            self._grads.append(buffer[off:off + n].view(s))
            off += n
        self._params = parameters if parameters is not None else [
            torch.empty(0) for _ in self._shapes]

    @classmethod
    def zeros(cls, shapes, dtype=torch.float32, device="cpu", **kw):
        return cls(torch.zeros(bucket_numel(shapes), dtype=dtype, device=device), shapes, **kw)

    # --- GradBucket surface -------------------------------------------------
    def buffer(self) -> torch.Tensor:
        return self._buffer

    def gradients(self) -> List[torch.Tensor]:
        return self._grads

    def index(self) -> int:
        return self._index

    def is_last(self) -> bool:
        return self._is_last

    def parameters(self):
        return self._params

    def set_buffer(self, buffer: torch.Tensor) -> None:
        self._buffer.copy_(buffer)

    # --- helpers ------------------------------------------------------------
    @property
    def shapes(self):
        return list(self._shapes)
