"""Communicators of the ARC-TopK exchange (libarctopk's ``arctopk_comm``).

The hook's two SUM all-reduces per bucket (the sketch and the packed values; reference
comm_hooks/group_topk_hook_no_reshape.py:58, :280) are issued by the native exchange step
(``arctopk_exchange_step``) itself, in the same host call as the kernels around them:

- on an ``nccl`` process group (RCCL on ROCm) through RCCL communicators this library
  owns, created over the group's ranks with the id exchanged through the default store;
  RCCL is the librccl.so torch already loaded (one RCCL per process);
- on any other backend (gloo: the CPU tests, two ranks sharing one GPU) through a callback
  into ``torch.distributed.all_reduce`` on the group, so the very same native
  orchestration runs in those tests.

Creating an RCCL communicator is collective over the group's ranks (it blocks until all
of them have called it); the hook creates its communicators at its first compressed call,
which every rank reaches at the same point of the same backward, or
``GroupTopKState.init_exchange_comms()`` does it earlier (register_comm_hook_for_ddp_model
calls it on every rank).
"""
from __future__ import annotations

import ctypes
import itertools
import logging
import os
from typing import Dict, Optional

import torch
import torch.distributed as dist

from allreducetopk_amd import _native as N

logger = logging.getLogger(__name__)

_DTYPE = {N.F32: torch.float32, N.BF16: torch.bfloat16}
_serial = itertools.count()


def rccl_path() -> str:
    """The RCCL library torch loaded (libtorch_hip links it), else ROCm's."""
    try:
        with open("/proc/self/maps") as fh:
            for line in fh:
                p = line.rsplit(None, 1)[-1]
                if os.path.basename(p).startswith("librccl.so"):
                    return p
    except OSError:
        pass
    cand = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return cand if os.path.exists(cand) else "librccl.so.1"


class Comm:
    """One arctopk_comm over the ranks of `group`."""

    def __init__(self, handle: int, group, kind: str):
        self.handle = handle
        self.group = group
        self.kind = kind
        self.size = N.lib().arctopk_comm_size(handle)
        self._fn = None          # the ctypes callback (kept alive with the communicator)
        self._views: Dict[int, torch.Tensor] = {}
        self._streams: Dict[int, torch.cuda.Stream] = {}
        self.error: Optional[BaseException] = None

    # ---- RCCL ---------------------------------------------------------------------
    @classmethod
    def rccl(cls, group, device: torch.device, tag: str) -> "Comm":
        """An RCCL communicator over `group`'s ranks (collective over them)."""
        L = N.lib()
        path = rccl_path().encode()
        ranks = dist.get_process_group_ranks(group)
        me = dist.get_rank(group)
        key = f"arctopk_comm/{tag}/{'-'.join(map(str, ranks))}/{next(_serial)}"
        store = dist.distributed_c10d._get_default_store()
        if me == 0:
            uid = ctypes.create_string_buffer(128)
            N.check(L.arctopk_comm_unique_id(path, uid), "arctopk_comm_unique_id")
            store.set(key, uid.raw)
            raw = uid.raw
        else:
            raw = bytes(store.get(key))
        h = ctypes.c_void_p()
        N.check(L.arctopk_comm_init_rccl(path, raw, len(ranks), me, device.index or 0, ctypes.byref(h)),
                f"arctopk_comm_init_rccl({tag}, {len(ranks)} ranks)")
        return cls(h.value, group, "rccl")

    # ---- callback (any torch.distributed backend) ----------------------------------
    @classmethod
    def callback(cls, group) -> "Comm":
        obj = cls.__new__(cls)
        fn = N.ALLREDUCE_FN(obj._allreduce)
        h = ctypes.c_void_p()
        N.check(N.lib().arctopk_comm_init_callback(fn, None, group.size(), dist.get_rank(group),
                                                   ctypes.byref(h)), "arctopk_comm_init_callback")
        cls.__init__(obj, h.value, group, "callback")
        obj._fn = fn
        return obj

    def register(self, t: torch.Tensor) -> None:
        """A buffer the native step may all-reduce through the callback (by its address)."""
        if self._fn is not None:
            self._views[t.data_ptr()] = t

    def known_stream(self, s: "torch.cuda.Stream") -> None:
        """A stream the native step may hand the callback (found by its raw handle)."""
        self._streams[s.cuda_stream] = s

    def _allreduce(self, _ctx, buf, count, dtype, stream) -> int:
        stream = stream or 0  # ctypes hands a null handle (the null stream) over as None
        try:
            t = self._views[buf]
            if t.dtype != _DTYPE[dtype] or count > t.numel():
                raise RuntimeError("exchange all-reduce of an unregistered view")
            if not t.is_cuda:  # host buffers (CPU tests of the plumbing): no stream
                dist.all_reduce(t[:count], group=self.group)
                return 0
            if torch.cuda.current_stream(t.device).cuda_stream == stream:
                dist.all_reduce(t[:count], group=self.group)
                return 0
            s = self._streams.get(stream)
            if s is None:
                s = torch.cuda.ExternalStream(stream, device=t.device)
                self._streams[stream] = s
            with torch.cuda.stream(s):
                dist.all_reduce(t[:count], group=self.group)
            return 0
        except BaseException as e:  # noqa: BLE001 -- re-raised by the hook after the native call
            self.error = e
            return 1

    def check(self, status: int, what: str) -> None:
        """Raise the callback's own exception if it failed, else the native status."""
        if status and self.error is not None:
            e, self.error = self.error, None
            raise e
        N.check(status, what)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and N._lib is not None:
            try:
                N._lib.arctopk_comm_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None


def make_comms(group, device: torch.device, mode: str):
    """(sketch communicator, packed-values communicator) over `group`.

    mode "separate": two communicators, so a bucket's sketch all-reduce never queues behind
    the previous bucket's packed all-reduce; "shared": one."""
    backend = dist.get_backend(group)
    if "nccl" in str(backend):
        packed = Comm.rccl(group, device, "packed")
        sketch = Comm.rccl(group, device, "sketch") if mode == "separate" else packed
    else:
        packed = Comm.callback(group)
        if mode == "separate":
            sketch = Comm.callback(dist.new_group(ranks=dist.get_process_group_ranks(group)))
        else:
            sketch = packed
    logger.info("ARC-TopK exchange: %s communicators over %d ranks (%s sketch)", packed.kind,
                packed.size, mode)
    return sketch, packed
