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

Creating an RCCL communicator is collective over the group's ranks (it waits until all
of them have called it); the hook creates its communicators at its first compressed call,
which every rank reaches at the same point of the same backward, or
``GroupTopKState.init_exchange_comms()`` does it earlier (register_comm_hook_for_ddp_model
calls it on every rank).

Failure behaviour (the reference's collectives run on ProcessGroupNCCL under
``init_process_group(timeout=...)``, cifar10/run_cifar10.py:55-58, whose watchdog turns a hung
or failed collective into an error): the RCCL communicators are created non-blocking with the
process group's timeout (a rank that never joins: ``RuntimeError`` after the timeout instead of
a hang), and the library's watchdog aborts them when a collective stays pending past the
timeout or RCCL reports an asynchronous error; the hook then raises ``RuntimeError`` at its
next call (or at ``flush_exchange``).  The callback communicators inherit the torch backend's
own timeout (gloo raises from ``dist.all_reduce``; the hook re-raises that exception).

``Comm.wire`` is a measurement-only stand-in (world size 1, results unchanged) whose
all-reduce costs the local GPU what an N-rank ring all-reduce would.
"""
from __future__ import annotations

import ctypes
import logging
import os
from typing import Dict, Optional

import torch
import torch.distributed as dist

from allreducetopk_amd import _native as N

logger = logging.getLogger(__name__)

_DTYPE = {N.F32: torch.float32, N.BF16: torch.bfloat16}
DEFAULT_TIMEOUT_S = 600.0  # ProcessGroupNCCL's default when a group's own cannot be read


def group_timeout_s(group) -> float:
    """The timeout of `group` (init_process_group / new_group(timeout=...)); ARCTOPK_COMM_TIMEOUT_S
    overrides it."""
    env = os.environ.get("ARCTOPK_COMM_TIMEOUT_S")
    if env:
        return float(env)
    for dev in ("cuda", "cpu"):
        try:
            return float(group._get_backend(torch.device(dev)).options._timeout.total_seconds())
        except Exception:  # noqa: BLE001 -- backend without options / not registered for dev
            continue
    t = getattr(dist.distributed_c10d, "default_pg_nccl_timeout", None) or \
        getattr(dist.distributed_c10d, "default_pg_timeout", None)
    return float(t.total_seconds()) if t is not None else DEFAULT_TIMEOUT_S


def _store_key(store, tag: str, ranks) -> str:
    """A key every rank of the group derives alike for its n-th communicator of `tag`: each rank
    counts itself in at the store, and the creation of generation g completes only once all
    ranks have joined it, so every count of g precedes every count of g + 1 (a
    process-local counter diverges when processes create different numbers of communicators)."""
    base = f"arctopk_comm/{tag}/{'-'.join(map(str, ranks))}"
    gen = (int(store.add(base + "/count", 1)) - 1) // len(ranks)
    return f"{base}/{gen}"


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
    def rccl(cls, group, device: torch.device, tag: str, timeout_s: Optional[float] = None) -> "Comm":
        """An RCCL communicator over `group`'s ranks (collective over them), created non-blocking
        and watched against `timeout_s` (default: the group's timeout)."""
        L = N.lib()
        path = rccl_path().encode()
        ranks = dist.get_process_group_ranks(group)
        me = dist.get_rank(group)
        store = dist.distributed_c10d._get_default_store()
        key = _store_key(store, tag, ranks)
        if me == 0:
            uid = ctypes.create_string_buffer(128)
            N.check(L.arctopk_comm_unique_id(path, uid), "arctopk_comm_unique_id")
            store.set(key, uid.raw)
            raw = uid.raw
        else:
            raw = bytes(store.get(key))
        timeout_s = group_timeout_s(group) if timeout_s is None else float(timeout_s)
        h = ctypes.c_void_p()
        N.check(L.arctopk_comm_init_rccl_timeout(path, raw, len(ranks), me, device.index or 0,
                                                 max(1, int(timeout_s * 1000)), ctypes.byref(h)),
                f"arctopk_comm_init_rccl({tag}, {len(ranks)} ranks, timeout {timeout_s:g} s)")
        c = cls(h.value, group, "rccl")
        c.timeout_s = timeout_s
        return c

    # ---- emulated wire (measurement only) ---------------------------------------------
    @classmethod
    def wire(cls, device: torch.device, ranks: int = 8, busbw_gbs: float = 350.0,
             latency_us: float = 15.0, blocks: int = 64) -> "Comm":
        """World size 1 (buffers unchanged) at the local cost of a `ranks`-rank ring all-reduce
        paced to `busbw_gbs` (arctopk_comm_init_wire)."""
        h = ctypes.c_void_p()
        N.check(N.lib().arctopk_comm_init_wire(int(ranks), float(busbw_gbs), float(latency_us), int(blocks),
                                               torch.device(device).index or 0, ctypes.byref(h)),
                "arctopk_comm_init_wire")
        c = cls(h.value, None, "wire")
        c.wire_params = dict(ranks=int(ranks), busbw_gbs=float(busbw_gbs), latency_us=float(latency_us),
                             blocks=int(blocks))
        return c

    def status(self) -> int:
        """0, or the communicator's sticky failure (watchdog timeout, RCCL error, abort)."""
        return int(N.lib().arctopk_comm_status(self.handle)) if self.handle else 0

    def raise_if_failed(self, what: str = "ARC-TopK exchange") -> None:
        st = self.status()
        if st:
            N.check(st, f"{what} ({self.kind} communicator over {self.size} ranks)")

    def abort(self) -> None:
        if self.handle:
            N.lib().arctopk_comm_abort(self.handle)

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
        """A buffer the native step may all-reduce through the callback (by its address).  An
        exchange group's sketch / packed buffers are slices of its bucket's, and the first group's
        start at the bucket's own address: the longest buffer registered at an address is kept
        (every shorter one is its prefix), so both the group's and the whole bucket's all-reduce
        find theirs."""
        if self._fn is not None:
            old = self._views.get(t.data_ptr())
            if old is None or t.numel() > old.numel() or t.dtype != old.dtype:
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


def make_comms(group, device: torch.device, mode: str, wire: Optional[dict] = None):
    """(sketch communicator, packed-values communicator) over `group`.

    mode "separate": two communicators, so a bucket's sketch all-reduce never queues behind
    the previous bucket's packed all-reduce; "shared": one.
    `wire`: emulated-wire parameters (Comm.wire) instead of real communicators."""
    if wire is not None:
        packed = Comm.wire(device, **wire)
        sketch = Comm.wire(device, **wire) if mode == "separate" else packed
        logger.info("ARC-TopK exchange: emulated wire %s (%s sketch)", packed.wire_params, mode)
        return sketch, packed
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
