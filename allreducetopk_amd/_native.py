"""ctypes binding of libarctopk.so (declared in include/arctopk.h).

The shipped hooks run only through this library: if it is missing or cannot
be loaded, ``lib()`` raises -- there is no CPU or eager-torch fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_uint64, c_void_p

import torch

PKG = os.path.dirname(os.path.abspath(__file__))
# ARCTOPK_LIB: an explicitly named library (A/B tuning variants) skips the source-hash check
LIB_OVERRIDE = os.environ.get("ARCTOPK_LIB")
LIB_PATH = LIB_OVERRIDE or os.path.join(PKG, "lib", "libarctopk.so")

EF_NONE, EF14, EF21 = 0, 1, 2
EF_CODE = {"noef": EF_NONE, "ef14": EF14, "ef21": EF21}
EINVAL = 1001  # ARCTOPK_EINVAL
SEG_RAW, SEG_SKETCH = 0, 1
F32 = 0
BF16 = 1
DTYPE_CODE = {torch.float32: F32, torch.bfloat16: BF16}  # bucket dtype -> ARCTOPK_F32 / _BF16

STATUS = {1001: "invalid argument", 1002: "ND tensor numel not divisible by 2*t^2",
          1003: "unsupported dtype", 1004: "empty tensor", 1005: "RCCL library not loadable",
          1006: "communicator timed out (a collective or the communicator's creation outlived the "
                "process group's timeout; every RCCL communicator of the library was aborted)",
          1007: "communicator aborted"}
ETIMEOUT, EABORTED = 1006, 1007
ECOMM = 1100  # + ncclResult_t
NMARKS = 8    # ARCTOPK_MARK_*: phase markers of a step
MARKS = {"start": 0, "draw": 1, "encode": 2, "sketch_allreduce": 3, "select": 4, "pack": 5,
         "packed_allreduce": 6, "decode": 7}
# the exchange's all-reduce callback: fn(ctx, buf, count, dtype, stream) -> status
ALLREDUCE_FN = ctypes.CFUNCTYPE(c_int32, c_void_p, c_void_p, c_int64, c_int32, c_void_p)


class PlanInfo(ctypes.Structure):
    _fields_ = [("numel", c_int64), ("sketch_len", c_int64), ("v_len", c_int64),
                ("packed_len", c_int64), ("sel_rows", c_int64), ("rows_total", c_int64),
                ("nseg", c_int32), ("r", c_int32), ("values_len", c_int64)]


class Segment(ctypes.Structure):
    _fields_ = [("offset", c_int64), ("n", c_int64), ("m", c_int64), ("k_rows", c_int64),
                ("sketch_off", c_int64), ("v_off", c_int64), ("packed_off", c_int64),
                ("row_off", c_int64), ("sel_off", c_int64), ("kind", c_int32), ("pad", c_int32)]


_SIGS = {
    "arctopk_plan_create": (c_int32, [POINTER(c_int64), POINTER(c_int32), c_int32, c_int32, c_double,
                                      c_int32, c_int32, POINTER(c_void_p)]),
    "arctopk_plan_destroy": (c_int32, [c_void_p]),
    "arctopk_plan_describe": (c_int32, [POINTER(c_int64), POINTER(c_int32), c_int32, c_int32, c_double,
                                        c_void_p, POINTER(PlanInfo)]),
    "arctopk_plan_query": (c_int32, [c_void_p, POINTER(PlanInfo)]),
    "arctopk_plan_group": (c_int32, [c_void_p, c_int32, c_int32, POINTER(c_void_p)]),
    "arctopk_plan_segment": (c_int32, [c_void_p, c_int32, POINTER(Segment)]),
    "arctopk_encode": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                 c_void_p]),
    "arctopk_select": (c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "arctopk_select_draw": (c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                      c_uint64, c_void_p, c_void_p]),
    "arctopk_plan_bind": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "arctopk_step": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                               c_uint64, c_void_p, c_uint64, c_void_p, c_void_p]),
    "arctopk_comm_unique_id": (c_int32, [c_char_p, c_void_p]),
    "arctopk_comm_init_rccl": (c_int32, [c_char_p, c_char_p, c_int32, c_int32, c_int32, POINTER(c_void_p)]),
    "arctopk_comm_init_rccl_timeout": (c_int32, [c_char_p, c_char_p, c_int32, c_int32, c_int32, c_int64,
                                                 POINTER(c_void_p)]),
    "arctopk_comm_status": (c_int32, [c_void_p]),
    "arctopk_comm_abort": (c_int32, [c_void_p]),
    "arctopk_comm_init_callback": (c_int32, [ALLREDUCE_FN, c_void_p, c_int32, c_int32, POINTER(c_void_p)]),
    "arctopk_comm_init_wire": (c_int32, [c_int32, c_double, c_double, c_int32, c_int32, POINTER(c_void_p)]),
    "arctopk_comm_destroy": (c_int32, [c_void_p]),
    "arctopk_comm_size": (c_int32, [c_void_p]),
    "arctopk_comm_allreduce": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p]),
    "arctopk_exchange_step": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                        c_uint64, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                        c_void_p, c_void_p, c_void_p]),
    "arctopk_exchange_trail": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                         c_uint64, c_void_p, c_void_p]),
    "arctopk_exchange_finish": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "arctopk_row_energy": (c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "arctopk_pack": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                               c_void_p]),
    "arctopk_decode": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                 c_void_p]),
    "arctopk_pack_segments": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_int32,
                                        c_void_p, c_void_p, c_void_p, c_void_p]),
    "arctopk_decode_segments": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_int32,
                                          c_int32, c_void_p, c_void_p, c_void_p]),
    "arctopk_sparse_workspace_bytes": (c_int64, [c_int32, POINTER(c_int64)]),
    "arctopk_topk_select": (c_int32, [c_void_p, c_int32, POINTER(c_int64), POINTER(c_int64),
                                      POINTER(c_int64), POINTER(c_int64), c_void_p, c_void_p, c_void_p,
                                      c_int32, c_int32, c_void_p]),
    "arctopk_ef14_fold": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p]),
    "arctopk_randk_select": (c_int32, [c_void_p, c_int32, POINTER(c_int64), POINTER(c_int64),
                                       POINTER(c_int64), POINTER(c_int64), c_uint64, c_void_p, c_void_p,
                                       c_void_p, c_int32, c_int32, c_void_p]),
    "arctopk_topk_select_ef14": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, POINTER(c_int64),
                                           POINTER(c_int64), POINTER(c_int64), POINTER(c_int64), c_void_p,
                                           c_void_p, c_void_p, c_int32, c_void_p]),
    "arctopk_randk_select_ef14": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, POINTER(c_int64),
                                            POINTER(c_int64), POINTER(c_int64), POINTER(c_int64), c_uint64,
                                            c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    "arctopk_sparse_gather": (c_int32, [c_void_p, c_int32, POINTER(c_int64), POINTER(c_int64),
                                        POINTER(c_int64), c_void_p, c_void_p, c_int32, c_void_p]),
    "arctopk_sparse_residual": (c_int32, [c_void_p, c_int32, POINTER(c_int64), POINTER(c_int64),
                                          POINTER(c_int64), c_void_p, c_void_p, c_int32, c_float, c_int32,
                                          c_void_p]),
    "arctopk_sparse_decode": (c_int32, [c_void_p, c_int64, c_int32, POINTER(c_int64), POINTER(c_int64),
                                        POINTER(c_int64), c_int64, c_void_p, c_void_p, c_int32, c_int32,
                                        c_int32, c_void_p, c_float, c_int32, c_void_p]),
    "arctopk_ef_apply": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p]),
    "arctopk_draw_bf16_normal": (c_int32, [c_uint64, c_int64, c_void_p]),
    "arctopk_draw_normal": (c_int32, [c_uint64, c_int32, c_int32, POINTER(c_int64), c_void_p]),
    "arctopk_draw_pool_create": (c_int32, [c_int32, POINTER(c_void_p)]),
    "arctopk_draw_pool_destroy": (c_int32, [c_void_p]),
    "arctopk_draw_submit": (c_int64, [c_void_p, c_uint64, c_int32, c_int32, POINTER(c_int64), c_void_p]),
    "arctopk_draw_wait": (c_int32, [c_void_p, c_int64]),
    "arctopk_draw_poll": (c_int32, [c_void_p, c_int64]),
    "arctopk_memcpy_h2d_async": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    "arctopk_event_create": (c_int32, [POINTER(c_void_p)]),
    "arctopk_event_destroy": (c_int32, [c_void_p]),
    "arctopk_event_record": (c_int32, [c_void_p, c_void_p]),
    "arctopk_event_wait": (c_int32, [c_void_p, c_void_p]),
    "arctopk_event_query": (c_int32, [c_void_p]),
    "arctopk_event_create_timed": (c_int32, [POINTER(c_void_p)]),
    "arctopk_event_elapsed_ms": (c_int32, [POINTER(ctypes.c_float), c_void_p, c_void_p]),
    "arctopk_round_bf16": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    "arctopk_diag_host_times": (c_int32, [c_void_p, c_int32, c_void_p]),
    "arctopk_draw_projections": (c_int32, [c_void_p, c_uint64, c_void_p, c_void_p]),
    "arctopk_plan_philox_advance": (c_int32, [c_void_p, POINTER(c_uint64)]),
    "arctopk_version": (c_char_p, []),
}

EXPORTS = tuple(_SIGS)

_lib = None
_lock = threading.Lock()


class NativeLibraryMissing(ImportError):
    pass


def lib() -> ctypes.CDLL:
    """Load libarctopk.so once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"libarctopk.so not found at {LIB_PATH}: build it with "
                "`python -m allreducetopk_amd.build` (hipcc, gfx950). There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if not LIB_OVERRIDE:
            _check_build(L)
        _lib = L
    return _lib


class StaleNativeLibrary(ImportError):
    pass


def _check_build(L) -> None:
    """Refuse a library built from other sources than the ones in this tree (the hash
    the build embedded in arctopk_version() vs the hash of csrc/ + arctopk.h now)."""
    from allreducetopk_amd import build as B
    ver = L.arctopk_version().decode()
    m = B.HASH_RE.search(ver.encode())
    if not os.path.isdir(B.CSRC):  # sources not shipped: nothing to compare against
        return
    want = B.source_hash()
    if m is None or m.group(1).decode() != want:
        raise StaleNativeLibrary(
            f"{LIB_PATH} was built from other sources ({ver!r}; sources hash {want}): rebuild "
            "with `python -m allreducetopk_amd.build` (or name a variant via ARCTOPK_LIB)")


def check(status: int, what: str) -> None:
    if status:
        st = int(status)
        msg = STATUS.get(st, f"RCCL error {st - ECOMM}" if ECOMM <= st < ECOMM + 100 else f"hip error {st}")
        raise RuntimeError(f"{what} failed: {msg} (status {int(status)})")


def i64_array(values):
    arr = (c_int64 * len(values))(*[int(v) for v in values])
    return arr


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


class DeviceEvent:
    """A device-scope HIP event (libarctopk's arctopk_event_*): ordering between this
    process's streams on one GPU without torch's system-scope release."""

    __slots__ = ("handle",)

    def __init__(self, timing: bool = False):
        h = ctypes.c_void_p()
        if timing:
            check(lib().arctopk_event_create_timed(ctypes.byref(h)), "arctopk_event_create_timed")
        else:
            check(lib().arctopk_event_create(ctypes.byref(h)), "arctopk_event_create")
        self.handle = h.value

    def elapsed_time(self, end: "DeviceEvent") -> float:
        """Milliseconds from this record to `end`'s (both timed events, both complete)."""
        ms = ctypes.c_float()
        check(lib().arctopk_event_elapsed_ms(ctypes.byref(ms), self.handle, end.handle),
              "arctopk_event_elapsed_ms")
        return float(ms.value)

    def record(self, stream: int) -> None:
        check(lib().arctopk_event_record(self.handle, stream), "arctopk_event_record")

    def wait(self, stream: int) -> None:
        """Make `stream` wait for the last record."""
        check(lib().arctopk_event_wait(stream, self.handle), "arctopk_event_wait")

    def query(self) -> bool:
        st = lib().arctopk_event_query(self.handle)
        if st not in (0, 1):
            check(st, "arctopk_event_query")
        return st == 0

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib is not None:
            try:
                _lib.arctopk_event_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None
