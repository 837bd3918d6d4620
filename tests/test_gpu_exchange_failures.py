"""Exchange robustness on one MI355X: communicator failures become RuntimeError, Futures of
direct callers are complete on return, and the emulated wire leaves results unchanged.

- A 2-rank RCCL communicator whose second rank never joins must fail within the timeout with
  RuntimeError, not hang (the reference's collectives run on ProcessGroupNCCL with a 30 s
  timeout: /root/reference/cifar10/run_cifar10.py:55-58; SURVEY.md 8(b) error convention).
- An aborted communicator makes the next hook call raise RuntimeError (sticky error).
- Without DDP, a hook's Future is complete when the hook returns (torch.futures.wait_all on
  the non-last buckets neither hangs nor sees stale data); with deferral the
  outputs are the same bits.
- The emulated-wire communicator (measurement only) leaves every output bit-identical.
"""
import ctypes
import time

import pytest
import torch

from parity import assert_bitwise, ensure_group

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SHAPES = {2: [[256, 512], [96, 40], [10]],
          1: [[130, 2048], [16, 8, 3, 3], [7], [40, 16]],
          0: [[64, 70], [16, 8, 1, 1], [1000], [8, 8, 5, 5]]}


def _grad(b, step):
    from allreducetopk_amd.bucket import bucket_numel
    return torch.randn(bucket_numel(SHAPES[b]), generator=torch.Generator().manual_seed(1000 * step + b))


def test_rccl_comm_creation_times_out_when_a_rank_never_joins():
    from allreducetopk_amd import _native as N
    from allreducetopk_amd import exchange as X
    torch.cuda.init()
    L = N.lib()
    path = X.rccl_path().encode()
    uid = ctypes.create_string_buffer(128)
    N.check(L.arctopk_comm_unique_id(path, uid), "arctopk_comm_unique_id")
    h = ctypes.c_void_p()
    t0 = time.time()
    st = L.arctopk_comm_init_rccl_timeout(path, uid.raw, 2, 0, 0, 3000, ctypes.byref(h))
    dt = time.time() - t0
    assert st == N.ETIMEOUT, f"status {st}"
    assert 2.5 < dt < 30.0, f"gave up after {dt:.1f} s (timeout 3 s)"
    with pytest.raises(RuntimeError, match="timed out"):
        N.check(st, "arctopk_comm_init_rccl_timeout")
    # the process and its device stay usable
    x = torch.ones(4, device=DEV)
    assert float((x + 1).sum()) == 8.0


def _state(force_exchange, defer=None, ef="ef14", seed=5):
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback=ef,
                          seed=seed)
    st.force_exchange = force_exchange
    st.defer_decode = defer
    return st


def _backward(st, step):
    from allreducetopk_amd.bucket import SyntheticBucket
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    futs, bufs = [], {}
    for b in (2, 1, 0):
        bufs[b] = _grad(b, step).to(DEV)
        futs.append(G.group_topk_hook(st, SyntheticBucket(bufs[b], SHAPES[b], index=b, is_last=(b == 0))))
    return futs, bufs


def test_aborted_communicator_makes_the_hook_raise():
    ensure_group("nccl")
    st = _state(force_exchange=True, defer=True)
    for f in _backward(st, 0)[0]:
        f.wait()
    torch.cuda.synchronize()
    sk, pk = st._comms[2], st._comms[3]
    assert sk.kind == "rccl" and sk.status() == 0 and pk.status() == 0
    pk.abort()
    from allreducetopk_amd.bucket import SyntheticBucket
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    with pytest.raises(RuntimeError, match="aborted"):
        G.group_topk_hook(st, SyntheticBucket(_grad(2, 1).to(DEV), SHAPES[2], index=2, is_last=False))
    torch.cuda.synchronize()


@pytest.mark.parametrize("force_exchange", [False, True])
def test_direct_caller_futures_complete_on_return(force_exchange):
    """A caller that is not DDP (SyntheticBucket, defer_decode left at None) gets a complete
    Future from every call: wait_all on the non-last buckets returns at once, with the same
    bits as the DDP-style deferred run."""
    ensure_group("nccl")
    outs = {}
    for defer in (None, True):
        st = _state(force_exchange, defer=defer)
        for step in range(3):
            futs, bufs = _backward(st, step)
            if defer is None:
                assert all(f.done() for f in futs), "a direct caller's Future is pending"
                torch.futures.wait_all(futs[:2])  # (C++ wait: would hang on a deferred Future)
            for f in futs:
                f.wait()
            torch.cuda.synchronize()
        outs[defer] = ({b: t.cpu() for b, t in bufs.items()}, {b: e.cpu() for b, e in st.error_dict.items()})
    for b in SHAPES:
        assert_bitwise(outs[None][0][b], outs[True][0][b], f"bucket {b} output, direct vs deferred")
        assert_bitwise(outs[None][1][b], outs[True][1][b], f"bucket {b} residual, direct vs deferred")


@pytest.mark.parametrize("ef", ["ef14", "ef21"])
def test_emulated_wire_leaves_results_unchanged(ef):
    """Forced exchange over emulated-wire communicators (an 8-rank ring's local HBM traffic,
    paced to 350 GB/s) gives the bits of the forced exchange over one-rank RCCL."""
    ensure_group("nccl")
    outs = {}
    for wire in (None, dict(ranks=8, busbw_gbs=350.0, latency_us=15.0, blocks=32)):
        st = _state(force_exchange=True, defer=True, ef=ef, seed=9)
        st.emulate_wire = wire
        for step in range(3):
            futs, bufs = _backward(st, step)
            for f in futs:
                f.wait()
        torch.cuda.synchronize()
        if wire is not None:
            assert st._comms[3].kind == "wire"
        outs[wire is None] = ({b: t.cpu() for b, t in bufs.items()},
                              {b: e.cpu() for b, e in st.error_dict.items()},
                              {b: e.cpu() for b, e in st.global_error_dict.items()})
    for i, what in enumerate(("output", "E", "gE")):
        for b in outs[True][i]:
            assert_bitwise(outs[False][i][b], outs[True][i][b], f"bucket {b} {what}, wire vs RCCL")


_WATCHDOG_CHILD = r"""
import ctypes, os, sys, time
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
from parity import ensure_group
ensure_group("nccl")
from allreducetopk_amd import _native as N
from allreducetopk_amd.bucket import SyntheticBucket
from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback="ef14")
st.force_exchange = True
st.defer_decode = True
shapes = [[256, 512], [96, 40], [10]]
def call(last):
    x = torch.randn(256 * 512 + 96 * 40 + 10, device="cuda:0")
    return G.group_topk_hook(st, SyntheticBucket(x, shapes, index=0, is_last=last))
call(True).wait(); torch.cuda.synchronize()
assert st._comms[3].timeout_s == 2.0
# a GPU "sleep" of exactly 6 s on the hook's stream (the emulated-wire kernel paced by the
# constant-rate clock), so the next collectives stay pending past the 2 s timeout
w = ctypes.c_void_p()
N.check(N.lib().arctopk_comm_init_wire(2, 1.0, 6.0e6, 1, 0, ctypes.byref(w)), "wire")
buf = torch.zeros(64, device="cuda:0")
N.check(N.lib().arctopk_comm_allreduce(w, buf.data_ptr(), 64, N.F32, torch.cuda.current_stream().cuda_stream), "sleep")
call(False)
time.sleep(4.5)  # the watchdog sees them pending past 2 s
print("ALIVE", flush=True)
try:
    call(True)
except RuntimeError as e:
    print("RAISED", e, flush=True)
torch.cuda.synchronize()
N.lib().arctopk_comm_destroy(w)
"""


@pytest.mark.parametrize("handling", ["default", "0"])
def test_watchdog_timeout_tears_down_or_raises(handling, tmp_path):
    """A collective pending past the communicator's timeout (one-rank RCCL behind a 6 s GPU
    sleep, ARCTOPK_COMM_TIMEOUT_S=2): by default the watchdog ends the process before any partially
    reduced update can be applied (ProcessGroupNCCL's async error handling); with
    ARCTOPK_ASYNC_ERROR_HANDLING=0 the process lives and the next hook call raises."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, ARCTOPK_COMM_TIMEOUT_S="2.0", MASTER_ADDR="127.0.0.1")
    env.pop("ARCTOPK_ASYNC_ERROR_HANDLING", None)
    env.pop("TORCH_NCCL_ASYNC_ERROR_HANDLING", None)
    if handling != "default":
        env["ARCTOPK_ASYNC_ERROR_HANDLING"] = handling
    script = tmp_path / "child.py"
    script.write_text(_WATCHDOG_CHILD)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, str(script)], cwd=repo, env=env, capture_output=True, text=True,
                       timeout=120)
    if handling == "default":
        assert r.returncode == 1, (r.returncode, r.stdout[-1000:], r.stderr[-2000:])
        assert "ending the process" in r.stderr and "ALIVE" not in r.stdout
    else:
        assert r.returncode == 0, (r.returncode, r.stdout[-1000:], r.stderr[-2000:])
        assert "ALIVE" in r.stdout and "RAISED" in r.stdout and "timed out" in r.stdout
