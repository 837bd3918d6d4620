"""Failure behaviour of the exchange's communicators, on CPU (no GPU needed).

The reference's collectives run on ProcessGroupNCCL under init_process_group(timeout=...)
(/root/reference/cifar10/run_cifar10.py:55-58): a peer that stops answering becomes an
error after the timeout, and SURVEY.md section 8(b) asks the same of the drop-in (errors
surface as RuntimeError).  The callback communicators (any non-NCCL backend) inherit the
torch backend's own timeout; these tests drive that path through the native all-reduce
entry point with a peer that never joins, and pin the group-deterministic store keys of the
RCCL communicators' unique ids.
"""
import datetime
import os
import sys
import tempfile
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _callback_worker(rank, ws, port, td):
    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=ws,
                            timeout=datetime.timedelta(seconds=3))
    from allreducetopk_amd import _native as N
    from allreducetopk_amd import exchange as X
    c = X.Comm.callback(dist.group.WORLD)
    buf = torch.ones(64)
    c.register(buf)
    # both ranks: a working all-reduce first
    c.check(N.lib().arctopk_comm_allreduce(c.handle, buf.data_ptr(), buf.numel(), N.F32, None), "allreduce")
    assert torch.equal(buf, torch.full((64,), 2.0))
    if rank == 1:  # then this peer stops answering (stays alive, issues nothing)
        time.sleep(8)
        open(os.path.join(td, "r1_done"), "w").close()
        return
    t0 = time.time()
    with pytest.raises(RuntimeError):
        c.check(N.lib().arctopk_comm_allreduce(c.handle, buf.data_ptr(), buf.numel(), N.F32, None),
                "allreduce")
    dt = time.time() - t0
    assert dt < 7.0, f"the callback communicator's error took {dt:.1f} s (group timeout 3 s)"
    open(os.path.join(td, "r0_raised"), "w").close()


def test_callback_comm_peer_never_answers_raises_runtime_error():
    from parity import rendezvous
    port = rendezvous()
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_callback_worker, args=(2, port, td), nprocs=2, join=True)
        assert os.path.exists(os.path.join(td, "r0_raised"))


def test_store_keys_are_group_deterministic():
    """Each rank derives the same key for its n-th communicator of a tag, however many
    communicators of other tags or groups it made before (the old process-local counter
    diverged then)."""
    from allreducetopk_amd import exchange as X
    store = dist.HashStore()
    ranks = [0, 1, 2]
    keys = {r: [] for r in ranks}
    for gen in range(3):
        for r in ranks:  # every rank of generation g counts in before any of g + 1 (collective init)
            keys[r].append(X._store_key(store, "packed", ranks))
        X._store_key(store, "sketch", [0, 1])  # another group's / tag's communicators interleave
        X._store_key(store, "sketch", [0, 1])
    assert keys[0] == keys[1] == keys[2]
    assert keys[0] == [f"arctopk_comm/packed/0-1-2/{g}" for g in range(3)]


def test_group_timeout_is_read_from_the_process_group():
    from allreducetopk_amd import exchange as X
    from parity import rendezvous
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    dist.init_process_group("gloo", init_method=rendezvous(), rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=42))
    try:
        assert X.group_timeout_s(dist.group.WORLD) == 42.0
        g = dist.new_group([0], timeout=datetime.timedelta(seconds=7))
        assert X.group_timeout_s(g) == 7.0
        os.environ["ARCTOPK_COMM_TIMEOUT_S"] = "1.5"
        assert X.group_timeout_s(g) == 1.5
    finally:
        os.environ.pop("ARCTOPK_COMM_TIMEOUT_S", None)
        dist.destroy_process_group()


def test_comm_status_abort_and_bad_wire_params_without_gpu():
    """Host-side ABI of the failure path: status of a fresh communicator is 0, abort makes it
    sticky (ARCTOPK_EABORTED), and a failed communicator takes no all-reduce."""
    import ctypes
    from allreducetopk_amd import _native as N
    L = N.lib()
    calls = []
    fn = N.ALLREDUCE_FN(lambda ctx, buf, n, dt, st: calls.append(n) or 0)
    h = ctypes.c_void_p()
    N.check(L.arctopk_comm_init_callback(fn, None, 2, 0, ctypes.byref(h)), "init_callback")
    buf = torch.zeros(8)
    assert L.arctopk_comm_status(h) == 0
    N.check(L.arctopk_comm_allreduce(h, buf.data_ptr(), 8, N.F32, None), "allreduce")
    assert calls == [8]
    assert L.arctopk_comm_abort(h) == 0
    assert L.arctopk_comm_status(h) == N.EABORTED
    assert L.arctopk_comm_allreduce(h, buf.data_ptr(), 8, N.F32, None) == N.EABORTED
    assert calls == [8]
    with pytest.raises(RuntimeError, match="aborted"):
        N.check(L.arctopk_comm_status(h), "status")
    assert L.arctopk_comm_destroy(h) == 0
    w = ctypes.c_void_p()
    assert L.arctopk_comm_init_wire(8, 0.0, 10.0, 32, 0, ctypes.byref(w)) == 1001  # busbw must be > 0
    assert L.arctopk_comm_init_wire(8, 350.0, 10.0, 32, 0, ctypes.byref(w)) == 0
    assert L.arctopk_comm_size(w) == 1  # results of a one-rank all-reduce
    assert L.arctopk_comm_destroy(w) == 0


def test_callback_registry_keeps_the_longest_view_at_an_address():
    """An exchange group's buffers are prefixes of its bucket's (the first group starts at the
    bucket's address): registering the group's view must not hide the bucket's (the N = 2 gloo
    rehearsal failed with 'exchange all-reduce of an unregistered view' before)."""
    from allreducetopk_amd import _native as N
    from allreducetopk_amd import exchange as X
    from parity import rendezvous
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    dist.init_process_group("gloo", init_method=rendezvous(), rank=0, world_size=1)
    try:
        c = X.Comm.callback(dist.group.WORLD)
        bucket = torch.ones(100)
        c.register(bucket)
        c.register(bucket[:40])  # the first group's slice, registered later
        for n in (100, 40):
            c.check(N.lib().arctopk_comm_allreduce(c.handle, bucket.data_ptr(), n, N.F32, None), "allreduce")
        c.register(bucket[60:])  # another group's slice: its own address
        c.check(N.lib().arctopk_comm_allreduce(c.handle, bucket[60:].data_ptr(), 40, N.F32, None), "allreduce")
        assert torch.equal(bucket, torch.ones(100))  # one rank: the sum is the value
    finally:
        dist.destroy_process_group()
