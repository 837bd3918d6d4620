"""world_size-2 paths on CPU over gloo (real processes, real DDP buckets).

* the oracle hook replays the reference's ws=2 golden vectors over a real gloo group;
* the oracle hook runs inside real DDP (bucket views, reverse-order buckets,
  is_last/iter accounting) and every rank ends with identical gradients equal to the
  in-process two-rank simulation;
* the shipped hooks' host paths that need no GPU (dense warm-up all-reduce, EF21
  first-call init, the 'none' compressor) run in DDP with gloo.
"""
import os
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _setup(rank, ws, port):
    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=port, rank=rank,
                            world_size=ws)


def _spawn(fn, *args, ws=2):
    from parity import rendezvous
    port = rendezvous()
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(fn, args=(ws, port, td) + args, nprocs=ws, join=True)


# ---------------------------------------------------------------------------
def _golden_worker(rank, ws, port, td, name):
    _setup(rank, ws, port)
    from allreducetopk_amd.bucket import SyntheticBucket
    from golden_io import Golden
    from oracle import arctopk as A
    g = Golden(name)
    m = g.meta
    st = A.OracleState(r=m["r"], compress_ratio=m["ratio"], start_compress_iter=m["start"],
                       use_error_feedback=m["ef"], seed=m["seed"])
    shapes = [tuple(s) for s in m["shapes"]]
    for it in range(m["iters"]):
        b = SyntheticBucket(g.t(rank, it, "G").clone(), shapes)
        out = A.oracle_group_topk_hook(st, b)
        assert torch.equal(out, g.t(rank, it, "out")), f"{name} it{it} rank{rank}"
        if g.has(rank, it, "E"):
            assert torch.equal(st.error_dict[0], g.t(rank, it, "E"))
        assert st.comm_bits_this_round == int(g.np(rank, it, "bits"))
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["arc_mix_ef14_ws2", "arc_mix_ef21_ws2", "arc_warmup_ef21_ws2",
                                  "arc_gmix_ef14_ws2", "arc_gmix_ef21_ws2"])
def test_oracle_hook_replays_ws2_golden_over_gloo(name):
    _spawn(_golden_worker, name)


# ---------------------------------------------------------------------------
class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = torch.nn.Conv2d(2, 8, 3)    # ND: [8, 2, 3, 3] -> m = 18
        self.fc = torch.nn.Linear(32, 24)        # 2-D
        self.head = torch.nn.Linear(24, 5)       # 2-D + 1-D bias

    def forward(self, x):
        y = torch.relu(self.conv(x)).mean(dim=(2, 3))
        y = torch.cat([y, y, y, y], dim=1)
        return self.head(torch.relu(self.fc(y)))


def _ddp_oracle_worker(rank, ws, port, td, ef):
    _setup(rank, ws, port)
    from torch.nn.parallel import DistributedDataParallel as DDP
    from oracle import arctopk as A
    torch.manual_seed(0)
    model = DDP(_Net(), bucket_cap_mb=0.001)  # several small buckets
    st = A.OracleState(r=4, compress_ratio=0.25, start_compress_iter=1, use_error_feedback=ef,
                       seed=11)
    seen = []
    sim = {}

    def hook(state, bucket):
        gin = bucket.buffer().clone()
        shapes = [tuple(t.shape) for t in bucket.gradients()]
        b = bucket.index()
        Es = state.error_dict.get(b)
        E_prev = Es.clone() if Es is not None else None
        gE_prev = state.global_error_dict.get(b)
        gE_prev = gE_prev.clone() if gE_prev is not None else None
        iter_before = state.iter
        seed_state = state.rng.get_state()
        out = A.oracle_group_topk_hook(state, bucket)
        # reference result for this call from both ranks' inputs, simulated in-process
        allg = [torch.empty_like(gin) for _ in range(ws)]
        dist.all_gather(allg, gin)
        alle = None
        if E_prev is not None:
            alle = [torch.empty_like(E_prev) for _ in range(ws)]
            dist.all_gather(alle, E_prev)
        seen.append((iter_before, b, out.clone()))
        if iter_before >= state.start_compress_iter and not (ef == "ef21" and E_prev is None):
            rng = torch.Generator()
            rng.set_state(seed_state)
            seed = int(torch.randint(0, 1_000_000_000, (1,), generator=rng).item())
            first = ef == "ef14" and E_prev is None
            res = A.simulate_step(allg, [None] * ws if (first or alle is None) else alle, gE_prev,
                                  shapes, 0.25, 4, ef, seed)
            sim[(iter_before, b)] = res["out"]
        fut = torch.futures.Future()
        fut.set_result(out)
        return fut

    model.register_comm_hook(st, hook)
    opt = torch.optim.SGD(model.parameters(), lr=0.01)
    g = torch.Generator().manual_seed(100 + rank)
    for step in range(4):
        x = torch.randn(4, 2, 6, 6, generator=g)
        loss = model(x).pow(2).sum()
        opt.zero_grad()
        loss.backward()
        for p in model.parameters():  # check_grad_identity (ref run_glue_no_trainer_new.py:78-98)
            ref = p.grad.clone()
            dist.broadcast(ref, 0)
            assert torch.equal(p.grad, ref), "ranks disagree after the hook"
        opt.step()
    assert st.iter == 4
    assert any(k[0] >= 1 for k in sim), "no compressed call was checked"
    for it, b, out in seen:
        if (it, b) in sim:
            assert torch.equal(out, sim[(it, b)]), f"iter {it} bucket {b}: DDP result != simulation"
    dist.destroy_process_group()


@pytest.mark.parametrize("ef", ["noef", "ef14", "ef21"])
def test_oracle_hook_in_real_ddp_ws2(ef):
    _spawn(_ddp_oracle_worker, ef)


# ---------------------------------------------------------------------------
def _product_host_paths_worker(rank, ws, port, td):
    _setup(rank, ws, port)
    from torch.nn.parallel import DistributedDataParallel as DDP
    from allreducetopk_amd.bucket import SyntheticBucket
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from allreducetopk_amd.comm_hooks.default_hooks import my_allreduce_hook
    from allreducetopk_amd.comm_hooks.utils import HookState
    torch.manual_seed(0)
    # dense warm-up path of the ARC hook and the 'none' compressor inside real DDP
    for make in ("warmup", "none"):
        model = DDP(_Net(), bucket_cap_mb=0.001)
        ref = _Net()
        ref.load_state_dict(model.module.state_dict())
        if make == "warmup":
            st = G.GroupTopKState(None, compress_ratio=0.2, start_compress_iter=100)
            model.register_comm_hook(st, G.group_topk_hook)
        else:
            st = HookState(None)
            model.register_comm_hook(st, my_allreduce_hook)
        g = torch.Generator().manual_seed(7 + rank)
        x = torch.randn(4, 2, 6, 6, generator=g)
        model(x).pow(2).sum().backward()
        xs = [torch.empty_like(x) for _ in range(ws)]
        dist.all_gather(xs, x)
        grads = []
        for xq in xs:
            ref.zero_grad()
            ref(xq).pow(2).sum().backward()
            grads.append([p.grad.clone() for p in ref.parameters()])
        for i, p in enumerate(model.parameters()):
            mean = sum(gr[i] for gr in grads) / ws
            assert torch.allclose(p.grad, mean, atol=1e-6, rtol=1e-5)
        nbits = sum(p.numel() for p in model.parameters()) * 32
        assert st.comm_bits_this_round == 2 * (ws - 1) * nbits
        assert st.iter == 1
    # EF21 first compressed call: dense mean, E = local grad, gE = mean (ref :236-250)
    st = G.GroupTopKState(None, compress_ratio=0.2, start_compress_iter=0, use_error_feedback="ef21")
    local = torch.randn(100, generator=torch.Generator().manual_seed(rank))
    out = G.group_topk_hook(st, SyntheticBucket(local.clone(), [(10, 10)])).wait()
    allv = [torch.empty_like(local) for _ in range(ws)]
    dist.all_gather(allv, local)
    mean = (allv[0] + allv[1]) / ws
    assert torch.equal(out, mean) and torch.equal(st.global_error_dict[0], mean)
    assert torch.equal(st.error_dict[0], local)
    assert st.comm_bits_this_round == 100 * 32
    dist.destroy_process_group()


def test_product_host_paths_ws2():
    _spawn(_product_host_paths_worker)


# ---------------------------------------------------------------------------
def _exchange_comm_worker(rank, ws, port, td, mode):
    os.environ["ARCTOPK_SKETCH_COMM"] = mode
    _setup(rank, ws, port)
    from allreducetopk_amd import _native as N
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0)
    assert st._comms is None, "the constructor must not be collective"
    st.init_exchange_comms("cpu")  # collective: every rank, same point (as the registry does)
    group, _, sk, pk = st._comms
    assert group is dist.group.WORLD and pk.kind == "callback" and pk.size == ws
    assert (sk is not pk) == (mode == "separate")
    if mode == "separate":
        assert sk.group is not pk.group
    # an all-reduce through the native communicator (libarctopk -> callback -> gloo)
    for c in {id(sk): sk, id(pk): pk}.values():
        t = torch.arange(6, dtype=torch.float32) * (rank + 1)
        c.register(t)
        c.check(N.lib().arctopk_comm_allreduce(c.handle, t.data_ptr(), 5, N.F32, None), "allreduce")
        want = torch.arange(6, dtype=torch.float32) * 3
        want[5] = 5 * (rank + 1)  # beyond `count`: untouched
        assert torch.equal(t, want)
    # an unregistered buffer is refused with the callback's own error
    u = torch.ones(4)
    with pytest.raises(KeyError):
        pk.check(N.lib().arctopk_comm_allreduce(pk.handle, u.data_ptr(), 4, N.F32, None), "allreduce")
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["separate", "shared"])
def test_exchange_communicators(mode):
    """The exchange's communicators are made by init_exchange_comms (collective; the
    registry calls it on every rank), never by the constructor, and all-reduce through the
    native library."""
    _spawn(_exchange_comm_worker, mode)


def _registry_worker(rank, ws, port, td):
    _setup(rank, ws, port)
    import argparse
    from torch.nn.parallel import DistributedDataParallel as DDP
    from allreducetopk_amd.comm_hooks.utils import add_comm_hook_args, register_comm_hook_for_ddp_model
    p = argparse.ArgumentParser()
    add_comm_hook_args(p)
    p.add_argument("--seed", type=int, default=0)
    args = p.parse_args(["--compressor", "group_topk_no_reshape", "--compress_ratio", "0.2"])
    st = register_comm_hook_for_ddp_model(DDP(_Net()), None, args)
    assert st._comms is not None and st._comms[3].size == ws
    dist.destroy_process_group()


def test_registry_creates_exchange_communicators():
    _spawn(_registry_worker)
