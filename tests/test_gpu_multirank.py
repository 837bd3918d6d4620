"""Multi-rank HIP path on one MI355X.

* Two ranks share cuda:0 over gloo (RCCL needs one GPU per rank): the native exchange step
  (arctopk_exchange_step) runs with its all-reduces routed through gloo, so the orchestration
  every rank runs at N > 1 is the one tested.  Every rank must select the same rows and
  produce the oracle's two-rank result bit for bit given those rows; including the hook
  inside a real two-rank DDP model on cuda:0.
* The forced exchange at world size 1 over one-rank RCCL communicators: the same native
  step with RCCL, buckets in flight, in DDP.
"""
import os
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
MIX = [[10], [40, 16], [4, 3, 3, 3], [16, 8, 3, 3], [16, 8, 1, 1], [96, 40], [7], [256, 512],
       [130, 2048]]


def _worker(rank, ws, port, td, ef, kind):
    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=port, rank=rank,
                            world_size=ws)
    from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from allreducetopk_amd.comm_hooks import sparse_hook as SH
    from oracle import arctopk as A
    from oracle import sparse as S
    dev = "cuda:0"
    n = bucket_numel(MIX)
    sync = kind == "arc_sync"  # the exchange without an exchange stream (all on the caller's)
    if sync:
        kind = "arc"
    if kind == "arc":
        st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                              use_error_feedback=ef, seed=77)
        st.async_exchange = not sync
        ost = A.OracleState(seed=77)
    else:
        st = SH.SparseState(None, compress_ratio=0.2, start_compress_iter=0, sparse_type="tensor",
                            random=(kind == "randk"), use_error_feedback=ef, random_seed=5,
                            index_source="hash")
        rng = torch.Generator().manual_seed(5)
    Es = None
    gE = None
    for it in range(3):
        Gl = torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + rank))
        allg = [torch.empty_like(Gl) for _ in range(ws)]
        dist.all_gather(allg, Gl)
        hook = G.group_topk_hook if kind == "arc" else SH.sparse_hook_sync
        out = hook(st, SyntheticBucket(Gl.to(dev), MIX)).wait()
        torch.cuda.synchronize()
        if ef == "ef21" and Es is None:
            Es = [g.clone() for g in allg]
            gE = (allg[0] + allg[1]) / ws
            assert torch.equal(out.cpu(), gE)
            continue
        first = ef == "ef14" and Es is None
        if kind == "arc":
            seed = ost.next_seed()
            plan = st._plans[0][1]
            rl = plan.rowlist.cpu()
            rows = [rl[s.sel_off:s.sel_off + s.k_rows].long() for s in plan.segments]
            assert st._comms is not None and st._comms[3].size == ws  # the exchange step ran
            other = [torch.empty_like(rl) for _ in range(ws)]
            dist.all_gather(other, rl)
            assert torch.equal(other[0], other[1]), "ranks selected different rows"
            res = A.simulate_step(allg, [None] * ws if (first or Es is None) else Es, gE, MIX, 0.2,
                                  4, ef, seed, rows_override=rows, proj_device=dev)
        else:
            idx = None
            seed = None
            if kind == "randk":
                seed = int(torch.randint(0, 1_000_000_000, (1,), generator=rng).item())
                from parity import device_randk_hash
                numels = [int(torch.Size(s).numel()) for s in MIX]
                ks = [max(1, int(x * 0.2)) for x in numels]
                idx = [device_randk_hash(numels, ks, seed, dev)] * ws
            res = S.simulate_step(allg, [None] * ws if (first or Es is None) else Es, gE, MIX, 0.2,
                                  ef, kind == "randk", seed, indices_override=idx)
        assert torch.equal(out.cpu(), res["out"]), f"it{it} rank{rank} output"
        if ef != "noef":
            assert torch.equal(st.error_dict[0].cpu(), res["E_new"][rank]), f"it{it} E"
            Es = res["E_new"]
        if ef == "ef21":
            gE = res["gE_new"]
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,ef", [("arc", "noef"), ("arc", "ef14"), ("arc", "ef21"),
                                     ("arc_sync", "ef14"), ("arc_sync", "ef21"),
                                     ("topk", "ef14"), ("topk", "ef21"), ("randk", "ef14")])
def test_two_ranks_one_gpu(kind, ef):
    from parity import rendezvous
    port = rendezvous()
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(2, port, td, ef, kind), nprocs=2, join=True)


# three buckets of different layouts per backward (DDP order: bucket 0 is hooked last)
MULTI = {2: [[256, 512], [96, 40], [10]],
         1: [[130, 2048], [16, 8, 3, 3], [7], [40, 16]],
         0: [[64, 70], [16, 8, 1, 1], [1000], [8, 8, 5, 5]]}


def _worker_multi(rank, ws, port, ef, sketch_comm, steps):
    """Every bucket of a backward in flight at once: the hook is called for buckets 2, 1, 0
    and the futures are waited only at the end of the step (DDP's finalize), so bucket b's
    packed all-reduce and side-stream decode overlap bucket b-1's encode, and a bucket's
    next call orders after its pending decode.  Each bucket's output, E and gE must equal
    the two-rank oracle bit for bit given the selected rows."""
    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    os.environ["ARCTOPK_SKETCH_COMM"] = sketch_comm
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=port, rank=rank,
                            world_size=ws)
    from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from oracle import arctopk as A
    dev = "cuda:0"
    st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                          use_error_feedback=ef, seed=31)
    st.defer_decode = True  # waits like DDP's finalize (after the backward's last bucket)
    assert st.async_exchange
    ost = A.OracleState(seed=31)
    order = [2, 1, 0]
    E = {b: None for b in order}
    gE = {b: None for b in order}
    for step in range(steps):
        allg, futs = {}, {}
        for b in order:
            shapes = MULTI[b]
            Gl = torch.randn(bucket_numel(shapes),
                             generator=torch.Generator().manual_seed(10_000 * step + 100 * b + rank))
            parts = [torch.empty_like(Gl) for _ in range(ws)]
            dist.all_gather(parts, Gl)
            allg[b] = parts
            futs[b] = G.group_topk_hook(st, SyntheticBucket(Gl.to(dev), shapes, index=b,
                                                            is_last=(b == 0)))
        outs = {b: futs[b].wait() for b in order}  # the caller's stream waits for each decode
        torch.cuda.synchronize()
        assert st.iter == step + 1
        if st._comms is not None:  # (EF21's first backward is the dense init: no exchange yet)
            sk, pk = st._comms[2], st._comms[3]
            assert (sk is not pk) == (sketch_comm == "separate") and pk.kind == "callback"
        for b in order:
            shapes = MULTI[b]
            if ef == "ef21" and E[b] is None:  # dense init call (no seed drawn)
                E[b] = [g.clone() for g in allg[b]]
                gE[b] = (allg[b][0] + allg[b][1]) / ws
                assert torch.equal(outs[b].cpu(), gE[b]), f"step{step} bucket{b} EF21 init"
                continue
            seed = ost.next_seed()
            plan = st._plans[b][1]
            rl = plan.rowlist.cpu()
            rows = [rl[s.sel_off:s.sel_off + s.k_rows].long() for s in plan.segments]
            other = [torch.empty_like(rl) for _ in range(ws)]
            dist.all_gather(other, rl)
            assert torch.equal(other[0], other[1]), f"step{step} bucket{b}: ranks selected different rows"
            first = ef == "ef14" and E[b] is None
            Es = [None] * ws if (ef == "noef" or first) else E[b]
            res = A.simulate_step(allg[b], Es, gE[b], shapes, 0.2, 4, ef, seed, rows_override=rows,
                                  proj_device=dev)
            assert torch.equal(outs[b].cpu(), res["out"]), f"step{step} bucket{b} rank{rank} output"
            if ef != "noef":
                assert torch.equal(st.error_dict[b].cpu(), res["E_new"][rank]), f"step{step} bucket{b} E"
                E[b] = res["E_new"]
            if ef == "ef21":
                assert torch.equal(st.global_error_dict[b].cpu(), res["gE_new"]), f"step{step} bucket{b} gE"
                gE[b] = res["gE_new"]
    assert st._comms is not None
    dist.destroy_process_group()


@pytest.mark.parametrize("ef,sketch_comm", [("ef14", "separate"), ("ef21", "separate"),
                                            ("noef", "shared"), ("ef14", "shared")])
def test_two_ranks_buckets_in_flight(ef, sketch_comm):
    from parity import rendezvous
    mp.spawn(_worker_multi, args=(2, rendezvous(), ef, sketch_comm, 3), nprocs=2, join=True)


class _DdpNet(torch.nn.Module):
    """Conv (ND, m = 18), linear weights (2-D) and biases (1-D): several DDP buckets at a
    0.5 MB cap (1.2 MB + 1.05 MB of linear weights)."""

    def __init__(self):
        super().__init__()
        self.body = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                                        torch.nn.Linear(16 * 6 * 6, 512), torch.nn.ReLU(),
                                        torch.nn.Linear(512, 512), torch.nn.ReLU(),
                                        torch.nn.Linear(512, 10))

    def forward(self, x):
        return self.body(x)


def _ddp_check(model, st, ost, ws, rank, ef, steps, x, flips_ok=2):
    """Run `steps` backwards of DDP(model) with group_topk_hook; every compressed bucket's
    input (all ranks) and residuals are captured before the hook, replayed through the
    oracle's ws-rank simulation with the rows the device selected, and the gradients DDP
    hands the parameters (after its finalize waited the hook's Future) must equal the
    oracle's output bit for bit (the reference's check_grad_identity intent,
    glue_fine-tuning/run_glue_no_trainer_new.py:78-98, made exact)."""
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from oracle import arctopk as A
    from parity import check_rows_tie_aware
    calls = []

    def gather(t):
        if ws == 1:
            return [t]
        parts = [torch.empty_like(t) for _ in range(ws)]
        dist.all_gather(parts, t)
        return parts

    def hook(state, bucket):
        it = state.iter
        b = bucket.index()
        E = state.error_dict.get(b)
        gE = state.global_error_dict.get(b)
        rec = dict(b=b, it=it, G=gather(bucket.buffer().detach().clone().cpu()),
                   E=None if E is None else gather(E.detach().clone().cpu()),
                   gE=None if gE is None else gE.detach().clone().cpu(),
                   shapes=[tuple(t.shape) for t in bucket.gradients()],
                   params=list(bucket.parameters()))
        fut = G.group_topk_hook(state, bucket)
        if it >= state.start_compress_iter and b in state._plans:  # (not on EF21's dense init)
            rec["plan"] = state._plans[b][1]
        calls.append(rec)
        return fut

    model.register_comm_hook(st, hook)
    flips = 0
    checked = 0
    for step in range(steps):
        model.zero_grad()
        start = len(calls)
        model(x).pow(2).mean().backward()
        torch.cuda.synchronize()
        step_calls = calls[start:]
        assert len({c["b"] for c in step_calls}) >= 2 or step == 0  # (DDP rebuilds its buckets after step 0)
        for c in step_calls:
            if c["it"] < st.start_compress_iter or (ef == "ef21" and c["E"] is None):
                continue
            seed = ost.next_seed()
            plan = c["plan"]
            rl = plan.rowlist.cpu()
            rows = [rl[s_.sel_off:s_.sel_off + s_.k_rows].long() for s_ in plan.segments]
            first = ef == "ef14" and c["E"] is None
            res = A.simulate_step(c["G"], [None] * ws if (ef == "noef" or first) else c["E"], c["gE"],
                                  c["shapes"], 0.2, 4, ef, seed, rows_override=rows, proj_device="cuda:0")
            for r_, nrm, s_ in zip(rows, res["norms"], plan.segments):
                flips += check_rows_tie_aware(r_, nrm, int(s_.k_rows), band=2e-4)
            off = 0
            for p, shp in zip(c["params"], c["shapes"]):
                nel = p.numel()
                assert torch.equal(p.grad.detach().flatten().cpu(), res["out"][off:off + nel]), \
                    f"rank{rank} step{step} bucket{c['b']} param grad differs from the oracle"
                off += nel
            if ef != "noef":
                assert torch.equal(st.error_dict[c["b"]].cpu(), res["E_new"][rank])
            if ef == "ef21":
                assert torch.equal(st.global_error_dict[c["b"]].cpu(), res["gE_new"])
            checked += 1
    assert st.iter == steps
    assert checked >= 2 * (steps - st.start_compress_iter - (ef == "ef21"))
    print(f"rank{rank}: {flips} rows differ from the oracle's selection (band 2e-4)")
    assert flips <= flips_ok, f"{flips} rows differ from the oracle's selection (near-ties only)"


@pytest.mark.parametrize("force_exchange", [False, True])
def test_hook_inside_ddp_rccl(force_exchange):
    """The shipped hook registered on a real DDP model (RCCL backend, world size 1): the
    one-call step, and the forced exchange (the N > 1 code path: one-rank RCCL communicators,
    exchange stream, device-aware Future through the Reducer's finalize)."""
    from parity import ensure_group
    ensure_group("nccl")
    from torch.nn.parallel import DistributedDataParallel as DDP
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from oracle import arctopk as A
    torch.manual_seed(0)
    model = DDP(_DdpNet().cuda(), device_ids=[0], bucket_cap_mb=0.5)
    st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=1,
                          use_error_feedback="ef14", seed=3)
    st.force_exchange = force_exchange
    x = torch.randn(8, 3, 8, 8, device="cuda")
    _ddp_check(model, st, A.OracleState(seed=3), 1, 0, "ef14", 4, x, flips_ok=0)
    if force_exchange:
        assert st._comms is not None and st._comms[3].kind == "rccl" and st._comms[3].size == 1


def _ddp_two_ranks_worker(rank, ws, port, ef):
    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=ws)
    from torch.nn.parallel import DistributedDataParallel as DDP
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from oracle import arctopk as A
    torch.manual_seed(0)
    model = DDP(_DdpNet().cuda(), device_ids=[0], bucket_cap_mb=0.5)
    st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=1,
                          use_error_feedback=ef, seed=9)
    assert st.async_exchange
    x = torch.randn(8, 3, 8, 8, generator=torch.Generator().manual_seed(50 + rank)).cuda()
    _ddp_check(model, st, A.OracleState(seed=9), ws, rank, ef, 4, x)
    assert st._comms[3].kind == "callback" and st._comms[3].size == ws
    dist.destroy_process_group()


@pytest.mark.parametrize("ef", ["ef14", "ef21"])
def test_hook_inside_ddp_two_ranks(ef):
    """Two DDP ranks on cuda:0 (gloo): the exchange step with its exchange-stream decode
    and device-aware Future through the Reducer's finalize, every parameter gradient vs the
    two-rank oracle."""
    from parity import rendezvous
    mp.spawn(_ddp_two_ranks_worker, args=(2, rendezvous(), ef), nprocs=2, join=True)


@pytest.mark.parametrize("ef,sketch_comm", [("ef14", "separate"), ("ef21", "separate"),
                                            ("ef14", "shared"), ("noef", "separate")])
def test_forced_exchange_buckets_in_flight(ef, sketch_comm):
    """The N > 1 code path at world size 1: one-rank RCCL communicators (both sketch modes),
    three buckets per backward hooked before any Future is waited (each bucket's packed
    all-reduce and decode on the exchange stream beside the next bucket's encode), three
    backwards; every output, E and gE vs the oracle bit for bit given the rows."""
    from parity import ensure_group
    ensure_group("nccl")
    from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from oracle import arctopk as A
    st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                          use_error_feedback=ef, seed=41)
    st.force_exchange = True
    st.defer_decode = True  # waits like DDP's finalize (after the backward's last bucket)
    st.sketch_comm = sketch_comm
    ost = A.OracleState(seed=41)
    order = [2, 1, 0]
    E = {b: None for b in order}
    gE = {b: None for b in order}
    dev = "cuda:0"
    for step in range(3):
        ins, futs = {}, {}
        for b in order:
            shapes = MULTI[b]
            Gl = torch.randn(bucket_numel(shapes), generator=torch.Generator().manual_seed(7000 * step + b))
            ins[b] = Gl
            futs[b] = G.group_topk_hook(st, SyntheticBucket(Gl.to(dev), shapes, index=b, is_last=(b == 0)))
        outs = {b: futs[b].wait() for b in order}
        torch.cuda.synchronize()
        if st._comms is not None:  # (EF21's first backward is the dense init: no exchange yet)
            sk, pk = st._comms[2], st._comms[3]
            assert pk.kind == "rccl" and pk.size == 1 and (sk is not pk) == (sketch_comm == "separate")
        for b in order:
            shapes = MULTI[b]
            if ef == "ef21" and E[b] is None:
                E[b] = [ins[b].clone()]
                gE[b] = ins[b].clone()
                assert torch.equal(outs[b].cpu(), gE[b])
                continue
            seed = ost.next_seed()
            plan = st._plans[b][1]
            rl = plan.rowlist.cpu()
            rows = [rl[s_.sel_off:s_.sel_off + s_.k_rows].long() for s_ in plan.segments]
            first = ef == "ef14" and E[b] is None
            res = A.simulate_step([ins[b]], [None] if (ef == "noef" or first) else E[b], gE[b], shapes, 0.2, 4,
                                  ef, seed, rows_override=rows, proj_device=dev)
            assert torch.equal(outs[b].cpu(), res["out"]), f"step{step} bucket{b} output"
            if ef != "noef":
                assert torch.equal(st.error_dict[b].cpu(), res["E_new"][0])
                E[b] = res["E_new"]
            if ef == "ef21":
                assert torch.equal(st.global_error_dict[b].cpu(), res["gE_new"])
                gE[b] = res["gE_new"]


def _golden_ws2_worker(rank, ws, port, name, group_bytes=0):
    """The reference's own two-rank outputs (tests/golden, made by running the reference
    hook over a real two-rank gloo group) replayed through the HIP hook -- ARC-TopK through
    the exchange step, TopK through sparse_hook_sync -- bit for bit.  group_bytes > 0: the
    ARC-TopK bucket runs as exchange groups of about that size (exchange_groups="all"), each
    with its own two-rank sketch and packed all-reduce, and both ranks' rows are compared."""
    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=ws)
    from allreducetopk_amd.bucket import SyntheticBucket
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from allreducetopk_amd.comm_hooks import sparse_hook, sparse_hook_c4
    from golden_io import Golden
    from parity import assert_bitwise, check_rows_tie_aware
    g = Golden(name)
    m = g.meta
    assert m["ws"] == ws
    shapes = [tuple(s) for s in m["shapes"]]
    if m["hook"] == "arc":
        st = G.GroupTopKState(None, r=m["r"], compress_ratio=m["ratio"], start_compress_iter=m["start"],
                              use_error_feedback=m["ef"], seed=m["seed"])
        st.projections = "host"  # the golden vectors come from the reference run on CPU
        if group_bytes:
            st.exchange_groups, st.group_bytes = "all", group_bytes
        hook = G.group_topk_hook
    else:
        mod = sparse_hook_c4 if m["hook"] == "sparse_c4" else sparse_hook
        st = mod.SparseState(None, compress_ratio=m["ratio"], start_compress_iter=m["start"],
                             sparse_type="tensor", random=m["random"], use_error_feedback=m["ef"],
                             random_seed=m["seed"])
        st.index_source = "host"  # RandK: the reference's CPU randperm draws (the fixtures')
        st.error_decay = m.get("error_decay", 1.0)
        if m.get("large_batch"):  # EF21 large-batch initialisation, from iteration iter0
            st.large_batch_init, st.iter = True, m["iter0"]
        hook = mod.sparse_hook_sync
    bf16 = m.get("dtype") == "bf16"
    from oracle import arctopk as A
    ost = A.OracleState(seed=m["seed"])
    flips = 0
    for it in range(m["iters"]):
        out = hook(st, SyntheticBucket(g.t(rank, it, "G").to("cuda:0"), shapes)).wait()
        torch.cuda.synchronize()
        if m["hook"] == "arc" and g.has(rank, it, "topk0_in"):
            plan = st._plans[0][1]
            rl = plan.rowlist.cpu()
            if group_bytes:  # the bucket really ran as >= 3 groups, and both ranks chose the same rows
                units = plan.groups(group_bytes)
                assert units is not None and len(units) >= 3, f"{name}: {units} groups"
                both = [torch.empty_like(rl) for _ in range(ws)]
                dist.all_gather(both, rl)
                assert all(torch.equal(both[0], x) for x in both[1:]), f"{name} it{it}: ranks' rows differ"
            rows = []
            for j, s_ in enumerate(plan.segments):
                r_ = rl[s_.sel_off:s_.sel_off + s_.k_rows].long()
                rows.append(r_)
                ref = g.t(rank, it, f"topk{j}_in")
                if bf16:  # bf16 norms tie often: the tie rule within one bf16 rounding of the sketch,
                    # and every row that differs from the exact rule on the reference's norms counted
                    flips += check_rows_tie_aware(r_, ref.float(), int(s_.k_rows), band=2.0 ** -7)
                else:
                    assert check_rows_tie_aware(r_, ref, int(s_.k_rows), band=0.0) == 0, \
                        f"{name} it{it} seg{j} rows"
            seed = ost.next_seed()
            assert int(g.np(rank, it, "seed")[0]) == seed
            if bf16:  # given the device's rows: the two-rank oracle (pinned to the same vectors)
                res = A.simulate_step([g.t(q, it, "G") for q in range(ws)], [None] * ws, None, shapes,
                                      m["ratio"], m["r"], m["ef"], seed, rows_override=rows)
                assert_bitwise(out, res["out"], f"{name} rank{rank} it{it} out given the rows")
        if not (bf16 and m["hook"] == "arc" and g.has(rank, it, "topk0_in")):
            assert_bitwise(out, g.t(rank, it, "out"), f"{name} rank{rank} it{it} out")
        if g.has(rank, it, "E"):
            assert_bitwise(st.error_dict[0], g.t(rank, it, "E"), f"{name} rank{rank} it{it} E")
        if g.has(rank, it, "gE"):
            assert_bitwise(st.global_error_dict[0], g.t(rank, it, "gE"), f"{name} rank{rank} it{it} gE")
        assert st.comm_bits_this_round == int(g.np(rank, it, "bits"))
        assert st.iter == int(g.np(rank, it, "iter_after"))
    # bf16: rows that differ from the reference's own selection (within the band) are counted
    # and bounded: none for these fixtures
    print(f"{name} rank{rank}: {flips} bf16 row flips vs the reference's norms")
    assert flips == 0, f"{name} rank{rank}: {flips} rows differ from the reference's selection"
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["arc_mix_ef14_ws2", "arc_mix_ef21_ws2", "arc_warmup_ef21_ws2",
                                  "arc_mix_noef_bf16_ws2", "topk_mix_ef14_ws2", "topk_mix_ef21_ws2",
                                  "topk_mix_ef21_decay07_ws2", "randk_mix_noef_ws2",
                                  "topk_largebatch_ef21_decay07_ws2", "randk_largebatch_ef21_ws2"])
def test_reference_ws2_golden_through_hip_hook(name):
    """Every ws=2 fixture of the reference, RandK included (index_source="host": its CPU
    torch.randperm draws, sparse_hook_c4.py:20)."""
    from parity import rendezvous
    mp.spawn(_golden_ws2_worker, args=(2, rendezvous(), name), nprocs=2, join=True)


@pytest.mark.parametrize("name", ["arc_gmix_ef14_ws2", "arc_gmix_ef21_ws2", "arc_gmix_noef_bf16_ws2"])
@pytest.mark.parametrize("group_bytes", [0, 8192])
def test_reference_ws2_golden_through_grouped_exchange(name, group_bytes):
    """The exchange pipeline below a bucket at two ranks: the reference's
    two-rank fixtures of a DDP-ordered mix (a bias or norm before each weight, so cuts land on
    1-D segments) replayed with every bucket cut into 6 groups of <= 8 KiB, each group's sketch
    and packed values all-reduced over the two ranks on its own -- outputs, E, gE and bits bit
    for bit, the same rows on both ranks -- and whole (group_bytes 0) for comparison."""
    from parity import rendezvous
    mp.spawn(_golden_ws2_worker, args=(2, rendezvous(), name, group_bytes), nprocs=2, join=True)
