"""Multi-rank HIP path on one MI355X: two ranks share cuda:0 over gloo (RCCL needs one
GPU per rank; the driver's 8-GPU bench covers RCCL).  Every rank must select the same
rows and produce the oracle's two-rank result bit for bit given those rows.  Plus the
shipped hook inside real DDP (NCCL=RCCL, world size 1)."""
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
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=ws)
    from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from allreducetopk_amd.comm_hooks import sparse_hook as SH
    from oracle import arctopk as A
    from oracle import sparse as S
    dev = "cuda:0"
    n = bucket_numel(MIX)
    if kind == "arc_pipe":  # force the pipelined pack / all-reduce / decode on this bucket
        G.BucketPlan.PIPELINE_MIN_BYTES = 64
        kind = "arc"
    if kind == "arc":
        st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                              use_error_feedback=ef, seed=77)
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
            if G.BucketPlan.PIPELINE_MIN_BYTES == 64:
                assert len(plan.groups) > 1, "pipelined path not exercised"
            other = [torch.empty_like(rl) for _ in range(ws)]
            dist.all_gather(other, rl)
            assert torch.equal(other[0], other[1]), "ranks selected different rows"
            res = A.simulate_step(allg, [None] * ws if (first or Es is None) else Es, gE, MIX, 0.2,
                                  4, ef, seed, rows_override=rows)
        else:
            idx = None
            seed = None
            if kind == "randk":
                seed = int(torch.randint(0, 1_000_000_000, (1,), generator=rng).item())
                from allreducetopk_amd import _native as N
                numels = [int(torch.Size(s).numel()) for s in MIX]
                ks = [max(1, int(x * 0.2)) for x in numels]
                kof = [sum(ks[:i]) for i in range(len(ks))]
                buf = torch.empty(sum(ks), dtype=torch.int32, device=dev)
                N.check(N.lib().arctopk_randk_indices(len(ks), N.i64_array(numels), N.i64_array(ks),
                                                      N.i64_array(kof), seed, buf.data_ptr(),
                                                      torch.cuda.current_stream().cuda_stream), "r")
                flat = buf.cpu()
                idx = [[flat[o:o + k] for o, k in zip(kof, ks)]] * ws
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
                                     ("arc_pipe", "ef14"), ("arc_pipe", "ef21"),
                                     ("topk", "ef14"), ("topk", "ef21"), ("randk", "ef14")])
def test_two_ranks_one_gpu(kind, ef):
    from parity import free_port
    port = free_port()
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(2, port, td, ef, kind), nprocs=2, join=True)


def test_hook_inside_ddp_rccl():
    """group_topk_hook registered on a real DDP model (RCCL backend, world size 1)."""
    from parity import ensure_group
    ensure_group("nccl")
    from torch.nn.parallel import DistributedDataParallel as DDP
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    from oracle import arctopk as A
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                              torch.nn.Linear(16 * 6 * 6, 64), torch.nn.ReLU(),
                              torch.nn.Linear(64, 10)).cuda()
    model = DDP(net, device_ids=[0])
    st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=1,
                          use_error_feedback="ef14", seed=3)
    captured = []

    def hook(state, bucket):
        captured.append((bucket.index(), bucket.buffer().detach().clone().cpu(),
                         [tuple(t.shape) for t in bucket.gradients()], state.iter))
        return G.group_topk_hook(state, bucket)

    model.register_comm_hook(st, hook)
    x = torch.randn(8, 3, 8, 8, device="cuda")
    for step in range(3):
        model.zero_grad()
        model(x).pow(2).mean().backward()
        torch.cuda.synchronize()
    assert st.iter == 3
    assert len(st.error_dict) >= 1
    # the last backward's buckets went through the codec: zero rows outside the selection
    for b, buf, shapes, it in captured[-len(st.error_dict):]:
        assert it == 2
        segs = A.segments(shapes, 0.2)
        ref_k = sum(s.k for s in segs)
        plan = st._plans[b][1]
        assert plan.info.values_len == ref_k
