"""The exchange pipeline below a bucket: a bucket run as groups of
consecutive tensors (arctopk_plan_group), each group its own encode -> sketch all-reduce ->
select -> pack -> packed all-reduce on the exchange stream.  Selection is per tensor and both
all-reduces are elementwise, so every output, E and gE must be the bits of the whole-bucket
exchange (reference: the per-tensor sketch all-reduce, group_topk_hook_no_reshape.py:33, :58,
:88; the packed all-reduce :280)."""
import pytest
import torch

from parity import assert_bitwise, ensure_group

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
# buckets whose tensors allow several aligned cuts (bucket order 2, 1, 0 as DDP calls them)
SHAPES = {2: [[256, 512], [96, 40], [10], [64, 64, 3, 3], [128, 256]],
          1: [[128, 2048], [16, 8, 3, 3], [8], [40, 16], [512, 64]],
          0: [[64, 72], [16, 8, 1, 1], [1000], [8, 8, 5, 5], [32, 32, 3, 3]]}


def _grad(b, step, dtype):
    from allreducetopk_amd.bucket import bucket_numel
    g = torch.randn(bucket_numel(SHAPES[b]), generator=torch.Generator().manual_seed(500 * step + b))
    return g.to(dtype)


def _run(groups, ef, defer=True, wire=None, projections="device", dtype=torch.float32, steps=3, pg=None):
    from allreducetopk_amd.bucket import SyntheticBucket
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    st = G.GroupTopKState(pg, r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback=ef,
                          seed=23)
    st.force_exchange = True
    st.defer_decode = defer
    st.emulate_wire = wire
    st.projections = projections
    st.exchange_groups = groups
    st.group_bytes = 4096  # every aligned tensor boundary
    outs = []
    for step in range(steps):
        futs, bufs = [], {}
        for b in (2, 1, 0):
            bufs[b] = _grad(b, step, dtype).to(DEV)
            futs.append(G.group_topk_hook(st, SyntheticBucket(bufs[b], SHAPES[b], index=b, is_last=(b == 0))))
        for f in futs:
            f.wait()
        torch.cuda.synchronize()
        outs.append({b: t.cpu() for b, t in bufs.items()})
    ngroups = {b: len(p[1].groups(st.group_bytes) or [p[1]]) for b, p in st._plans.items()}
    return (outs, {b: e.cpu() for b, e in st.error_dict.items()},
            {b: e.cpu() for b, e in st.global_error_dict.items()}, ngroups)


def _same(a, c, tag):
    for step, (x, y) in enumerate(zip(a[0], c[0])):
        for b in x:
            assert_bitwise(y[b], x[b], f"{tag}: step {step} bucket {b} output")
    for i, what in ((1, "E"), (2, "gE")):
        for b in a[i]:
            assert_bitwise(c[i][b], a[i][b], f"{tag}: bucket {b} {what}")


@pytest.mark.parametrize("ef,projections,dtype", [("ef14", "device", torch.float32),
                                                  ("ef21", "device", torch.float32),
                                                  ("noef", "host", torch.float32),
                                                  ("ef14", "device", torch.bfloat16)])
def test_grouped_exchange_is_bit_identical(ef, projections, dtype):
    ensure_group("nccl")
    ref = _run("off", ef, projections=projections, dtype=dtype)
    for mode in ("all", "auto"):
        got = _run(mode, ef, projections=projections, dtype=dtype)
        assert min(got[3].values()) >= 3, got[3]  # the buckets really ran as groups
        _same(ref, got, f"groups={mode}")


def test_grouped_exchange_beside_the_emulated_wire_and_for_direct_callers():
    ensure_group("nccl")
    ref = _run("off", "ef14")
    wire = dict(ranks=8, busbw_gbs=350.0, latency_us=15.0, blocks=64)
    _same(ref, _run("all", "ef14", wire=wire), "groups over the emulated wire")
    _same(ref, _run("all", "ef14", defer=None), "groups, direct caller")


def test_grouped_exchange_direct_caller_futures_complete_on_return():
    from allreducetopk_amd.bucket import SyntheticBucket
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
    ensure_group("nccl")
    st = G.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback="ef14")
    st.force_exchange = True
    st.exchange_groups = "all"
    st.group_bytes = 4096
    futs = [G.group_topk_hook(st, SyntheticBucket(_grad(b, 0, torch.float32).to(DEV), SHAPES[b], index=b,
                                                  is_last=False)) for b in (2, 1, 0)]
    assert all(f.done() for f in futs) and not st._x_pend
    torch.cuda.synchronize()


def test_grouped_exchange_over_callback_communicators():
    """The same through callback communicators (a gloo group: the path every non-NCCL backend and
    the two-ranks-on-one-GPU tests take).  The first group's buffers start at the bucket's own
    address, so the callback's buffer registry must keep both (an N = 2 gloo rehearsal of
    bench.py failed there)."""
    import torch.distributed as dist
    ensure_group("nccl")
    ref = _run("off", "ef14")
    g = dist.new_group([0], backend="gloo")
    _same(ref, _run("auto", "ef14", pg=g), "groups over a gloo callback communicator")
    _same(ref, _run("off", "ef14", pg=g), "whole buckets over a gloo callback communicator")


def test_every_run_group_runs_returns_is_a_valid_native_group():
    """group_runs must only return runs arctopk_plan_group accepts -- including a
    run that starts with a 1-D segment (DDP's reverse order) whose first SKETCH tensor's V
    offset is what the native planner checks (r = 2 and 3 make 3x3-conv V offsets 4 mod 8)."""
    from test_capi import GROUP_SHAPE_SETS
    from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan
    built = 0
    for shapes in GROUP_SHAPE_SETS:
        if sum(torch.Size(s).numel() for s in shapes) > (1 << 24):
            continue  # (the 256 MiB sets: cut at 1 KiB they are thousands of native plans)
        for r in (2, 3, 4):
            for dtype in (torch.float32, torch.bfloat16):
                plan = BucketPlan([tuple(s) for s in shapes], r, 0.2, dtype, DEV)
                for target in (1 << 12, 1 << 16):
                    groups = plan.groups(target)  # arctopk_plan_group for every run: raises on EINVAL
                    built += len(groups or [])
    assert built > 0
