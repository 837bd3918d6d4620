"""ARC-TopK HIP path vs the CPU oracle, on an MI355X (run with -m gpu).

Parity bar (BASELINE north_star): selected rows identical to the reference's
(exactly, when the select kernel is fed the oracle's sketch; modulo sketch
rounding at the k-th energy end to end), and every output / residual
bit-identical given the selected rows (the codec only copies, adds and
divides fp32 values in the reference's order).  The sketch itself (G @ V, a
2048-term fp32 dot product) is compared to torch CPU mm within 2e-5 relative.
"""
import pytest
import torch

from allreducetopk_amd import _native as N
from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import (BucketPlan, GroupTopKState,
                                                                      group_topk_hook)
from golden_io import Golden, case_names
from oracle import arctopk as A
from parity import (assert_bitwise, assert_close_rel, check_rows_tie_aware, ensure_group)

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
MIX = [[10], [40, 16], [4, 3, 3, 3], [16, 8, 3, 3], [16, 8, 1, 1], [96, 40], [7], [256, 512],
       [33, 130], [1000], [64, 70], [8, 8, 5, 5], [130, 2048], [9, 5632], [6, 4101]]
# Segments past the single-block select (> 15360 rows): multi-block radix select, and more
# of them than one select batch holds (48).
LARGE = [[20000, 8], [30], [512, 512, 3, 3], [16000, 3], [7, 9]] + [[15400, 2]] * 50
SHAPE_SETS = {"mix": MIX, "large": LARGE}


@pytest.fixture(scope="module", autouse=True)
def group():
    ensure_group("nccl")
    yield


def _rand_bucket(shapes, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(bucket_numel(shapes), generator=g)


def _gpu_rows(plan: BucketPlan):
    rl = plan.rowlist.cpu()
    out = []
    for s in plan.segments:
        out.append(rl[s.sel_off:s.sel_off + s.k_rows].long())
    return out


def test_plan_geometry_matches_oracle():
    plan = BucketPlan([tuple(s) for s in MIX], 4, 0.2, torch.float32, DEV)
    segs = A.segments(MIX, 0.2)
    for s, o in zip(plan.segments, segs):
        assert (s.offset, s.n, s.m, s.k_rows) == (o.offset, o.n, o.m, o.k_rows)
    assert plan.info.values_len == sum(o.k for o in segs)


@pytest.mark.parametrize("ef,which", [("noef", "mix"), ("ef14", "mix"), ("ef21", "mix"),
                                      ("ef14", "large"), ("ef21", "large")])
def test_kernel_phases_bitexact(ef, which):
    """encode -> select (fed the oracle's sketch) -> pack -> decode, phase by phase."""
    shapes = SHAPE_SETS[which]
    segs = A.segments(shapes, 0.2)
    plan = BucketPlan([tuple(s) for s in shapes], 4, 0.2, torch.float32, DEV)
    G = _rand_bucket(shapes, 1)
    E = _rand_bucket(shapes, 2) * 0.5 if ef != "noef" else None
    gE = _rand_bucket(shapes, 3) if ef == "ef21" else None
    seed = 987654
    Vs = A.draw_projections(seed, segs, 4)
    X, Ps = A.encode(G, E, ef, segs, Vs)
    # --- encode
    Vflat = torch.cat([v.flatten() for v in Vs if v is not None]).to(DEV)
    g_d = G.to(DEV)
    e_d = E.to(DEV) if E is not None else None
    stream = torch.cuda.current_stream().cuda_stream
    plan.encode(g_d, e_d, N.EF_CODE[ef], True, Vflat, stream)
    torch.cuda.synchronize()
    sk = plan.sketch_view.cpu()
    for s, P in zip(plan.segments, Ps):
        n = P.numel()
        got = sk[s.sketch_off:s.sketch_off + n].view_as(P)
        if s.kind == N.SEG_RAW:
            assert_bitwise(got, P, f"RAW sketch seg@{s.offset}")
        else:
            assert_close_rel(got, P, 2e-5, f"sketch seg@{s.offset} m={s.m}")
    if ef == "ef14":
        assert_bitwise(e_d, X, "E := G + E after encode")
    # --- select on the oracle's sketch: bit-exact energies and the exact tie rule
    ref_sketch = torch.cat([p.flatten() for p in Ps])
    plan.sketch[:ref_sketch.numel()].copy_(ref_sketch.to(DEV))
    energy = torch.empty(plan.info.rows_total, device=DEV)
    plan.row_energy(1, energy, stream)
    plan.select(1, stream)
    torch.cuda.synchronize()
    norms, _ = A.select(Ps, 1, segs)
    en = energy.cpu()
    for s, nrm in zip(plan.segments, norms):
        assert_bitwise(en[s.row_off:s.row_off + s.n], nrm, f"energy seg@{s.offset}")
    rows = _gpu_rows(plan)
    for r_, nrm, s in zip(rows, norms, plan.segments):
        diff = check_rows_tie_aware(r_, nrm, int(s.k_rows), band=0.0)
        assert diff == 0
        assert torch.all(r_[1:] > r_[:-1]), "row list must be ascending"
    sm = plan.slotmap.cpu()
    for s, r_ in zip(plan.segments, rows):
        slots = sm[s.row_off:s.row_off + s.n]
        assert int((slots >= 0).sum()) == s.k_rows
        assert torch.equal(slots[r_], torch.arange(s.k_rows, dtype=torch.int32))
    # --- pack (rows ascending) and residual
    Xo = X.clone()
    vals = A.pack(Xo, rows, segs, ef)
    plan.pack(g_d, e_d, N.EF_CODE[ef], stream)
    torch.cuda.synchronize()
    assert_bitwise(plan.packed_values(), vals, "packed values")
    if ef == "ef14":
        assert_bitwise(e_d, Xo, "EF14 residual")
    elif ef == "ef21":
        assert_bitwise(e_d, E + Xo, "EF21 residual")
    # --- decode
    out = torch.empty_like(g_d)
    ge_d = gE.to(DEV) if gE is not None else None
    plan.decode(1, N.EF_CODE[ef], ge_d, out, stream)
    torch.cuda.synchronize()
    ref_out = A.decode(vals, 1, rows, segs, G.numel(), G.dtype)
    if ef == "ef21":
        ref_out = gE + ref_out
        sel_mask = torch.zeros(G.numel(), dtype=torch.bool)
        for s, r_ in zip(segs, rows):
            sel_mask[s.offset:s.offset + s.numel].view(s.n, s.m)[r_] = True
        assert_bitwise(ge_d.cpu()[sel_mask], ref_out[sel_mask], "gE (selected rows)")
        assert_bitwise(ge_d.cpu()[~sel_mask], gE[~sel_mask], "gE (untouched rows)")
    assert_bitwise(out, ref_out, "decoded bucket")


@pytest.mark.parametrize("ef,which", [("noef", "mix"), ("ef14", "mix"), ("ef21", "mix"),
                                      ("ef14", "large")])
def test_hook_end_to_end_vs_oracle(ef, which):
    shapes = SHAPE_SETS[which]
    numel = bucket_numel(shapes)
    st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                        use_error_feedback=ef, seed=1234)
    ost = A.OracleState(r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback=ef,
                        seed=1234)
    E = gE = None
    flips = 0
    for it in range(4):
        G = _rand_bucket(shapes, 100 + it)
        bucket = SyntheticBucket(G.to(DEV), shapes, index=0, is_last=True)
        out = group_topk_hook(st, bucket).wait()
        torch.cuda.synchronize()
        if ef == "ef21" and E is None:  # init call
            E, gE = G.clone(), G.clone()
            assert_bitwise(out, G, "EF21 init out")
            continue
        seed = ost.next_seed()
        plan = st._plans[0][1]
        rows = _gpu_rows(plan)
        first_ef14 = (ef == "ef14" and E is None)
        res = A.simulate_step([G], [None if first_ef14 else E], gE, shapes, 0.2, 4, ef, seed,
                              rows_override=rows, proj_device=DEV)
        for r_, nrm, s in zip(rows, res["norms"], plan.segments):
            flips += check_rows_tie_aware(r_, nrm, int(s.k_rows), band=2e-4)
        assert_bitwise(out, res["out"], f"it{it} output bucket")
        if ef in ("ef14", "ef21"):
            assert_bitwise(st.error_dict[0], res["E_new"][0], f"it{it} E")
            E = res["E_new"][0]
        if ef == "ef21":
            assert torch.equal(st.global_error_dict[0].cpu(), res["gE_new"])
            gE = res["gE_new"]
        assert st.iter == it + 1
    assert flips <= 2, f"{flips} rows differ from the oracle's selection (near-ties only)"
    assert numel == bucket.buffer().numel()


@pytest.mark.parametrize("name", [n for n in case_names("arc_") if n.endswith("ws1") and "bf16" not in n])
def test_golden_vectors_on_gpu(name):
    """Replay reference-generated golden vectors through the HIP hook."""
    g = Golden(name)
    m = g.meta
    shapes = [tuple(s) for s in m["shapes"]]
    st = GroupTopKState(None, r=m["r"], compress_ratio=m["ratio"],
                        start_compress_iter=m["start"], use_error_feedback=m["ef"], seed=m["seed"])
    st.projections = "host"  # the golden vectors come from the reference run on CPU
    for it in range(m["iters"]):
        G = g.t(0, it, "G")
        bucket = SyntheticBucket(G.to(DEV), shapes, index=0, is_last=True)
        out = group_topk_hook(st, bucket).wait()
        torch.cuda.synchronize()
        ties = m.get("ties", False)
        if g.has(0, it, "topk0_in") and not ties:
            plan = st._plans[0][1]
            for j, r_ in enumerate(_gpu_rows(plan)):
                ref = g.t(0, it, f"topk{j}_idx")
                assert sorted(r_.tolist()) == sorted(ref.tolist()), f"{name} it{it} seg{j} rows"
        if ties and g.has(0, it, "topk0_in"):
            plan = st._plans[0][1]
            for j, r_ in enumerate(_gpu_rows(plan)):
                check_rows_tie_aware(r_, g.t(0, it, f"topk{j}_in"), int(g.np(0, it, f"topk{j}_k")))
            # zero-energy ties select all-zero rows: outputs agree regardless of which
        assert_bitwise(out, g.t(0, it, "out"), f"{name} it{it} out")
        if g.has(0, it, "E"):
            assert_bitwise(st.error_dict[0], g.t(0, it, "E"), f"{name} it{it} E")
        if g.has(0, it, "gE"):
            assert_bitwise(st.global_error_dict[0], g.t(0, it, "gE"), f"{name} it{it} gE")
        assert st.comm_bits_this_round == int(g.np(0, it, "bits"))


@pytest.mark.parametrize("ef", ["noef", "ef14", "ef21"])
def test_headline_bucket_properties(ef):
    """16 x [2048, 2048] fp32 (256 MiB): size-independent invariants at full size."""
    shapes = [[2048, 2048]] * 16
    numel = bucket_numel(shapes)
    torch.manual_seed(0)
    G0 = torch.randn(numel, device=DEV)
    st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                        use_error_feedback=ef, seed=1234)
    bucket = SyntheticBucket(G0.clone(), shapes)
    group_topk_hook(st, bucket).wait()  # EF21: init call
    G1 = torch.randn(numel, device=DEV)
    E_before = st.error_dict[0].clone() if ef != "noef" else None
    gE_before = st.global_error_dict[0].clone() if ef == "ef21" else None
    bucket = SyntheticBucket(G1.clone(), shapes)
    out = group_topk_hook(st, bucket).wait()
    torch.cuda.synchronize()
    plan = st._plans[0][1]
    k_rows = plan.segments[0].k_rows
    assert k_rows == 409 and plan.info.values_len == 13_402_112
    rows = _gpu_rows(plan)
    energy = torch.empty(plan.info.rows_total, device=DEV)
    plan.row_energy(1, energy, torch.cuda.current_stream().cuda_stream)
    en = energy.cpu()
    sel = torch.zeros(numel // 2048, dtype=torch.bool)
    for s, r_ in zip(plan.segments, rows):
        e = en[s.row_off:s.row_off + s.n]
        mask = torch.zeros(s.n, dtype=torch.bool)
        mask[r_] = True
        assert e[mask].min() >= e[~mask].max(), "a dropped row outranks a selected one"
        sel[s.row_off:s.row_off + s.n] = mask
    out2 = out.view(-1, 2048)
    X = G1 if ef == "noef" else (G1 + E_before if ef == "ef14" else G1 - E_before)
    X2 = X.view(-1, 2048)
    selc = sel.to(DEV)
    if ef in ("noef", "ef14"):
        assert torch.equal(out2[~selc], torch.zeros_like(out2[~selc]))
        assert torch.equal(out2[selc], X2[selc])  # ws = 1: the mean is the row itself
    if ef == "ef14":  # conservation: out + E_new == G + E_old, bit for bit
        assert torch.equal(out + st.error_dict[0], X)
    if ef == "ef21":
        E2 = st.error_dict[0].view(-1, 2048)
        assert torch.equal(E2[~selc], E_before.view(-1, 2048)[~selc])
        assert torch.equal(E2[selc], (E_before.view(-1, 2048) + X2)[selc])
        assert torch.equal(out2[selc], (gE_before.view(-1, 2048) + X2)[selc])
        assert torch.equal(out2[~selc], gE_before.view(-1, 2048)[~selc])


def test_encode_rejects_bad_layout():
    buf = torch.zeros(100, device=DEV)
    st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0)
    with pytest.raises(RuntimeError):
        group_topk_hook(st, SyntheticBucket(buf, [[3, 5, 2], [70]]))  # 30 % 8 != 0


@pytest.mark.parametrize("ef", ["ef14", "ef21"])
def test_resume_from_state_dict_is_bit_identical(ef, tmp_path):
    """Checkpoint the hook state after two calls, restore it into a fresh state (and a
    fresh projection prefetcher) and continue: outputs and residuals match an
    uninterrupted run bit for bit."""
    shapes = MIX

    def mk():
        return GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                              use_error_feedback=ef, seed=55)

    def call(st, it):
        G = _rand_bucket(shapes, 300 + it).to(DEV)
        out = group_topk_hook(st, SyntheticBucket(G, shapes, index=0, is_last=True)).wait()
        torch.cuda.synchronize()
        return out.clone()

    ref = mk()
    ref_outs = [call(ref, it) for it in range(4)]
    a = mk()
    for it in range(2):
        call(a, it)
    torch.save(a.state_dict(), tmp_path / "ck.pt")
    b = mk()
    b.load_state_dict(torch.load(tmp_path / "ck.pt", weights_only=True), device=DEV)
    for it in range(2, 4):
        assert_bitwise(call(b, it), ref_outs[it], f"resumed it{it}")
    assert_bitwise(b.error_dict[0], ref.error_dict[0], "resumed E")
    assert b.iter == ref.iter


def test_resume_from_cpu_checkpoint_without_device():
    """A checkpoint loaded with map_location='cpu' and no device argument: the hook moves
    the residuals to the bucket's device on first use (never hands a host pointer to a
    kernel) and continues bit-identically."""
    shapes = MIX

    def mk():
        return GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                              use_error_feedback="ef21", seed=56)

    def call(st, it):
        G = _rand_bucket(shapes, 400 + it).to(DEV)
        out = group_topk_hook(st, SyntheticBucket(G, shapes, index=0, is_last=True)).wait()
        torch.cuda.synchronize()
        return out.clone()

    ref = mk()
    ref_outs = [call(ref, it) for it in range(4)]
    a = mk()
    for it in range(2):
        call(a, it)
    sd = {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in a.state_dict().items()}
    sd["error_dict"] = {b: t.cpu() for b, t in sd["error_dict"].items()}
    sd["global_error_dict"] = {b: t.cpu() for b, t in sd["global_error_dict"].items()}
    b = mk()
    b.load_state_dict(sd)
    assert b.error_dict[0].device.type == "cpu"
    for it in range(2, 4):
        assert_bitwise(call(b, it), ref_outs[it], f"resumed it{it}")
    assert b.error_dict[0].is_cuda and b.global_error_dict[0].is_cuda


def test_plan_follows_a_rebuilt_bucket_on_the_same_buffer():
    """DDP rebuilds its buckets after the first iteration and the caching allocator may
    give the new bucket the old buffer: same pointer and numel, other tensors.  The hook
    must notice the new layout (shapes re-checked during the first iterations after
    compression starts) and encode with a plan of the new geometry."""
    shapes_a = [[64, 256], [128], [32, 16, 3, 3], [200, 96]]
    shapes_b = [[200, 96], [32, 16, 3, 3], [64, 256], [128]]  # same numel, other order
    assert bucket_numel(shapes_a) == bucket_numel(shapes_b)
    st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                        use_error_feedback="noef", seed=8)
    ost = A.OracleState(seed=8)
    buf = torch.empty(bucket_numel(shapes_a), device=DEV)
    for it, shapes in enumerate([shapes_a, shapes_b, shapes_b]):
        G = _rand_bucket(shapes, 600 + it)
        buf.copy_(G)
        out = group_topk_hook(st, SyntheticBucket(buf, shapes, index=0, is_last=True)).wait()
        torch.cuda.synchronize()
        plan = st._plans[0][1]
        assert [tuple(s) for s in plan.shapes] == [tuple(s) for s in shapes]
        seed = ost.next_seed()
        rows = _gpu_rows(plan)
        res = A.simulate_step([G], [None], None, shapes, 0.2, 4, "noef", seed, rows_override=rows,
                              proj_device=DEV)
        assert_bitwise(out, res["out"], f"call {it} output")


def test_device_rng_left_where_the_reference_leaves_it():
    """After a compressed call the global generators sit where the reference's would: the
    CPU generator freshly seeded with the call's seed, the bucket device's generator
    seeded and advanced past one torch.randn(m, r) per 2-D/ND tensor (ref :49, :79, :255)."""
    shapes = [[64, 256], [128], [32, 16, 3, 3], [200, 96], [40000, 4]]
    st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                        use_error_feedback="noef", seed=12)
    seed = A.OracleState(seed=12).next_seed()
    group_topk_hook(st, SyntheticBucket(_rand_bucket(shapes, 1).to(DEV), shapes)).wait()
    torch.cuda.synchronize()
    after_hook = (torch.cuda.default_generators[0].get_offset(),
                  torch.randn(3, device=DEV).cpu(), torch.randn(3).clone())
    torch.manual_seed(seed)  # the reference's draws, on the device
    for s in A.segments(shapes, 0.2):
        if s.kind == A.SKETCH:
            torch.randn(s.m, 4, device=DEV)
    ref = (torch.cuda.default_generators[0].get_offset(), torch.randn(3, device=DEV).cpu(),
           torch.randn(3).clone())
    assert after_hook[0] == ref[0]
    assert torch.equal(after_hook[1], ref[1]) and torch.equal(after_hook[2], ref[2])


@pytest.mark.parametrize("fill", ["zero", "two_levels"])
def test_select_degenerate_energies(fill):
    """All-equal energies (zero gradients) and two energy levels on large segments: the
    exact tie rule picks the lowest rows, through the full-rescan select path."""
    shapes = [tuple(s) for s in LARGE[:5]]
    segs = A.segments(shapes, 0.2)
    plan = BucketPlan(shapes, 4, 0.2, torch.float32, DEV)
    stream = torch.cuda.current_stream().cuda_stream
    Ps = []
    for s in segs:
        if fill == "zero":
            P = torch.zeros(s.n, 4)
        else:
            lv = (torch.arange(s.n) % 3 == 0).float() * 2.0 + 1.0
            P = lv[:, None].expand(s.n, 4).contiguous()
        Ps.append(P[:, 0].contiguous() if s.kind == A.RAW else P)
    ref = torch.cat([p.flatten() for p in Ps])
    plan.sketch[:ref.numel()].copy_(ref.to(DEV))
    plan.select(1, stream)
    torch.cuda.synchronize()
    norms, _ = A.select(Ps, 1, segs)
    for r_, nrm, s in zip(_gpu_rows(plan), norms, plan.segments):
        assert check_rows_tie_aware(r_, nrm, int(s.k_rows), band=0.0) == 0
        assert torch.all(r_[1:] > r_[:-1])


@pytest.mark.parametrize("fill", ["band", "zero_rows"])
def test_select_crowded_first_bin(fill):
    """The k-th energy's 12-bit first-pass bin holding far more candidates than a write block
    stages (the fused refine-in-write path's global-memory rounds): "band" = every energy
    distinct inside one bin, so both 10-bit rounds run; "zero_rows" = 90 % all-zero rows
    around ragged non-zero ones (the Llama embedding case), resolved by the shared-bit
    decision.  Exact top-k under the tie rule, ascending rows."""
    shapes = [(200000, 8), (70000, 8), (300, 4)]
    segs = A.segments(shapes, 0.2)
    plan = BucketPlan(shapes, 4, 0.2, torch.float32, DEV)
    stream = torch.cuda.current_stream().cuda_stream
    gen = torch.Generator().manual_seed(5)
    Ps = []
    for s in segs:
        P = torch.zeros(s.n, 4)
        if fill == "band":  # energies in [1, 1 + 1/17): one 12-bit bin of the key bits
            P[:, 0] = torch.sqrt(1.0 + torch.rand(s.n, generator=gen) / 17.0)
        else:
            nz = torch.arange(s.n) % 10 == 3
            P[nz] = torch.randn(int(nz.sum()), 4, generator=gen)
        Ps.append(P)
    ref = torch.cat([p.flatten() for p in Ps])
    plan.sketch[:ref.numel()].copy_(ref.to(DEV))
    plan.select(1, stream)
    torch.cuda.synchronize()
    norms, _ = A.select(Ps, 1, segs)
    for r_, nrm, s in zip(_gpu_rows(plan), norms, plan.segments):
        assert check_rows_tie_aware(r_, nrm, int(s.k_rows), band=0.0) == 0
        assert torch.all(r_[1:] > r_[:-1])


def test_select_across_calls_with_jumping_energies():
    """The multi-block select on one plan over calls whose energies stay put, jump by 1e5 up or
    1e-7 down, collapse to ties or to zero, and come back (its workspace -- histograms, item
    states, arrival counters -- is left clean by each call): every call exact under the tie
    rule (1 M-row 1x1-conv items, 131 K-row 3x3 items, a 40 K-row 2-D item, and 1-D tensors
    riding along)."""
    shapes = [(2048, 1024, 1, 1), (512, 512, 3, 3), (40000, 8), (2048,), (512,)]
    segs = A.segments(shapes, 0.2)
    plan = BucketPlan(shapes, 4, 0.2, torch.float32, DEV)
    stream = torch.cuda.current_stream().cuda_stream
    gen = torch.Generator().manual_seed(11)
    for call, scale in enumerate([1.0, 1.0, 1.5, 1e5, 1e5, 1e-7, 0.0, 1.0, 300.0]):
        Ps = []
        for s in segs:
            w = s.n if s.kind == A.RAW else s.n * 4
            P = (torch.randn(w, generator=gen) * scale).reshape(-1, 1 if s.kind == A.RAW else 4)
            if call == 4:  # half the rows tied at one value
                P[::2] = P[0]
            Ps.append(P[:, 0].contiguous() if s.kind == A.RAW else P)
        ref = torch.cat([p.flatten() for p in Ps])
        plan.sketch[:ref.numel()].copy_(ref.to(DEV))
        plan.select(1, stream)
        torch.cuda.synchronize()
        norms, _ = A.select(Ps, 1, segs)
        for j, (r_, nrm, s) in enumerate(zip(_gpu_rows(plan), norms, plan.segments)):
            sm = plan.slotmap[s.row_off:s.row_off + s.n].cpu()
            kth = torch.topk(nrm.double(), int(s.k_rows)).values.min().item()
            assert torch.unique(r_).numel() == int(s.k_rows), (
                f"call {call} (scale {scale}) seg {j}: {torch.unique(r_).numel()} distinct rows of "
                f"{int(s.k_rows)}, {int((sm >= 0).sum())} slots set, k-th energy {kth:.6e}, "
                f"{int((nrm.double() > kth).sum())} above it, {int((nrm.double() == kth).sum())} equal")
            assert check_rows_tie_aware(r_, nrm, int(s.k_rows), band=0.0) == 0, f"call {call} seg {j}"
            assert torch.all(r_[1:] > r_[:-1]), f"call {call} seg {j}: rows not ascending"
            sm = plan.slotmap[s.row_off:s.row_off + s.n].cpu()
            assert torch.equal(sm[r_], torch.arange(int(s.k_rows), dtype=sm.dtype)), f"call {call} seg {j} slots"
            assert int((sm >= 0).sum()) == int(s.k_rows)


@pytest.mark.parametrize("name", [n for n in case_names("arc_") if "bf16" in n and n.endswith("ws1")])
def test_bf16_golden_on_gpu(name):
    """bf16 buckets against reference-generated golden vectors.

    bf16 norms tie often at the k-th value and the reference's topk tie order is
    implementation-defined, so: energies from the reference's own sketch are compared
    bit for bit, the device's selected rows must satisfy the reference's norms under the
    tie rule (within one bf16 rounding of the sketch), and every output / residual is
    bit-exact against the oracle (pinned to the same golden vectors) given those rows.
    """
    g = Golden(name)
    m = g.meta
    shapes = [tuple(s) for s in m["shapes"]]
    ef = m["ef"]
    segs = A.segments(shapes, m["ratio"])
    st = GroupTopKState(None, r=m["r"], compress_ratio=m["ratio"],
                        start_compress_iter=m["start"], use_error_feedback=ef, seed=m["seed"])
    st.projections = "host"  # the golden vectors come from the reference run on CPU
    ost = A.OracleState(seed=m["seed"])
    E_prev = gE_prev = None
    stream = torch.cuda.current_stream().cuda_stream
    for it in range(m["iters"]):
        G = g.t(0, it, "G")
        assert G.dtype == torch.bfloat16
        out = group_topk_hook(st, SyntheticBucket(G.to(DEV), shapes, index=0, is_last=True)).wait()
        torch.cuda.synchronize()
        if ef == "ef21" and E_prev is None:  # dense init call: bit-exact vs the reference
            assert_bitwise(out, g.t(0, it, "out"), f"{name} it{it} init out")
            E_prev, gE_prev = G.clone(), g.t(0, it, "gE")
            assert_bitwise(st.global_error_dict[0], gE_prev, f"{name} it{it} init gE")
            continue
        plan = st._plans[0][1]
        rows = _gpu_rows(plan)
        # select math on the reference's own (all-reduced) sketch: bit-exact energies
        ref_sk = torch.cat([g.t(0, it, f"AR{j}").flatten() for j in range(len(segs))])
        plan.sketch[:ref_sk.numel()].copy_(ref_sk.to(DEV))
        energy = torch.empty(plan.info.rows_total, device=DEV)
        plan.row_energy(1, energy, stream)
        torch.cuda.synchronize()
        en = energy.cpu()
        for j, s in enumerate(plan.segments):
            ref_norm = g.t(0, it, f"topk{j}_in").float()
            assert_bitwise(en[s.row_off:s.row_off + s.n], ref_norm, f"{name} it{it} energy seg{j}")
            # rows chosen from the device's own sketch: the reference's norms, tie rule, one
            # bf16 rounding (2^-8 relative) of band for sketch values summed in another order
            check_rows_tie_aware(rows[j], ref_norm, int(s.k_rows), band=2.0 ** -7)
        seed = ost.next_seed()
        assert int(g.np(0, it, "seed")[0]) == seed
        res = A.simulate_step([G], [E_prev], gE_prev, shapes, m["ratio"], m["r"], ef, seed,
                              rows_override=rows)
        assert_bitwise(out, res["out"], f"{name} it{it} out given the rows")
        if ef != "noef":
            assert_bitwise(st.error_dict[0], res["E_new"][0], f"{name} it{it} E given the rows")
            E_prev = res["E_new"][0]
        if ef == "ef21":
            assert_bitwise(st.global_error_dict[0], res["gE_new"], f"{name} it{it} gE")
            gE_prev = res["gE_new"]
        assert st.comm_bits_this_round == int(g.np(0, it, "bits"))


def test_bf16_headline_bucket_properties():
    """16 x [2048, 2048] bf16 (128 MiB), EF14: exact k, kept rows outrank dropped rows, and
    out + E_new == G + E_old bit for bit (all in bf16)."""
    shapes = [[2048, 2048]] * 16
    numel = bucket_numel(shapes)
    torch.manual_seed(0)
    st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                        use_error_feedback="ef14", seed=1234)
    group_topk_hook(st, SyntheticBucket(torch.randn(numel, device=DEV).bfloat16(), shapes)).wait()
    G1 = torch.randn(numel, device=DEV).bfloat16()
    E_before = st.error_dict[0].clone()
    assert E_before.dtype == torch.bfloat16
    out = group_topk_hook(st, SyntheticBucket(G1.clone(), shapes)).wait()
    torch.cuda.synchronize()
    plan = st._plans[0][1]
    rows = _gpu_rows(plan)
    energy = torch.empty(plan.info.rows_total, device=DEV)
    plan.row_energy(1, energy, torch.cuda.current_stream().cuda_stream)
    en = energy.cpu()
    for s, r_ in zip(plan.segments, rows):
        assert r_.numel() == s.k_rows == 409
        e = en[s.row_off:s.row_off + s.n]
        mask = torch.zeros(s.n, dtype=torch.bool)
        mask[r_] = True
        assert e[mask].min() >= e[~mask].max(), "a dropped row outranks a selected one"
    X = G1 + E_before  # bf16 add, as the reference's input_tensor.add_(error)
    assert torch.equal(out + st.error_dict[0], X)


def test_device_bf16_rounding_matches_torch():
    """The kernels' fp32 -> bf16 rounding (gfx950 v_cvt_pk_bf16_f32 + NaN fix-up) equals
    torch's CPU .to(bfloat16) bit for bit: random values over the whole exponent range,
    exact ties, subnormals, signed zeros, infinities, NaN."""
    g = torch.Generator().manual_seed(7)
    bits = torch.randint(0, 2 ** 32, (1 << 20,), generator=g, dtype=torch.int64)
    special = torch.tensor([0x00000001, 0x00008000, 0x00018000, 0x007FFFFF, 0x00800000, 0x3F808000,
                            0x3F818000, 0x3F80FFFF, 0x7F7FFFFF, 0x7F800000, 0xFF800000, 0x80000000,
                            0x00000000, 0x7FC00001, 0xFFFFFFFF, 0x7F808000, 0x80008000],
                           dtype=torch.int64)
    x = torch.cat([bits, special]).to(torch.int32).view(torch.float32)
    # c10::BFloat16's round_to_nearest_even, restated on the bits (torch's vectorised CPU
    # casts may use the host's bf16 instructions, which flush subnormals)
    u = torch.cat([bits, special]) & 0xFFFFFFFF
    ref = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    ref[torch.isnan(x)] = 0x7FC0
    ref = ref.to(torch.int32).to(torch.int16)
    xd = x.to(DEV)
    out = torch.empty(x.numel(), dtype=torch.int16, device=DEV)
    N.check(N.lib().arctopk_round_bf16(xd.data_ptr(), out.data_ptr(), x.numel(),
                                       torch.cuda.current_stream().cuda_stream), "arctopk_round_bf16")
    got = out.cpu()
    bad = (got != ref).nonzero().flatten()
    assert bad.numel() == 0, [(hex(int(x[i].view(torch.int32)) & 0xFFFFFFFF), hex(int(got[i]) & 0xFFFF),
                               hex(int(ref[i]) & 0xFFFF)) for i in bad[:5]]


@pytest.mark.parametrize("projections", ["host", "device"])
def test_projection_prestaging_under_reordering_and_reseed(projections):
    """Projections are prepared a call early for the predicted next (bucket, seed): host
    mode copies the CPU-stream V a call early, device mode draws it in the previous call's
    select launch (arctopk_select_draw).  Calls out of the predicted order, an rng
    repositioned between calls, and calls on another stream must still encode with the
    projections of their own seed: every call's rows are checked against the oracle's
    energies (wrong projections would rank rows differently) and its output bit for bit.
    Bucket 1 has a segment large enough for the multi-block select, so the draw also rides
    in the refine launch."""
    shapes_a = [[256, 1024], [64, 512], [300], [32, 16, 3, 3]]
    shapes_b = [[128, 2048], [16, 8, 1, 1], [40, 96], [24000, 12]]
    layouts = {0: shapes_a, 1: shapes_b, 2: shapes_a}
    st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                        use_error_feedback="noef", seed=99)
    st.projections = projections
    ost = A.OracleState(r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback="noef",
                        seed=99)
    order = ([0, 1, 2] * 4 + [2, 0, 1, 1, 0] + [0, 1, 2] * 3 + ["reseed"] + [0, 1, 2] * 3 + [1, 2]
             + ["stream", 0, 1, "stream", 2, 0, "stream", 1, 2])
    flips = 0
    side = torch.cuda.Stream()
    on_side = False
    for step, b in enumerate(order):
        if b == "reseed":  # both rngs repositioned: the look-ahead's seeds no longer come true
            st.rng.manual_seed(4242)
            ost.rng.manual_seed(4242)
            continue
        if b == "stream":  # the caller moves to another stream (and back)
            on_side = not on_side
            continue
        shapes = layouts[b]
        G = _rand_bucket(shapes, 1000 + step)
        with torch.cuda.stream(side if on_side else torch.cuda.default_stream()):
            Gd = G.to(DEV)
            out = group_topk_hook(st, SyntheticBucket(Gd, shapes, index=b, is_last=(b == 2))).wait()
        torch.cuda.synchronize()
        seed = ost.next_seed()
        plan = st._plans[b][1]
        rows = _gpu_rows(plan)
        res = A.simulate_step([G], [None], None, shapes, 0.2, 4, "noef", seed, rows_override=rows,
                              proj_device=DEV if projections == "device" else None)
        for r_, nrm, s in zip(rows, res["norms"], plan.segments):
            flips += check_rows_tie_aware(r_, nrm, int(s.k_rows), band=2e-4)
        assert_bitwise(out, res["out"], f"call {step} (bucket {b}) output")
    assert flips <= 2, f"{flips} rows differ from the oracle's selection (near-ties only)"
    hits = st.prestage_hits if projections == "host" else st.predraw_hits
    assert hits > 10, f"projections prepared a call early were used {hits} times"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_device_projection_draw_matches_torch_randn_on_device(dtype):
    """arctopk_draw_projections reproduces the reference's projections as drawn on a GPU:
    torch.manual_seed(seed) then torch.randn(m, r, device=cuda, dtype) per 2-D/ND tensor
    in bucket order (group_topk_hook_no_reshape.py:49, :79, :255), bit for bit, including
    draws large enough that torch's grid saturates (threads loop, components 1-3 used); and
    arctopk_plan_philox_advance equals the device generator's offset after those draws."""
    import ctypes
    sets = [MIX, LARGE[:5], [[2048, 2048]] * 3 + [[7], [5632, 2048]],
            [[8, 300000], [2, 3, 3, 3], [10], [2, 140000]]]
    for si, shapes in enumerate(sets):
        shapes = [tuple(s) for s in shapes]
        plan = BucketPlan(shapes, 4, 0.2, dtype, DEV)
        segs = A.segments(shapes, 0.2)
        for seed in (0, 123456789, 999_999_999):
            V = torch.empty(max(1, plan.info.v_len), dtype=dtype, device=DEV)
            N.check(N.lib().arctopk_draw_projections(plan.handle, seed, V.data_ptr(),
                                                     torch.cuda.current_stream().cuda_stream),
                    "arctopk_draw_projections")
            torch.manual_seed(seed)
            ref = torch.cat([torch.randn(s.m, 4, device=DEV, dtype=dtype).flatten()
                             for s in segs if s.kind == A.SKETCH])
            off = torch.cuda.default_generators[0].get_offset()
            iv = torch.int16 if dtype == torch.bfloat16 else torch.int32
            got = V[:ref.numel()]
            bad = (got.view(iv) != ref.view(iv)).sum().item()
            assert bad == 0, f"set {si} seed {seed}: {bad} of {ref.numel()} values differ"
            adv = ctypes.c_uint64()
            N.check(N.lib().arctopk_plan_philox_advance(plan.handle, ctypes.byref(adv)), "advance")
            assert adv.value == off, f"set {si}: philox advance {adv.value} vs torch {off}"


@pytest.mark.parametrize("ef", ["ef14", "ef21"])
def test_torch_op_layer_matches_direct_calls(ef):
    """torch.ops.arctopk.* (allreducetopk_amd/ops.py) run the same kernels as the C entry
    points: one call through the ops and one through the BucketPlan methods on identical
    inputs give bit-identical sketch, rows, slots, packed values, residuals and output."""
    import allreducetopk_amd.ops  # noqa: F401
    shapes = [tuple(s) for s in MIX]
    code = N.EF_CODE[ef]
    outs = []
    for use_ops in (False, True):
        plan = BucketPlan(shapes, 4, 0.2, torch.float32, DEV)
        h = plan.handle.value
        G = _rand_bucket(MIX, 77).to(DEV)
        E = _rand_bucket(MIX, 78).to(DEV) * 0.1
        gE = _rand_bucket(MIX, 79).to(DEV)
        V = plan.V_ring[0]
        s = torch.cuda.current_stream().cuda_stream
        if use_ops:
            torch.ops.arctopk.draw_projections(h, 12345, V)
            torch.ops.arctopk.encode(h, G, E, code, True, V, plan.sketch)
            torch.ops.arctopk.select(h, plan.sketch, 1, plan.rowlist, plan.slotmap)
            torch.ops.arctopk.pack(h, G, E, code, plan.rowlist, plan.slotmap, plan.packed)
            torch.ops.arctopk.decode(h, plan.packed, plan.slotmap, 1, code,
                                     gE if ef == "ef21" else None, G)
        else:
            N.check(N.lib().arctopk_draw_projections(plan.handle, 12345, V.data_ptr(), s), "draw")
            plan.encode(G, E, code, True, V, s)
            plan.select(1, s)
            plan.pack(G, E, code, s)
            plan.decode(1, code, gE if ef == "ef21" else None, G, s)
        torch.cuda.synchronize()
        outs.append([t.clone().cpu() for t in (plan.sketch, plan.rowlist, plan.slotmap, plan.packed, E, gE, G)])
    for a, b_, what in zip(outs[0], outs[1], ("sketch", "rowlist", "slotmap", "packed", "E", "gE", "out")):
        assert_bitwise(b_, a, f"ops vs direct: {what}")


@pytest.mark.parametrize("ef", ["noef", "ef21"])
def test_public_decode_needs_only_its_slot_map(ef):
    """arctopk_decode on a fresh plan with a slot map and packed buffer built by the caller (no
    select or pack ever ran on the plan), then again after a pack of OTHER rows on the same
    plan: the short-row (mode 3) chunks derive their packed ranges from the slot map handed in,
    never from the plan's last pack."""
    shapes = [[40, 16, 3, 3], [10], [96, 40], [64, 64, 3, 3], [33, 130], [8, 8, 5, 5]]
    segs = A.segments(shapes, 0.2)
    numel = bucket_numel(shapes)
    plan = BucketPlan([tuple(s) for s in shapes], 4, 0.2, torch.float32, DEV)
    stream = torch.cuda.current_stream().cuda_stream
    ws = 2
    for trial in range(2):
        g = torch.Generator().manual_seed(77 + trial)
        rows = [torch.sort(torch.randperm(s.n, generator=g)[:s.k_rows]).values for s in plan.segments]
        sm = torch.full((plan.info.rows_total,), -1, dtype=torch.int32)
        packed = torch.zeros(plan.info.packed_len)
        vals = []
        for s, r_ in zip(plan.segments, rows):
            sm[s.row_off + r_] = torch.arange(s.k_rows, dtype=torch.int32)
            v = torch.randn(s.k_rows * s.m, generator=g)
            packed[s.packed_off:s.packed_off + v.numel()] = v
            vals.append(v)
        gE = torch.randn(numel, generator=g)
        out = torch.full((numel,), float("nan"), device=DEV)
        gE_d = gE.to(DEV) if ef == "ef21" else None
        packed_d, sm_d = packed.to(DEV), sm.to(DEV)  # (kept alive: the allocator reuses freed blocks)
        N.check(N.lib().arctopk_decode(plan.handle, packed_d.data_ptr(), sm_d.data_ptr(), ws,
                                       N.EF_CODE[ef], N.ptr(gE_d), out.data_ptr(), stream), "arctopk_decode")
        torch.cuda.synchronize()
        ref = A.decode(torch.cat(vals), ws, rows, segs, numel, torch.float32)
        if ef == "ef21":  # out = gE + scatter(mean); gE[sel] = out[sel]
            ref = gE + ref
            assert_bitwise(gE_d, ref, f"trial {trial} gE")
        assert_bitwise(out, ref, f"trial {trial} output")
        if trial == 0:  # a pack of other rows on the same plan rewrites the plan's own chunk table
            G = _rand_bucket(shapes, 5).to(DEV)
            plan.encode(G, None, N.EF_NONE, True, torch.randn(max(1, plan.info.v_len), device=DEV), stream)
            plan.select(1, stream)
            plan.pack(G, None, N.EF_NONE, stream)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("ef", ["noef", "ef14", "ef21"])
def test_row_path_sketch_matches_fp32_accumulation(dtype, ef):
    """The wave-per-row encode (m >= 64) of every dtype against the sketch the reference forms,
    X.view(n, m) @ V with fp32 accumulation and one rounding to the bucket dtype (CPU `mm`;
    another summation order: within one rounding of the dtype).  Structured inputs pin the
    column <-> projection pairing exactly (a bf16 path that paired the wrong elements passed
    every property test of round 5: the bf16 goldens have no m >= 64 tensor)."""
    shapes = [[16, 64], [8], [64, 128], [100, 72], [256, 2048]]
    n_el = bucket_numel(shapes)
    g = torch.Generator().manual_seed(17)
    G = torch.randn(n_el, generator=g).to(dtype)
    E = torch.randn(n_el, generator=g).to(dtype)
    p = BucketPlan([tuple(s) for s in shapes], 4, 0.2, dtype, DEV)
    V = torch.randn(p.info.v_len, generator=g).to(dtype)
    code = {"noef": N.EF_NONE, "ef14": N.EF14, "ef21": N.EF21}[ef]
    Ed = E.to(DEV)
    p.encode(G.to(DEV), Ed if ef != "noef" else None, code, True, V.to(DEV), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    X = G if ef == "noef" else (G + E if ef == "ef14" else G - E)  # rounded to the dtype, as the reference
    sk = p.sketch.cpu()
    tol = 2.0 ** -7 if dtype == torch.bfloat16 else 2e-5
    for s in p.segments:
        if s.kind == N.SEG_RAW:
            continue
        x = X[s.offset:s.offset + s.n * s.m].view(s.n, s.m).float()
        v = V[s.v_off:s.v_off + s.m * 4].view(s.m, 4).float()
        ref = (x @ v).to(dtype).float()
        d = sk[s.sketch_off:s.sketch_off + s.n * 4].view(s.n, 4).float()
        scale = (x.abs() @ v.abs()).clamp_min(1e-30)  # the sum's magnitude bounds its rounding
        bad = ((d - ref).abs() > tol * scale).sum().item()
        assert bad == 0, f"{dtype} {ef} [{s.n}, {s.m}]: {bad} sketch entries off by more than one rounding"
    if ef == "ef14":
        assert torch.equal(Ed.cpu(), X), "E := G + E (rounded to the dtype)"
    # the pairing, exactly: G[r][c] = c + 1 and V[c][j] = [c == j]  ->  sketch[r][j] = j + 1
    q = BucketPlan([(4, 64)], 4, 0.25, dtype, DEV)
    Gc = (torch.arange(64, dtype=torch.float32) + 1).repeat(4).to(dtype)
    Vi = torch.zeros(64, 4)
    for j in range(4):
        Vi[j, j] = 1.0
    q.encode(Gc.to(DEV), None, N.EF_NONE, True, Vi.flatten().to(dtype).to(DEV), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = torch.tensor([1.0, 2.0, 3.0, 4.0]).repeat(4, 1)
    assert torch.equal(q.sketch[:16].view(4, 4).float().cpu(), want)
