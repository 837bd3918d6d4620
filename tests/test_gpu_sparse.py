"""TopK / RandK HIP path vs the CPU oracle and the reference's golden vectors (MI355X)."""
import pytest
import torch

from allreducetopk_amd import _native as N
from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel
from allreducetopk_amd.comm_hooks import sparse_hook, sparse_hook_c4
from golden_io import Golden, case_names
from oracle import sparse as S
from parity import assert_bitwise, check_rows_tie_aware, device_randk_hash, ensure_group

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SHAPES = [[10], [40, 16], [4, 3, 3, 3], [96, 40], [256, 512], [1000], [3, 7]]
# more tensors than one select batch (48), and tensors large enough for many hist blocks
LARGE = [[300000], [3, 5], [1000, 300], [512, 64, 3, 3]] + [[2000]] * 60
SHAPE_SETS = {"small": SHAPES, "large": LARGE}


@pytest.fixture(scope="module", autouse=True)
def group():
    ensure_group("nccl")
    yield


def _rand(shapes, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(bucket_numel(shapes), generator=g)


@pytest.mark.parametrize("ef,which", [("noef", "small"), ("ef14", "small"), ("ef21", "small"),
                                      ("ef14", "large"), ("ef21", "large")])
def test_topk_hook_vs_oracle(ef, which):
    shapes = SHAPE_SETS[which]
    st = sparse_hook.SparseState(None, compress_ratio=0.2, start_compress_iter=0,
                                 sparse_type="tensor", random=False, use_error_feedback=ef)
    E = gE = None
    for it in range(3):
        G = _rand(shapes, 50 + it)
        out = sparse_hook.sparse_hook_sync(st, SyntheticBucket(G.to(DEV), shapes)).wait()
        torch.cuda.synchronize()
        if ef == "ef21" and E is None:
            E, gE = G.clone(), G.clone()
            continue
        res = S.simulate_step([G], [E if not (ef == "ef14" and E is None) else None], gE, shapes,
                              0.2, ef, False, None)
        assert_bitwise(out, res["out"], f"it{it} out")
        if ef != "noef":
            assert_bitwise(st.error_dict[0], res["E_new"][0], f"it{it} E")
            E = res["E_new"][0]
        if ef == "ef21":
            assert_bitwise(st.global_error_dict[0], res["gE_new"], f"it{it} gE")
            gE = res["gE_new"]


def test_topk_select_kernel_ties_and_order():
    """Exact tie rule (lowest index first) and ascending output on a tie-heavy tensor."""
    L = N.lib()
    n = 100_000
    x = torch.zeros(n)
    g = torch.Generator().manual_seed(3)
    nz = torch.randperm(n, generator=g)[:30_000]
    x[nz] = torch.randn(30_000, generator=g)
    x[nz[:500]] = 2.5          # a large block of exact |x| ties
    x[nz[500:1000]] = -2.5
    k = 20_000
    xd = x.to(DEV)
    idx = torch.empty(k, dtype=torch.int32, device=DEV)
    vals = torch.empty(k, device=DEV)
    ws = torch.empty(int(L.arctopk_sparse_workspace_bytes(1, N.i64_array([n]))), dtype=torch.uint8,
                     device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    N.check(L.arctopk_topk_select(xd.data_ptr(), 1, N.i64_array([0]), N.i64_array([n]),
                                  N.i64_array([k]), N.i64_array([0]), idx.data_ptr(),
                                  vals.data_ptr(), ws.data_ptr(), 0, 0, st), "topk_select")
    torch.cuda.synchronize()
    i = idx.cpu().long()
    assert torch.all(i[1:] > i[:-1])
    assert torch.equal(vals.cpu(), x[i])
    check_rows_tie_aware(i, x.abs(), k, band=0.0)
    # zero ties: k beyond the non-zeros selects the lowest-index zeros
    k2 = 40_000
    idx2 = torch.empty(k2, dtype=torch.int32, device=DEV)
    vals2 = torch.empty(k2, device=DEV)
    N.check(L.arctopk_topk_select(xd.data_ptr(), 1, N.i64_array([0]), N.i64_array([n]),
                                  N.i64_array([k2]), N.i64_array([0]), idx2.data_ptr(),
                                  vals2.data_ptr(), ws.data_ptr(), 0, 0, st), "topk_select")
    torch.cuda.synchronize()
    assert check_rows_tie_aware(idx2.cpu(), x.abs(), k2, band=0.0) == 0


@pytest.mark.parametrize("case", ["constant", "mostly_zero", "two_values"])
def test_topk_select_degenerate_large(case):
    """Multi-range tensors whose k-th |x| bin is too full for the candidate list (the
    select rescans the full tensor) and exact ties across many ranges."""
    L = N.lib()
    n = 3_000_000
    g = torch.Generator().manual_seed(11)
    if case == "constant":
        x = torch.full((n,), -0.75)
    elif case == "mostly_zero":
        x = torch.zeros(n)
        nz = torch.randperm(n, generator=g)[:200_000]
        x[nz] = torch.randn(200_000, generator=g)
    else:
        x = torch.where(torch.rand(n, generator=g) < 0.5, torch.tensor(1.5), torch.tensor(-3.0))
    k = 600_000
    numels = [n, 5000]
    ks = [k, 1000]
    xd = torch.cat([x, torch.randn(5000, generator=g)]).to(DEV)
    idx = torch.empty(sum(ks), dtype=torch.int32, device=DEV)
    vals = torch.empty(sum(ks), device=DEV)
    ws = torch.empty(int(L.arctopk_sparse_workspace_bytes(2, N.i64_array(numels))), dtype=torch.uint8,
                     device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    N.check(L.arctopk_topk_select(xd.data_ptr(), 2, N.i64_array([0, n]), N.i64_array(numels),
                                  N.i64_array(ks), N.i64_array([0, k]), idx.data_ptr(),
                                  vals.data_ptr(), ws.data_ptr(), 0, 0, st), "topk_select")
    torch.cuda.synchronize()
    i = idx.cpu().long()
    xa = xd.cpu()
    assert check_rows_tie_aware(i[:k], x.abs(), k, band=0.0) == 0
    assert torch.all(i[1:k] > i[:k - 1])
    assert torch.equal(vals.cpu()[:k], x[i[:k]])
    assert check_rows_tie_aware(i[k:], xa[n:].abs(), 1000, band=0.0) == 0
    if case == "constant":
        assert torch.equal(i[:k], torch.arange(k))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("zero", [0, 1])
def test_randk_select_kernel_vs_restatement(dtype, zero):
    """arctopk_randk_select against the restated index rule (oracle randk_hash_indices):
    bit-exact ascending indices per tensor, gathered values, and (zero_selected) x with
    exactly those entries zeroed -- over tensors from n = 1 and k = n to a multi-range 3M
    tensor, more tensors than one launch batch."""
    L = N.lib()
    g = torch.Generator().manual_seed(21)
    numels = [1, 7, 64, 1000, 4096, 65_537, 3_000_000] + [300 + 37 * i for i in range(40)]
    ks = [1, 7, 13, 1, 4096, 13_107, 600_000] + [max(1, (300 + 37 * i) // 5) for i in range(40)]
    offs = [sum(numels[:i]) for i in range(len(numels))]
    kof = [sum(ks[:i]) for i in range(len(ks))]
    x = torch.randn(sum(numels), generator=g).to(dtype)
    xd = x.to(DEV)
    idx = torch.empty(sum(ks), dtype=torch.int32, device=DEV)
    vals = torch.empty(sum(ks), dtype=dtype, device=DEV)
    ws = torch.empty(int(L.arctopk_sparse_workspace_bytes(len(numels), N.i64_array(numels))),
                     dtype=torch.uint8, device=DEV)
    seed = 123_456_789
    N.check(L.arctopk_randk_select(xd.data_ptr(), len(numels), N.i64_array(offs), N.i64_array(numels),
                                   N.i64_array(ks), N.i64_array(kof), seed, idx.data_ptr(),
                                   vals.data_ptr(), ws.data_ptr(), N.DTYPE_CODE[dtype], zero,
                                   torch.cuda.current_stream().cuda_stream), "randk_select")
    torch.cuda.synchronize()
    i, v, xo = idx.cpu().long(), vals.cpu(), xd.cpu()
    expect_x = x.clone()
    for t, (n, k, o, ko) in enumerate(zip(numels, ks, offs, kof)):
        ref = S.randk_hash_indices(n, k, seed, t).long()
        assert torch.equal(i[ko:ko + k], ref), f"tensor {t} (n={n}, k={k}) indices"
        assert torch.equal(v[ko:ko + k], x[o + ref]), f"tensor {t} values"
        if zero:
            expect_x[o + ref] = 0
    assert_bitwise(xo, expect_x, "x after the select")


@pytest.mark.parametrize("err_in", [1, 0])
def test_topk_select_ef14_fold(err_in):
    """arctopk_topk_select_ef14 (the EF14 fold in the first histogram pass) gives the bits of
    arctopk_ef14_fold then arctopk_topk_select(E, zero_selected=1); a tensor of numel % 4 != 0 is
    refused (ARCTOPK_EINVAL, nothing enqueued) and the hook then folds first."""
    L = N.lib()
    g = torch.Generator().manual_seed(23)
    numels = [4096, 65_536, 1_000_000, 8, 3_000_000] + [1024 + 64 * i for i in range(40)]
    ks = [1, 13_107, 200_000, 3, 600_000] + [max(1, (1024 + 64 * i) // 5) for i in range(40)]
    offs = [sum(numels[:i]) for i in range(len(numels))]
    kof = [sum(ks[:i]) for i in range(len(ks))]
    G = torch.randn(sum(numels), generator=g)
    E0 = torch.randn(sum(numels), generator=g)
    E0[offs[3]:offs[3] + 8] = 0.5  # ties across G + E
    G[offs[3]:offs[3] + 8] = 0.25
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(int(L.arctopk_sparse_workspace_bytes(len(numels), N.i64_array(numels))),
                     dtype=torch.uint8, device=DEV)
    args = (len(numels), N.i64_array(offs), N.i64_array(numels), N.i64_array(ks), N.i64_array(kof))
    # reference: fold, then select
    Gr, Er = G.to(DEV), E0.to(DEV)
    idx_r = torch.empty(sum(ks), dtype=torch.int32, device=DEV)
    val_r = torch.empty(sum(ks), device=DEV)
    N.check(L.arctopk_ef14_fold(Gr.data_ptr(), Er.data_ptr(), Gr.numel(), err_in, 0, st), "fold")
    N.check(L.arctopk_topk_select(Er.data_ptr(), *args, idx_r.data_ptr(), val_r.data_ptr(), ws.data_ptr(), 0, 1,
                                  st), "select")
    # fused
    Gd, Ed = G.to(DEV), E0.to(DEV)
    idx = torch.empty(sum(ks), dtype=torch.int32, device=DEV)
    val = torch.empty(sum(ks), device=DEV)
    N.check(L.arctopk_topk_select_ef14(Gd.data_ptr(), Ed.data_ptr(), err_in, *args, idx.data_ptr(),
                                       val.data_ptr(), ws.data_ptr(), 0, st), "select_ef14")
    torch.cuda.synchronize()
    assert_bitwise(idx, idx_r, "indices")
    assert_bitwise(val, val_r, "values")
    assert_bitwise(Ed, Er, "E")
    assert_bitwise(Gd, G, "G untouched")
    bad = [7] + numels[1:]
    assert L.arctopk_topk_select_ef14(Gd.data_ptr(), Ed.data_ptr(), err_in, len(bad), N.i64_array(offs),
                                      N.i64_array(bad), N.i64_array([1] + ks[1:]), N.i64_array(kof),
                                      idx.data_ptr(), val.data_ptr(), ws.data_ptr(), 0, st) == N.EINVAL


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("err_in", [1, 0])
def test_randk_select_ef14_fold(dtype, err_in):
    """arctopk_randk_select_ef14: the EF14 pre-apply folded into the draw's write pass gives the
    bits of arctopk_ef14_fold then arctopk_randk_select(E, zero_selected=1): X = G + E rounded to
    the dtype (err_in; else X = G), vals = X[idx] at the restated indices, E := X with them zeroed,
    G untouched."""
    L = N.lib()
    g = torch.Generator().manual_seed(22)
    numels = [5, 4096, 65_537, 1_000_003] + [700 + 13 * i for i in range(50)]
    ks = [2, 819, 13_107, 200_000] + [max(1, (700 + 13 * i) // 5) for i in range(50)]
    offs = [sum(numels[:i]) for i in range(len(numels))]
    kof = [sum(ks[:i]) for i in range(len(ks))]
    G = torch.randn(sum(numels), generator=g).to(dtype)
    E0 = torch.randn(sum(numels), generator=g).to(dtype)
    Gd, Ed = G.to(DEV), E0.to(DEV)
    idx = torch.empty(sum(ks), dtype=torch.int32, device=DEV)
    vals = torch.empty(sum(ks), dtype=dtype, device=DEV)
    ws = torch.empty(int(L.arctopk_sparse_workspace_bytes(len(numels), N.i64_array(numels))),
                     dtype=torch.uint8, device=DEV)
    seed = 987_654_321
    N.check(L.arctopk_randk_select_ef14(Gd.data_ptr(), Ed.data_ptr(), err_in, len(numels), N.i64_array(offs),
                                        N.i64_array(numels), N.i64_array(ks), N.i64_array(kof), seed,
                                        idx.data_ptr(), vals.data_ptr(), ws.data_ptr(), N.DTYPE_CODE[dtype],
                                        torch.cuda.current_stream().cuda_stream), "randk_select_ef14")
    torch.cuda.synchronize()
    X = (G.float() + E0.float()).to(dtype) if err_in else G.clone()  # torch's own bf16 add rounding
    expect_E = X.clone()
    i, v = idx.cpu().long(), vals.cpu()
    for t, (n, k, o, ko) in enumerate(zip(numels, ks, offs, kof)):
        ref = S.randk_hash_indices(n, k, seed, t).long()
        assert torch.equal(i[ko:ko + k], ref), f"tensor {t} indices"
        assert_bitwise(v[ko:ko + k], X[o + ref], f"tensor {t} values")
        expect_E[o + ref] = 0
    assert_bitwise(Ed, expect_E, "E after the select")
    assert_bitwise(Gd, G, "G untouched")


@pytest.mark.parametrize("ef", ["noef", "ef14", "ef21"])
@pytest.mark.parametrize("source", ["torch", "host", "hash"])
def test_randk_hook_vs_oracle(ef, source):
    st = sparse_hook.SparseState(None, compress_ratio=0.2, start_compress_iter=0,
                                 sparse_type="tensor", random=True, use_error_feedback=ef,
                                 random_seed=9, index_source=source)
    rng = torch.Generator().manual_seed(9)
    E = gE = None
    numels = [int(torch.Size(s).numel()) for s in SHAPES]
    ks = [max(1, int(n * 0.2)) for n in numels]
    for it in range(3):
        G = _rand(SHAPES, 70 + it)
        out = sparse_hook.sparse_hook_sync(st, SyntheticBucket(G.to(DEV), SHAPES)).wait()
        torch.cuda.synchronize()
        if ef == "ef21" and E is None:
            E, gE = G.clone(), G.clone()
            continue
        seed = int(torch.randint(0, 1_000_000_000, (1,), generator=rng).item())
        if source == "torch":  # the device draw the hook made (deterministic per seed)
            torch.manual_seed(seed)
            idx = [torch.randperm(n, device=DEV)[:k].cpu() for n, k in zip(numels, ks)]
        elif source == "host":  # the reference's CPU draw
            torch.manual_seed(seed)
            idx = [torch.randperm(n)[:k] for n, k in zip(numels, ks)]
        else:
            idx = device_randk_hash(numels, ks, seed, DEV)
            for t, (n, k) in enumerate(zip(numels, ks)):  # the device draw is the restated rule
                assert torch.equal(idx[t], S.randk_hash_indices(n, k, seed, t)), f"tensor {t} draw"
        res = S.simulate_step([G], [E if not (ef == "ef14" and E is None) else None], gE, SHAPES,
                              0.2, ef, True, None, indices_override=[idx])
        assert_bitwise(out, res["out"], f"it{it} out")
        if ef != "noef":
            assert_bitwise(st.error_dict[0], res["E_new"][0], f"it{it} E")
            E = res["E_new"][0]
        if ef == "ef21":
            gE = res["gE_new"]


@pytest.mark.parametrize("name", [n for n in case_names("topk_") if n.endswith("ws1")])
def test_topk_golden_on_gpu(name):
    g = Golden(name)
    m = g.meta
    mod = sparse_hook_c4 if m["hook"] == "sparse_c4" else sparse_hook
    st = mod.SparseState(None, compress_ratio=m["ratio"], start_compress_iter=m["start"],
                         sparse_type="tensor", random=False, use_error_feedback=m["ef"],
                         random_seed=m["seed"])
    st.error_decay = m.get("error_decay", 1.0)  # EF21 residual scaling (set by hand, as a driver would)
    if m.get("large_batch"):  # EF21 large-batch initialisation (set by hand; from iteration iter0)
        st.large_batch_init, st.iter = True, m["iter0"]
    shapes = [tuple(s) for s in m["shapes"]]
    for it in range(m["iters"]):
        out = mod.sparse_hook_sync(st, SyntheticBucket(g.t(0, it, "G").to(DEV), shapes)).wait()
        torch.cuda.synchronize()
        assert_bitwise(out, g.t(0, it, "out"), f"{name} it{it} out")
        if g.has(0, it, "E"):
            assert_bitwise(st.error_dict[0], g.t(0, it, "E"), f"{name} it{it} E")
        if g.has(0, it, "gE"):
            assert_bitwise(st.global_error_dict[0], g.t(0, it, "gE"), f"{name} it{it} gE")
        assert st.comm_bits_this_round == int(g.np(0, it, "bits"))
        assert st.iter == int(g.np(0, it, "iter_after"))


@pytest.mark.parametrize("name", [n for n in case_names("randk_") if n.endswith("ws1")])
def test_randk_golden_on_gpu(name):
    """The reference's RandK fixtures (its CPU torch.randperm draws after the global reseed,
    sparse_hook_c4.py:20, :269-274) through the HIP hook with index_source="host": outputs,
    residuals and bits bit for bit."""
    g = Golden(name)
    m = g.meta
    assert m["random"]
    mod = sparse_hook_c4 if m["hook"] == "sparse_c4" else sparse_hook
    st = mod.SparseState(None, compress_ratio=m["ratio"], start_compress_iter=m["start"],
                         sparse_type="tensor", random=True, use_error_feedback=m["ef"],
                         random_seed=m["seed"])
    st.index_source = "host"
    st.error_decay = m.get("error_decay", 1.0)
    shapes = [tuple(s) for s in m["shapes"]]
    for it in range(m["iters"]):
        out = mod.sparse_hook_sync(st, SyntheticBucket(g.t(0, it, "G").to(DEV), shapes)).wait()
        torch.cuda.synchronize()
        assert_bitwise(out, g.t(0, it, "out"), f"{name} it{it} out")
        if g.has(0, it, "E"):
            assert_bitwise(st.error_dict[0], g.t(0, it, "E"), f"{name} it{it} E")
        if g.has(0, it, "gE"):
            assert_bitwise(st.global_error_dict[0], g.t(0, it, "gE"), f"{name} it{it} gE")
        assert st.comm_bits_this_round == int(g.np(0, it, "bits"))


def test_topk_headline_bucket_properties():
    """16 x [2048, 2048]: |selected| >= |dropped| per tensor, k exact, EF14 conservation."""
    shapes = [[2048, 2048]] * 16
    n = bucket_numel(shapes)
    torch.manual_seed(1)
    G = torch.randn(n, device=DEV)
    E0 = torch.randn(n, device=DEV) * 0.1
    st = sparse_hook.SparseState(None, compress_ratio=0.2, start_compress_iter=0,
                                 sparse_type="tensor", random=False, use_error_feedback="ef14")
    st.error_dict[0] = E0.clone()
    X = G + E0
    out = sparse_hook.sparse_hook_sync(st, SyntheticBucket(G.clone(), shapes)).wait()
    torch.cuda.synchronize()
    assert torch.equal(out + st.error_dict[0], X)
    nz = (out != 0).view(16, -1)
    assert torch.all(nz.sum(1) <= 838_860)
    ax = X.abs().view(16, -1)
    for t in range(16):
        sel = (out.view(16, -1)[t] != 0) | ((X.view(16, -1)[t] == 0) & (st.error_dict[0].view(16, -1)[t] == 0))
        assert ax[t][sel].min() >= ax[t][~sel].max()


def _split(flat: torch.Tensor, ks):
    out, o = [], 0
    for k in ks:
        out.append(flat[o:o + k].long())
        o += k
    return out


@pytest.mark.parametrize("ef,which", [("noef", "small"), ("ef14", "small"), ("ef21", "small"),
                                      ("ef14", "large")])
def test_topk_hook_bf16_vs_oracle(ef, which):
    """bf16 buckets (the Llama driver's default dtype; reference sparse_hook.py:16-34 works in
    the bucket dtype): the selected indices satisfy the oracle's |x| (bf16 magnitudes tie
    often and torch.topk's tie order is implementation-defined, so ties are checked by the
    exact tie rule), and given them the output, E and gE are bit-exact with every add and
    divide rounded to bf16."""
    shapes = SHAPE_SETS[which]
    st = sparse_hook.SparseState(None, compress_ratio=0.2, start_compress_iter=0,
                                 sparse_type="tensor", random=False, use_error_feedback=ef)
    E = gE = None
    ties = 0
    for it in range(3):
        G = _rand(shapes, 150 + it).to(torch.bfloat16)
        out = sparse_hook.sparse_hook_sync(st, SyntheticBucket(G.to(DEV), shapes)).wait()
        torch.cuda.synchronize()
        if ef == "ef21" and E is None:
            E, gE = G.clone(), G.clone()
            continue
        Ein = E if not (ef == "ef14" and E is None) else None
        X = S.encode(G, Ein, ef)
        rows = _split(st.last_indices.cpu(), st.last_k)
        off = 0
        for s, r, k in zip(shapes, rows, st.last_k):
            n = S.numel_of(s)
            ties += check_rows_tie_aware(r, X[off:off + n].float().abs(), k, band=0.0)
            off += n
        res = S.simulate_step([G], [Ein], gE, shapes, 0.2, ef, False, None, indices_override=[rows])
        assert_bitwise(out, res["out"], f"it{it} out")
        if ef != "noef":
            assert_bitwise(st.error_dict[0], res["E_new"][0], f"it{it} E")
            E = res["E_new"][0]
        if ef == "ef21":
            assert_bitwise(st.global_error_dict[0], res["gE_new"], f"it{it} gE")
            gE = res["gE_new"]
        assert st.comm_bits_this_round >= 0


@pytest.mark.parametrize("ef", ["noef", "ef14", "ef21"])
def test_randk_hook_bf16_vs_oracle(ef):
    """RandK on a bf16 bucket (device index source): values, the bf16 division by the world
    size, the scatter and the residuals bit-exact against the oracle in bf16."""
    st = sparse_hook.SparseState(None, compress_ratio=0.2, start_compress_iter=0,
                                 sparse_type="tensor", random=True, use_error_feedback=ef,
                                 random_seed=9, index_source="hash")
    E = gE = None
    for it in range(3):
        G = _rand(SHAPES, 170 + it).to(torch.bfloat16)
        out = sparse_hook.sparse_hook_sync(st, SyntheticBucket(G.to(DEV), SHAPES)).wait()
        torch.cuda.synchronize()
        if ef == "ef21" and E is None:
            E, gE = G.clone(), G.clone()
            continue
        rows = _split(st.last_indices.cpu(), st.last_k)
        res = S.simulate_step([G], [E if not (ef == "ef14" and E is None) else None], gE, SHAPES,
                              0.2, ef, True, None, indices_override=[rows])
        assert_bitwise(out, res["out"], f"it{it} out")
        if ef != "noef":
            assert_bitwise(st.error_dict[0], res["E_new"][0], f"it{it} E")
            E = res["E_new"][0]
        if ef == "ef21":
            assert_bitwise(st.global_error_dict[0], res["gE_new"], f"it{it} gE")
            gE = res["gE_new"]


@pytest.mark.parametrize("c4", [False, True])
def test_large_batch_ef21_failures_match_reference(c4):
    """The reference's large-batch EF21 hook raises TypeError at iteration 0 (its
    default_hooks._allreduce_fut call lacks the required hook_state), and its registered copy
    raises AttributeError at the first compressed call (cal_k(state, tensor) called as
    cal_k(tensor, ratio)): the same exceptions at the same points (tests/golden/
    large_batch_errors.json)."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "large_batch_errors.json")) as f:
        cases = json.load(f)["cases"]
    mod = sparse_hook_c4 if c4 else sparse_hook
    shapes = [(10,), (40, 16), (4, 3, 3, 3), (96, 40)]
    st = mod.SparseState(None, compress_ratio=0.2, start_compress_iter=3, sparse_type="tensor",
                         use_error_feedback="ef21")
    st.large_batch_init = True
    mk = lambda: SyntheticBucket(_rand(shapes, 3).to(DEV), shapes)  # noqa: E731
    ref = cases["sparse_c4_iter0" if c4 else "sparse_iter0"]
    with pytest.raises(TypeError) as ei:
        mod.sparse_hook_sync(st, mk())
    assert str(ei.value) == ref["message"] and st.iter == ref["iter_after"]
    mod.sparse_hook_sync(st, mk()).wait()  # iterations 1, 2: accumulate
    mod.sparse_hook_sync(st, mk()).wait()
    if c4:
        ref = cases["sparse_c4_compressed"]
        with pytest.raises(AttributeError) as ei:
            mod.sparse_hook_sync(st, mk())
        assert str(ei.value) == ref["message"] and st.iter == ref["iter_after"]
    else:
        mod.sparse_hook_sync(st, mk()).wait()
        assert st.iter == 4
    torch.cuda.synchronize()
