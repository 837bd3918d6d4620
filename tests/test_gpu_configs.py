"""HIP hooks vs the CPU oracle at the BASELINE configs' own bucket sizes (MI355X, -m gpu).

BASELINE.json's configs and north_star, and the bucket each one hooks:

  north_star     the 256 MiB headline bucket, 16 x [2048, 2048] fp32, EF14 and EF21
  configs[1]     ResNet-18 CIFAR (cifar10/run_cifar10.py:153, cifar10/resnet.py:103-104) as
                 its three DDP buckets, EF14, several backwards on one hook state
  configs[2]     RoBERTa-base: the [50265, 768] word-embedding bucket, EF14
  configs[3]     ResNet-50 stage-4 1x1 / 3x3 conv mix through ARC-TopK, TopK and RandK
                 (cifar10/run_cifar100_resnet50.py:155)
  configs[4]     Llama-1B: the [32000, 2048] embedding bucket with ~90 % all-zero rows (only
                 the batch's tokens have gradient), EF21 -- the k-th energy is 0, so ~400
                 zero rows tie at the threshold (reference topk at
                 comm_hooks/group_topk_hook_no_reshape.py:63)

Bar (north_star: indices bit-exact, decompressed gradients within 1e-6):

* select, exactly: the device select kernels fed the oracle's all-reduced sketch must pick
  exactly the oracle's rows under the tie rule (strictly-above rows plus the lowest-index
  ties), for every bucket of every config -- zero tolerance;
* end to end: the device's own sketch is summed in another fp32 order than CPU sgemm, so
  a row within rounding of the k-th energy could flip; the rows must satisfy the oracle's
  energies within a 2e-4 relative band, and the number of rows that differ from the
  oracle's exact selection is counted, printed and must be 0 for the committed seeds;
* given those rows every output, residual and global residual is compared BIT FOR BIT with
  the oracle (stricter than 1e-6).

TopK / RandK select exactly (no sketch), so their outputs are bit-exact end to end.
"""
import pytest
import torch

from allreducetopk_amd import _native as N
from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel
from allreducetopk_amd.comm_hooks import sparse_hook
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import GroupTopKState, group_topk_hook
from workloads import WORKLOADS, ddp_buckets, resnet18_cifar_shapes, resnet50_cifar_shapes
from oracle import arctopk as A
from oracle import sparse as S
from parity import assert_bitwise, check_rows_tie_aware, device_randk_hash, ensure_group

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
MAX_FLIPS = 0  # end-to-end rows differing from the oracle's exact selection (committed seeds)


@pytest.fixture(scope="module", autouse=True)
def group():
    ensure_group("nccl")
    yield


def _rows(plan):
    rl = plan.rowlist.cpu()
    return [rl[s.sel_off:s.sel_off + s.k_rows].long() for s in plan.segments]


class ArcRun:
    """Drives one GroupTopKState over a sequence of calls per bucket and replays every
    compressed call through the oracle (single rank)."""

    def __init__(self, ef, seed=1234, force_exchange=False, select_streams=None):
        self.ef = ef
        self.st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0,
                                 use_error_feedback=ef, seed=seed)
        self.st.force_exchange = force_exchange
        if select_streams is not None:  # default: the state's ("auto": select streams for <= 64 MiB)
            self.st.select_streams = select_streams
        self.st.defer_decode = True  # every bucket's Future is waited after the last one, as DDP does
        self.ost = A.OracleState(r=4, compress_ratio=0.2, start_compress_iter=0,
                                 use_error_feedback=ef, seed=seed)
        self.E, self.gE = {}, {}
        self.flips = 0
        self.checked = 0

    def step(self, grads):
        """grads: {bucket index: (shapes, G cpu)}, hooked in dict order; the futures are
        waited at the end as DDP's finalize does."""
        futs = {}
        items = list(grads.items())
        for j, (b, (shapes, G)) in enumerate(items):
            futs[b] = group_topk_hook(self.st, SyntheticBucket(G.to(DEV), shapes, index=b,
                                                               is_last=(j == len(items) - 1)))
        outs = {b: f.wait() for b, f in futs.items()}
        torch.cuda.synchronize()
        for b, (shapes, G) in items:
            out = outs[b]
            if self.ef == "ef21" and b not in self.E:  # dense init call
                assert_bitwise(out, G, f"bucket {b} EF21 init")
                self.E[b], self.gE[b] = G.clone(), G.clone()
                continue
            seed = self.ost.next_seed()
            plan = self.st._plans[b][1]
            rows = _rows(plan)
            E_prev = self.E.get(b) if self.ef != "noef" else None
            res = A.simulate_step([G], [E_prev], self.gE.get(b), shapes, 0.2, 4, self.ef, seed,
                                  rows_override=rows, proj_device=DEV)
            for r_, nrm, s in zip(rows, res["norms"], plan.segments):
                self.flips += check_rows_tie_aware(r_, nrm, int(s.k_rows), band=2e-4)
                assert torch.all(r_[1:] > r_[:-1]), "row list must be ascending"
            assert_bitwise(out, res["out"], f"bucket {b} output")
            # the select kernels fed the oracle's all-reduced sketch: exactly the oracle's rows
            ref_sketch = torch.cat([p_.flatten() for p_ in res["P_sum"]])
            plan.sketch[:ref_sketch.numel()].copy_(ref_sketch.to(DEV))
            plan.select(1, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            for j, (r_, nrm, s) in enumerate(zip(_rows(plan), res["norms"], plan.segments)):
                assert check_rows_tie_aware(r_, nrm, int(s.k_rows), band=0.0) == 0, \
                    f"bucket {b} segment {j}: select on the oracle's sketch differs from the oracle"
            if self.ef != "noef":
                assert_bitwise(self.st.error_dict[b], res["E_new"][0], f"bucket {b} E")
                self.E[b] = res["E_new"][0]
            if self.ef == "ef21":
                assert_bitwise(self.st.global_error_dict[b], res["gE_new"], f"bucket {b} gE")
                self.gE[b] = res["gE_new"]
            self.checked += 1
        print(f"end-to-end row flips vs the oracle so far: {self.flips} ({self.checked} calls)")
        assert self.flips <= MAX_FLIPS, f"{self.flips} rows differ from the oracle's selection"


def _randn(n, seed, scale=1.0):
    return torch.randn(n, generator=torch.Generator().manual_seed(seed)) * scale


@pytest.mark.parametrize("ef,force_exchange", [("ef14", False), ("ef21", False), ("ef14", True)])
def test_headline_256mib_vs_oracle(ef, force_exchange):
    """north_star's bucket: 16 x [2048, 2048] fp32 = 256 MiB, ratio 0.2, r 4 (also through the
    N > 1 code path: the exchange step over a one-rank RCCL communicator)."""
    shapes = [[2048, 2048]] * 16
    n = bucket_numel(shapes)
    run = ArcRun(ef, force_exchange=force_exchange)
    for it in range(3):
        run.step({0: (shapes, _randn(n, 500 + it))})
    assert run.checked == (3 if ef == "ef14" else 2)
    assert run.st._plans[0][1].info.values_len == 13_402_112


def test_llama_embedding_zero_row_ties_ef21():
    """configs[4]: [32000, 2048] embedding, 3,000 token rows with gradient per call, the
    rest exactly zero; EF21 steady state selects k = 6,400 rows, so every row with
    nonzero D = G - E is selected and the remainder are zero-energy ties (whichever the
    device takes, outputs and residuals are bit-identical to the oracle's)."""
    shapes = [[32000, 2048]]
    n = bucket_numel(shapes)
    run = ArcRun("ef21", seed=77)
    g = torch.Generator().manual_seed(4)
    zero_ties = []
    for it in range(3):
        G = torch.zeros(32000, 2048)
        tok = torch.randperm(32000, generator=g)[:3000]
        G[tok] = torch.randn(3000, 2048, generator=g) * 1e-2
        run.step({0: (shapes, G.view(-1))})
        if it:
            plan = run.st._plans[0][1]
            en = torch.empty(plan.info.rows_total, device=DEV)
            plan.row_energy(1, en, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            e = en.cpu()
            zero_ties.append(int((e[_rows(plan)[0]] == 0).sum()))
    assert n == 32000 * 2048
    assert all(z > 0 for z in zero_ties), f"no zero-energy ties exercised: {zero_ties}"


def test_roberta_embedding_ef14():
    """configs[2]: RoBERTa-base word embedding [50265, 768] (147 MiB), EF14."""
    shapes = [[50265, 768]]
    n = bucket_numel(shapes)
    run = ArcRun("ef14", seed=5)
    for it in range(3):
        run.step({0: (shapes, _randn(n, 700 + it))})
    assert run.checked == 3


@pytest.mark.parametrize("ef", ["ef14", "noef", "ef21"])
def test_zero_ahead_drain_large_buckets(ef):
    """The zero-ahead drain (the exchange path's backward-last step on a bucket of >= 64 MiB zeroes the
    bucket while its packed values are on the wire; the decode after the wire writes only the
    selected rows; EF21 keeps the whole decode) gives the bits of the world-size-1 step path: two
    64 MiB buckets over two backwards, forced exchange (one-rank RCCL) against the step path."""
    shapes = [[4096, 4096]]
    n = bucket_numel(shapes)
    assert n * 4 >= 64 << 20
    outs = {}
    for force in (False, True):
        st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback=ef, seed=21)
        st.force_exchange = force
        st.defer_decode = True
        res = []
        for it in range(3 if ef == "ef21" else 2):  # (EF21: a dense init backward first)
            futs = [group_topk_hook(st, SyntheticBucket(_randn(n, 50 + 10 * it + b).to(DEV), shapes, index=b,
                                                        is_last=(b == 1))) for b in range(2)]
            res.append([f.wait().cpu() for f in futs])
        torch.cuda.synchronize()
        outs[force] = (res, {b: e.cpu() for b, e in st.error_dict.items()},
                       {b: e.cpu() for b, e in st.global_error_dict.items()})
    step, fx = outs[False], outs[True]
    for it, (a, c) in enumerate(zip(step[0], fx[0])):
        for b in range(2):
            assert_bitwise(c[b], a[b], f"backward {it} bucket {b} output")
    for b in step[1]:
        assert_bitwise(fx[1][b], step[1][b], f"bucket {b} E")
    for b in step[2]:
        assert_bitwise(fx[2][b], step[2][b], f"bucket {b} gE")


@pytest.mark.parametrize("force_exchange,select_streams,trail", [(False, "auto", True), (True, "auto", True),
                                                                 (False, "off", True), (True, "off", True),
                                                                 (False, "auto", False), (False, "on", True)])
def test_resnet18_ddp_buckets_ef14(force_exchange, select_streams, trail):
    """configs[1]: the CIFAR ResNet-18's three DDP buckets (reverse parameter order,
    1 MiB first bucket, 25 MiB cap), hooked in bucket order over three backwards on one
    state: per-bucket plans, residuals and projections stay separate.  With the exchange
    step (one-rank RCCL) two buckets per backward are overlapped and deferred.  "auto": each
    bucket's select, pack and decodes on one of the two select streams.
    trail: the 20 KB first bucket is a trailing step, its encode and selects carried by the
    second bucket's launches (world size 1; the exchange path enqueues it on its own)."""
    layouts = ddp_buckets(resnet18_cifar_shapes())
    assert len(layouts) == 3 and sum(bucket_numel(sh) for sh in layouts) == 11_173_962
    run = ArcRun("ef14", seed=11, force_exchange=force_exchange, select_streams=select_streams)
    if not trail:
        run.st.trail_bytes = 0
    for it in range(3):
        run.step({b: (sh, _randn(bucket_numel(sh), 900 + 10 * it + b)) for b, sh in enumerate(layouts)})
    assert run.checked == 9
    assert (run.st.trail_calls > 0) == (trail and not force_exchange and select_streams != "on"), run.st.trail_calls


@pytest.mark.parametrize("force_exchange,select_streams,ef", [(False, "auto", "ef14"), (True, "auto", "ef14"),
                                                              (False, "off", "ef14"), (False, "auto", "ef21"),
                                                              (True, "auto", "noef")])
def test_resnet50_ddp_buckets_ef14(force_exchange, select_streams, ef):
    """configs[3]'s model as DDP hooks it: the CIFAR-100 ResNet-50's five DDP buckets (161
    tensors: 1x1 convs of m = 2, 3x3 convs of m = 18, BatchNorm vectors, the [100, 2048]
    classifier), hooked in bucket order over two backwards on one state (EF21 / noef also
    through the select streams: EF21's pack then runs on the select stream, not in the next
    encode)."""
    layouts = ddp_buckets(resnet50_cifar_shapes())
    assert len(layouts) == 5 and sum(bucket_numel(sh) for sh in layouts) == 23_705_252
    run = ArcRun(ef, seed=13, force_exchange=force_exchange, select_streams=select_streams)
    if ef == "ef21":  # the dense init backward, then two compressed ones
        run.step({b: (sh, _randn(bucket_numel(sh), 1600 + b)) for b, sh in enumerate(layouts)})
    for it in range(2):
        run.step({b: (sh, _randn(bucket_numel(sh), 1700 + 10 * it + b)) for b, sh in enumerate(layouts)})
    assert run.checked == 10
    if select_streams == "auto":
        assert run.st._sel_streams, "the select streams were not used"
    if not force_exchange and ef != "ef21" and select_streams == "off":  # the 0.8 MiB first bucket
        assert run.st.trail_calls > 0  # trails into the second (not in a select-stream backward)


def test_resnet50_ddp_buckets_topk_ef14():
    """configs[3]'s TopK baseline (topk_sync, sparse_hook.py:163-304) on the model's five DDP
    buckets, hooked in order on one state over two backwards: indices satisfy the exact tie
    rule against the oracle's |X|, and given them every output and residual is bit-exact."""
    layouts = ddp_buckets(resnet50_cifar_shapes())
    st = sparse_hook.SparseState(None, compress_ratio=0.2, start_compress_iter=0,
                                 sparse_type="tensor", random=False, use_error_feedback="ef14")
    E = {}
    for it in range(2):
        for b, sh in enumerate(layouts):
            G = _randn(bucket_numel(sh), 1800 + 10 * it + b)
            out = sparse_hook.sparse_hook_sync(st, SyntheticBucket(G.to(DEV), sh, index=b,
                                                                   is_last=(b == len(layouts) - 1))).wait()
            torch.cuda.synchronize()
            X = S.encode(G, E.get(b), "ef14")
            idx = _split(st.last_indices.cpu(), st.last_k)
            off = 0
            for t, s_ in zip(idx, sh):
                nel = bucket_numel([s_])
                assert check_rows_tie_aware(t, X[off:off + nel].abs(), t.numel(), band=0.0) == 0
                off += nel
            res = S.simulate_step([G], [E.get(b)], None, sh, 0.2, "ef14", False, None, indices_override=[idx])
            assert_bitwise(out, res["out"], f"it{it} bucket {b} out")
            assert_bitwise(st.error_dict[b], res["E_new"][0], f"it{it} bucket {b} E")
            E[b] = res["E_new"][0]


RESNET50 = WORKLOADS["resnet50_mixed"][1]


def test_llama_layer_mix_ef21():
    """configs[4]'s transformer layer as one bucket: RMSNorm weights (1-D), the MLP
    [5632, 2048] / [2048, 5632] and attention [2048, 2048] projections, EF21 (the Llama
    driver's mode), two buckets per backward."""
    shapes = WORKLOADS["llama_layer_mixed"][1]
    n = bucket_numel(shapes)
    run = ArcRun("ef21", seed=31)
    for it in range(3):
        run.step({b: (shapes, _randn(n, 1500 + 10 * it + b, 1e-2)) for b in range(2)})
    assert run.checked == 4


@pytest.mark.parametrize("ef,nb,force_exchange", [("ef14", 1, False), ("ef21", 1, False),
                                                   ("ef14", 2, False), ("ef21", 2, True)])
def test_resnet50_mix_arc(ef, nb, force_exchange):
    """configs[3] through ARC-TopK: 1x1 convs (m = 2, sketch twice the tensor; 524,288 and
    1,048,576-row segments), 3x3 convs (m = 18) and 1-D BatchNorm tensors in one bucket.  With
    two buckets per backward the first bucket's deferred decode rides in the second bucket's
    last select launch (the write launch; the 1 M-row items take the refine launch before it)."""
    n = bucket_numel(RESNET50)
    run = ArcRun(ef, seed=21, force_exchange=force_exchange)
    for it in range(3):
        run.step({b: (RESNET50, _randn(n, 1100 + 10 * it + b)) for b in range(nb)})


def test_conv3x3_stack_ef14():
    """28 x [512, 512, 3, 3] (m = 18, 131,072 rows each, 896 ranges of the multi-block
    select: more write blocks than stay resident at once, so the refine has a launch of its
    own before the write launch) and the short-row (mode 3) decode."""
    shapes = WORKLOADS["resnet18_conv"][1]
    n = bucket_numel(shapes)
    run = ArcRun("ef14", seed=41)
    for it in range(2):
        run.step({0: (shapes, _randn(n, 1300 + it))})
    assert run.checked == 2


@pytest.mark.parametrize("ef", ["ef14", "ef21"])
def test_resnet50_mix_topk(ef):
    """configs[3] through the TopK baseline (exact element top-k of |x| per tensor)."""
    n = bucket_numel(RESNET50)
    st = sparse_hook.SparseState(None, compress_ratio=0.2, start_compress_iter=0,
                                 sparse_type="tensor", random=False, use_error_feedback=ef)
    E = gE = None
    for it in range(3):
        G = _randn(n, 1200 + it)
        out = sparse_hook.sparse_hook_sync(st, SyntheticBucket(G.to(DEV), RESNET50)).wait()
        torch.cuda.synchronize()
        if ef == "ef21" and E is None:
            E, gE = G.clone(), G.clone()
            continue
        # exact |x| ties at the k-th value occur in ~1 M-element tensors (torch.topk's tie
        # order is implementation-defined; the device takes the lowest indices): the
        # device's indices must satisfy the exact tie rule against the oracle's |X|, and
        # given them every output is bit-exact
        X = S.encode(G, E, ef)
        idx = _split(st.last_indices.cpu(), st.last_k)
        off = 0
        for t, s_ in zip(idx, RESNET50):
            nel = bucket_numel([s_])
            assert check_rows_tie_aware(t, X[off:off + nel].abs(), t.numel(), band=0.0) == 0
            off += nel
        res = S.simulate_step([G], [E], gE, RESNET50, 0.2, ef, False, None, indices_override=[idx])
        assert_bitwise(out, res["out"], f"it{it} out")
        assert_bitwise(st.error_dict[0], res["E_new"][0], f"it{it} E")
        E = res["E_new"][0]
        if ef == "ef21":
            assert_bitwise(st.global_error_dict[0], res["gE_new"], f"it{it} gE")
            gE = res["gE_new"]


def _split(flat, ks):
    out, o = [], 0
    for k in ks:
        out.append(flat[o:o + k])
        o += k
    return out


def test_resnet50_mix_randk():
    """configs[3] through the RandK baseline, device index source (keyed permutation);
    the indices are regenerated from the same seed and fed to the oracle."""
    n = bucket_numel(RESNET50)
    st = sparse_hook.SparseState(None, compress_ratio=0.2, start_compress_iter=0,
                                 sparse_type="tensor", random=True, use_error_feedback="ef14",
                                 random_seed=9, index_source="hash")
    rng = torch.Generator().manual_seed(9)
    numels = [bucket_numel([s]) for s in RESNET50]
    ks = [max(1, int(x * 0.2)) for x in numels]
    E = None
    for it in range(3):
        G = _randn(n, 1300 + it)
        out = sparse_hook.sparse_hook_sync(st, SyntheticBucket(G.to(DEV), RESNET50)).wait()
        torch.cuda.synchronize()
        seed = int(torch.randint(0, 1_000_000_000, (1,), generator=rng).item())
        idx = device_randk_hash(numels, ks, seed, DEV)
        res = S.simulate_step([G], [E], None, RESNET50, 0.2, "ef14", True, None,
                              indices_override=[idx])
        assert_bitwise(out, res["out"], f"it{it} out")
        assert_bitwise(st.error_dict[0], res["E_new"][0], f"it{it} E")
        E = res["E_new"][0]
