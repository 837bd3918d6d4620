"""Host-side logic of the drop-in hooks (CPU): state, registry, flags, k, projections."""
import argparse

import pytest
import torch

from allreducetopk_amd.bucket import SyntheticBucket
from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as G
from allreducetopk_amd.comm_hooks import sparse_hook, sparse_hook_c4
from allreducetopk_amd.comm_hooks.projections import ProjectionSource, draw_host
from allreducetopk_amd.comm_hooks.utils import (HookState, add_comm_hook_args, dtype_bits,
                                                register_comm_hook_for_ddp_model, tensor_bits)
from golden_io import Golden, case_names
from oracle import arctopk as A
from oracle import sparse as S

SHAPES = [(10,), (40, 16), (4, 3, 3, 3), (16, 8, 3, 3), (16, 8, 1, 1), (96, 40), (7,),
          (2048, 2048), (32000, 2048), (512, 512, 3, 3), (5461, 2048)]


@pytest.mark.parametrize("ratio", [0.2, 0.08, 0.01, 1.0])
def test_cal_k_matches_reference_formula(ratio):
    st = G.GroupTopKState(None, compress_ratio=ratio)
    for s in SHAPES:
        t = torch.empty(s)
        assert G.cal_k(st, t) == A.cal_k(s, ratio)
        assert sparse_hook.cal_k(t, ratio) == S.cal_k(t.numel(), ratio)


def test_state_defaults_match_reference():
    st = G.GroupTopKState(None)
    assert (st.r, st.compress_ratio, st.start_compress_iter, st.use_error_feedback, st.seed,
            st.error_decay) == (4, 0.08, 2, "noef", 0, 1.0)
    sp = sparse_hook.SparseState(None)
    assert (sp.compress_ratio, sp.start_compress_iter, sp.sparse_type, sp.random,
            sp.use_error_feedback, sp.random_seed, sp.large_batch_init) == \
        (0.01, 2, "row", False, "noef", 0, False)
    c4 = sparse_hook_c4.SparseState(None, compress_ratio=0.2, start_compress_iter=3)
    assert c4.gradual_compression and c4.warmup_iters == 103 and not c4.compression_started


def test_gradual_ratio_matches_reference_formula():
    st = sparse_hook_c4.SparseState(None, compress_ratio=0.1, start_compress_iter=5)
    assert st.get_current_compress_ratio() == 0.1  # not started yet
    st.compression_started = True
    for it in range(5, 300, 7):
        st.iter = it
        assert st.get_current_compress_ratio() == S.gradual_ratio(0.1, it, 5)


def test_seed_sequence_matches_reference_golden():
    """The projection seeds drawn per call equal the reference's state.rng draws."""
    for name in case_names("arc_mix_ef14_ws1"):
        g = Golden(name)
        ps = ProjectionSource(4, depth=3, workers=1)
        rng = torch.Generator().manual_seed(g.meta["seed"])
        for it in range(g.meta["iters"]):
            assert ps.consume_seed(rng) == int(g.np(0, it, "seed")[0])


def test_seed_lookahead_predicts_and_resynchronises():
    """peek_next_seed (batched look-ahead draws) always names the seed the next
    consume_seed returns -- across look-ahead refills and after the rng is repositioned
    (the pre-drawn projections of arctopk_select_draw are keyed on it)."""
    ps = ProjectionSource(4, depth=3, workers=1)
    rng = torch.Generator().manual_seed(7)
    ref = torch.Generator().manual_seed(7)
    hits = 0
    for call in range(70):
        if call in (23, 50):  # repositioned between calls, both generators alike
            rng.manual_seed(1000 + call)
            ref.manual_seed(1000 + call)
        peek = ps.peek_next_seed()
        seed = ps.consume_seed(rng)
        assert seed == int(torch.randint(0, 1_000_000_000, (1,), generator=ref).item())
        hits += peek == seed
    assert hits >= 70 - 3  # first call and the two repositions
    ps.close()


@pytest.mark.parametrize("seed", [0, 1, 440527571, 999_999_999])
def test_projection_draw_matches_reference_stream(seed):
    shapes = [(10,), (40, 16), (4, 3, 3, 3), (16, 8, 1, 1), (96, 40), (2048, 2048), (5461, 33),
              (4, 2, 5, 5)]
    segs = A.segments(shapes, 0.2)
    ref = torch.cat([v.flatten() for v in A.draw_projections(seed, segs, 4) if v is not None])
    ms = [s.m for s in segs if s.kind == A.SKETCH]
    got = draw_host(seed, ms, 4, torch.float32, pin=False)
    assert torch.equal(got[:ref.numel()], ref)


def test_projection_prefetch_is_transparent():
    ps = ProjectionSource(4, depth=4, workers=2)
    rng = torch.Generator().manual_seed(5)
    ms = (2048, 40, 18)
    vals = []
    for _ in range(6):
        seed = ps.consume_seed(rng)
        slot = ps.get(seed, ms, torch.float32)
        vals.append((seed, slot.host.clone()))
        ps.release(slot)
        ps.prefetch([ms] * 4, torch.float32)
    ps.close()
    assert ps.hits >= 4
    for seed, v in vals:
        assert torch.equal(v, draw_host(seed, ms, 4, torch.float32, pin=False))


def test_bits_helpers():
    assert dtype_bits(torch.zeros(1)) == 32 and dtype_bits(torch.zeros(1, dtype=torch.bfloat16)) == 16
    assert dtype_bits(torch.zeros(1, dtype=torch.int32)) == 32
    assert dtype_bits(torch.zeros(1, dtype=torch.bool)) == 1
    assert dtype_bits(torch.zeros(1, dtype=torch.complex64)) == 64
    assert tensor_bits(torch.zeros(3, 5)) == 15 * 32


def test_hookstate_iter_and_momentum():
    st = HookState(None)
    st.start_compress_iter = 2
    b_last = SyntheticBucket(torch.ones(4), [(4,)], is_last=True)
    b_mid = SyntheticBucket(torch.ones(4), [(4,)], is_last=False)
    st.maybe_increase_iter(b_mid)
    assert st.iter == 0
    st.maybe_increase_iter(b_last)
    assert st.iter == 1
    p = torch.nn.Parameter(torch.zeros(4))
    b = SyntheticBucket(torch.full((4,), 2.0), [(4,)], parameters=[p])
    st.init_momentum_field({p: {"exp_avg": torch.full((4,), 10.0)}}, 0.9)
    st.iter = 2
    st.maybe_accumulate_momentum_on_bucket(b)
    assert st.adam_freeze_key
    assert torch.allclose(b.buffer(), torch.full((4,), 0.1 * 2.0 + 0.9 * 10.0))


class _FakeModel:
    def __init__(self):
        self.hooks = []
        self.lin = torch.nn.Linear(3, 2)

    def register_comm_hook(self, state, hook):
        self.hooks.append((state, hook))

    def named_parameters(self):
        return self.lin.named_parameters()


def _args(**kw):
    p = argparse.ArgumentParser()
    add_comm_hook_args(p)
    p.add_argument("--seed", type=int, default=0)
    a = p.parse_args([])
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_flags_defaults_match_reference():
    a = _args()
    assert (a.compressor, a.start_compress_iter, a.use_error_feedback, a.sparse_type,
            a.compress_ratio, a.r, a.check_grad) == ("none", 10, "noef", "tensor", 0.08, 4, False)


@pytest.mark.parametrize("comp,cls,hook", [
    ("group_topk_no_reshape", G.GroupTopKState, G.group_topk_hook),
    ("topk_sync", sparse_hook_c4.SparseState, sparse_hook_c4.sparse_hook_sync),
    ("randk_sync", sparse_hook_c4.SparseState, sparse_hook_c4.sparse_hook_sync),
])
def test_registry(comp, cls, hook):
    m = _FakeModel()
    st = register_comm_hook_for_ddp_model(m, None, _args(compressor=comp, compress_ratio=0.2,
                                                         use_error_feedback="ef14", seed=3))
    assert isinstance(st, cls) and m.hooks == [(st, hook)]
    assert st.compress_ratio == 0.2 and st.use_error_feedback == "ef14"
    assert set(st.param_to_name.values()) == {"weight", "bias"}
    if comp != "group_topk_no_reshape":
        assert st.random == (comp == "randk_sync") and st.random_seed == 3


def test_registry_none_noop_and_unknown():
    m = _FakeModel()
    st = register_comm_hook_for_ddp_model(m, None, _args(compressor="none", start_compress_iter=4))
    assert isinstance(st, HookState) and st.start_compress_iter == 4
    m2 = _FakeModel()
    assert register_comm_hook_for_ddp_model(m2, None, _args(compressor="noop")) is None
    assert len(m2.hooks) == 1
    with pytest.raises(ValueError):
        register_comm_hook_for_ddp_model(_FakeModel(), None, _args(compressor="bogus"))


def test_compressed_path_refuses_cpu_buckets():
    """No silent CPU fallback: the codec needs the HIP library and a GPU bucket."""
    import torch.distributed as dist
    from parity import ensure_group
    owned = not dist.is_initialized()
    ensure_group("gloo")
    st = G.GroupTopKState(None, compress_ratio=0.2, start_compress_iter=0, use_error_feedback="noef")
    with pytest.raises((RuntimeError, ImportError)):
        G.group_topk_hook(st, SyntheticBucket(torch.randn(640), [(40, 16)]))
    sp = sparse_hook.SparseState(None, compress_ratio=0.2, start_compress_iter=0,
                                 sparse_type="tensor")
    with pytest.raises(RuntimeError):
        sparse_hook.sparse_hook_sync(sp, SyntheticBucket(torch.randn(640), [(40, 16)]))
    if owned:  # do not leak a CPU group into GPU tests collected in the same process
        dist.destroy_process_group()


@pytest.mark.parametrize("which", ["arc", "sparse"])
def test_state_dict_roundtrip_weights_only(tmp_path, which):
    """EF state checkpoint: scalars, rng position and residuals survive torch.save /
    torch.load(weights_only=True); the restored rng continues the same seed sequence."""
    from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import GroupTopKState
    from allreducetopk_amd.comm_hooks.sparse_hook import SparseState
    mk = (lambda: GroupTopKState(None, r=4, compress_ratio=0.2, use_error_feedback="ef21", seed=9)) \
        if which == "arc" else \
        (lambda: SparseState(None, compress_ratio=0.2, use_error_feedback="ef21", random_seed=9))
    st = mk()
    st.iter = 17
    st.comm_bits_this_round = 12345
    st.error_dict = {0: torch.randn(100), 3: torch.randn(7)}
    st.global_error_dict = {0: torch.randn(100)}
    torch.randint(0, 10, (5,), generator=st.rng)  # move the rng
    path = tmp_path / "hook.pt"
    torch.save(st.state_dict(), path)
    st2 = mk()
    st2.load_state_dict(torch.load(path, weights_only=True))
    assert st2.iter == 17 and st2.comm_bits_this_round == 12345
    assert sorted(st2.error_dict) == [0, 3]
    for b in st.error_dict:
        assert torch.equal(st2.error_dict[b], st.error_dict[b])
        assert st2.error_dict[b].data_ptr() != st.error_dict[b].data_ptr()
    assert torch.equal(st2.global_error_dict[0], st.global_error_dict[0])
    a = torch.randint(0, 1_000_000_000, (4,), generator=st.rng)
    b = torch.randint(0, 1_000_000_000, (4,), generator=st2.rng)
    assert torch.equal(a, b)


def test_bf16_projection_tables_match_torch():
    """libarctopk's table-driven bf16 draw equals torch's CPU bf16 normal_ bit for bit: 8M
    draws at four seeds exercise every one of the 65,536 (u[j], u[j+8]) table cells."""
    import numpy as np
    from allreducetopk_amd.comm_hooks.projections import draw_bf16_into
    seen = np.zeros((256, 256), dtype=bool)
    for seed in (0, 1, 123456789, 999_999_999):
        n = 1 << 21
        ref = torch.randn(n, dtype=torch.bfloat16, generator=torch.Generator().manual_seed(seed))
        got = torch.empty(n, dtype=torch.bfloat16)
        draw_bf16_into(seed, got)
        assert torch.equal(got, ref), f"seed {seed}: {(got != ref).sum().item()} values differ"
        st = np.random.RandomState(seed).get_state()  # torch's CPU generator = mt19937(seed)
        bg = np.random.MT19937()
        bg.state = {"bit_generator": "MT19937", "state": {"key": st[1], "pos": st[2]}}
        d = (bg.random_raw(n) & 0xFF).reshape(-1, 2, 8)
        seen[d[:, 0].ravel(), d[:, 1].ravel()] = True
    assert seen.all(), "not every table cell was exercised"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_native_projection_draw_matches_torch(dtype):
    """libarctopk's one-call projection draw (arctopk_draw_normal) equals per-tensor torch
    CPU randn from one generator bit for bit (-0 vs +0 included): tensors of < 16 values
    (scalar Box-Muller with the generator's cached sample carried across tensors), whole
    16-blocks, recomputed tails, and 4 M values of one tensor."""
    import ctypes
    import random
    from allreducetopk_amd.comm_hooks import projections as PJ
    assert PJ.native_ok(dtype)
    iv = torch.int16 if dtype == torch.bfloat16 else torch.int32
    rng = random.Random(5)
    cases = [[1 << 22], [2, 16, 8, 3], [4101, 7, 17, 16, 1]]
    cases += [[rng.choice([1, 2, 3, 5, 8, 12, 15, 16, 17, 33, 72, 100, 4096, 4101])
               for _ in range(rng.randint(1, 8))] for _ in range(60)]
    for sizes in cases:
        seed = rng.randrange(1_000_000_000)
        g = torch.Generator().manual_seed(seed)
        ref = torch.cat([torch.randn(n, dtype=dtype, generator=g) for n in sizes])
        got = torch.empty_like(ref)
        PJ._draw_native(seed, (ctypes.c_int64 * len(sizes))(*sizes), len(sizes), dtype, got)
        diff = (got.view(iv) != ref.view(iv)).sum().item()
        assert diff == 0, f"sizes {sizes[:6]} seed {seed}: {diff} values differ"


@pytest.mark.parametrize("seed", [0, 440527571])
def test_f32_projection_draw_matches_reference_stream(seed):
    """A bucket's fp32 projections equal the reference's per-tensor torch.randn(m, r)."""
    for shapes in ([(2048, 2048)] * 3 + [(40, 16), (4, 3, 3, 3)],
                   [(40, 16), (16, 8, 1, 1), (96, 40), (5461, 33), (10, 2), (7, 3)]):
        segs = A.segments(shapes, 0.2)
        ref = torch.cat([v.flatten() for v in A.draw_projections(seed, segs, 4, torch.float32)
                         if v is not None])
        ms = [s.m for s in segs if s.kind == A.SKETCH]
        got = draw_host(seed, ms, 4, torch.float32, pin=False)
        assert torch.equal(got[:ref.numel()].view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("seed", [0, 440527571])
def test_bf16_projection_draw_matches_reference_stream(seed):
    """A bucket's bf16 projections (fast path and torch fallback) equal the reference's
    per-tensor torch.randn(m, r, dtype=bf16) after the global reseed."""
    for shapes in ([(2048, 2048)] * 3 + [(40, 16), (4, 3, 3, 3)],   # fast path: m*r % 16 == 0
                   [(40, 16), (16, 8, 1, 1), (96, 40), (5461, 33)]):  # m*r = 8, 132: fallback
        segs = A.segments(shapes, 0.2)
        ref = torch.cat([v.flatten() for v in A.draw_projections(seed, segs, 4, torch.bfloat16)
                         if v is not None])
        ms = [s.m for s in segs if s.kind == A.SKETCH]
        got = draw_host(seed, ms, 4, torch.bfloat16, pin=False)
        assert torch.equal(got[:ref.numel()], ref)


def test_state_rng_is_lazy_but_exact():
    """GroupTopKState hands out seeds from a batched look-ahead and draws them from
    state.rng lazily: every observation of the generator (the attribute, state_dict) sees
    exactly one draw per call, as the reference's randint at :254 leaves it, and a caller
    who reseeds the exposed generator gets that sequence from the next call on."""
    from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import GroupTopKState
    st = GroupTopKState(None, seed=5)
    ref = torch.Generator().manual_seed(5)

    def ref_seed():
        return int(torch.randint(0, 1_000_000_000, (1,), generator=ref).item())
    assert [st._next_seed() for _ in range(40)] == [ref_seed() for _ in range(40)]
    assert torch.equal(st.state_dict()["rng_state"], ref.get_state())
    assert not st._rng_strict  # checkpointing does not expose the generator
    g = st.rng
    assert torch.equal(g.get_state(), ref.get_state())
    g.manual_seed(9)
    ref.manual_seed(9)
    assert [st._next_seed() for _ in range(5)] == [ref_seed() for _ in range(5)]
    st2 = GroupTopKState(None, seed=1)
    st2.load_state_dict(st.state_dict())
    assert [st2._next_seed() for _ in range(3)] == [ref_seed() for _ in range(3)]


def test_torch_op_layer_registered():
    """torch.ops.arctopk.* exist with schemas that declare what each op mutates (so the
    dispatcher, torch.compile and graph capture see the codec phases as ops)."""
    import allreducetopk_amd.ops  # noqa: F401
    sch = {name: str(getattr(torch.ops.arctopk, name).default._schema)
           for name in ("draw_projections", "encode", "select", "pack", "decode")}
    import re

    def mutated(s):
        return set(re.findall(r"Tensor\(a\d+!\)\?? (\w+)", s))
    assert mutated(sch["draw_projections"]) == {"V"}
    assert mutated(sch["encode"]) == {"err", "sketch"}
    assert mutated(sch["select"]) == {"rowlist", "slotmap"}
    assert mutated(sch["pack"]) == {"err", "packed"}
    assert mutated(sch["decode"]) == {"gerr", "out"}
