"""The C-ABI library: loads, exports every entry point include/arctopk.h declares, and
its host-only geometry (no GPU needed) agrees with the oracle's reading of the
reference's cal_k / reshape rules (group_topk_hook_no_reshape.py:16-102, :173-187)."""
import ctypes
import os
import re

import pytest

from allreducetopk_amd import _native as N
from allreducetopk_amd.build import LIB, build
from oracle import arctopk as A

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                      "arctopk.h")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        build()
    return N.lib()


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(arctopk_\w+)\s*\(", src,
                                 flags=re.M)))


def test_header_declares_expected_api():
    names = declared_functions()
    for must in ("arctopk_plan_create", "arctopk_encode", "arctopk_select", "arctopk_pack",
                 "arctopk_decode", "arctopk_topk_select", "arctopk_sparse_decode"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert names, "no declarations parsed"
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"declared but not exported: {missing}"
    assert set(names) == set(N.EXPORTS), "ctypes bindings out of sync with include/arctopk.h"


def test_version_string(lib):
    assert b"gfx950" in lib.arctopk_version()


def _describe(lib, shapes, r=4, ratio=0.2):
    dims = [int(d) for s in shapes for d in s]
    nd = [len(s) for s in shapes]
    segs = (N.Segment * len(shapes))()
    info = N.PlanInfo()
    st = lib.arctopk_plan_describe((ctypes.c_int64 * max(1, len(dims)))(*dims),
                                   (ctypes.c_int32 * len(nd))(*nd), len(nd), r, ratio,
                                   ctypes.cast(segs, ctypes.c_void_p), ctypes.byref(info))
    return st, list(segs), info


SHAPE_SETS = [
    [[2048, 2048]] * 16,
    [[10], [40, 16], [4, 3, 3, 3], [16, 8, 3, 3], [16, 8, 1, 1], [96, 40], [7]],
    [[512, 512, 3, 3], [512], [256, 128, 1, 1], [64, 3, 7, 7]],
    [[32000, 2048], [2048], [5461, 2048], [2048, 5461]],
    [[1], [3, 1], [5, 4, 2, 2], [2, 1, 1, 1]],
    [[8, 300000], [2, 3, 3, 3], [10], [2, 140000]],  # wide rows: m * r < 2^31 only
]


@pytest.mark.parametrize("shapes", SHAPE_SETS)
@pytest.mark.parametrize("ratio", [0.2, 0.08, 0.5, 1.0, 0.001])
def test_plan_geometry_matches_oracle(lib, shapes, ratio):
    st, segs, info = _describe(lib, shapes, 4, ratio)
    assert st == 0
    ref = A.segments(shapes, ratio)
    sk = pk = vals = 0
    for s, o in zip(segs, ref):
        assert (s.offset, s.n, s.m, s.k_rows) == (o.offset, o.n, o.m, o.k_rows)
        assert s.kind == o.kind
        assert s.k_rows * s.m == A.cal_k(o.shape, ratio)
        assert s.sketch_off == sk and s.packed_off == pk
        sk += s.n if s.kind == N.SEG_RAW else s.n * 4
        pk += s.k_rows * s.m
        vals += s.k_rows * s.m
        pk = (pk + 3) // 4 * 4  # segments start 16-B aligned in the packed buffer
    assert info.numel == sum(o.numel for o in ref)
    assert info.packed_len == pk and info.sketch_len == sk
    assert info.values_len == vals == sum(A.cal_k(o.shape, ratio) for o in ref)


def test_plan_errors(lib):
    assert _describe(lib, [[3, 5, 2]])[0] == 1002       # 30 % (2*2*2) != 0: reshape raises
    assert _describe(lib, [[4, 0]])[0] == 1004          # empty tensor
    assert _describe(lib, [[4, 4]], r=0)[0] == 1001
    assert _describe(lib, [[4, 4]], r=9)[0] == 1001
    assert _describe(lib, [[4, 4]], ratio=0.0)[0] == 1001
    assert _describe(lib, [[4, 4]], ratio=1.5)[0] == 1001
    assert _describe(lib, [[1, 1 << 29]], r=4)[0] == 1001  # V = m x r past 32-bit indexing


def test_nd_indivisible_matches_reference_error():
    with pytest.raises(RuntimeError):
        A.geometry([3, 5, 2])


def test_compute_entry_points_reject_null_without_touching_device(lib):
    # argument validation happens before any HIP call
    assert lib.arctopk_encode(None, 0, 0, 0, 1, 0, 0, None) == 1001
    assert lib.arctopk_select(None, 0, 1, 0, 0, None) == 1001
    assert lib.arctopk_pack(None, 0, 0, 0, 0, 0, 0, None) == 1001
    assert lib.arctopk_decode(None, 0, 0, 1, 0, 0, 0, None) == 1001
    assert lib.arctopk_ef_apply(None, None, 10, 1, 1, 0, None) == 1001
    assert lib.arctopk_sparse_workspace_bytes(2, N.i64_array([10, 4_000_000])) > 500_000 * 8
    assert lib.arctopk_sparse_workspace_bytes(0, None) == -1001
    assert lib.arctopk_sparse_workspace_bytes(1, N.i64_array([0])) == -1001


def test_library_matches_its_sources(lib):
    """Build integrity: the loaded library carries the hash of the sources next to it, and
    the loader refuses a library whose embedded hash differs (a stale or foreign build)."""
    from allreducetopk_amd import build as B
    assert B.embedded_hash(LIB) == B.source_hash()
    assert f"src:{B.source_hash()}".encode() in lib.arctopk_version()

    class Fake:
        def __init__(self, ver):
            self.arctopk_version = lambda: ver
    with pytest.raises(N.StaleNativeLibrary):
        N._check_build(Fake(b"libarctopk 0.2 gfx950 src:0123456789abcdef"))
    with pytest.raises(N.StaleNativeLibrary):
        N._check_build(Fake(b"libarctopk 0.1 gfx950 (no hash)"))
    N._check_build(Fake(f"libarctopk src:{B.source_hash()}".encode()))


def test_residual_checks_before_any_kernel():
    """A residual on the wrong device is moved to the bucket's; a wrong size or dtype
    raises (a host pointer must never reach a kernel)."""
    import torch
    from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import _residual_on
    bucket = torch.zeros(12)
    table = {0: torch.ones(12, dtype=torch.float64)}
    with pytest.raises(RuntimeError, match="dtype|float64"):
        _residual_on(table, 0, bucket, "error_dict")
    table = {0: torch.ones(13)}
    with pytest.raises(RuntimeError, match="changed size"):
        _residual_on(table, 0, bucket, "error_dict")
    t = torch.arange(24.0)[::2]  # non-contiguous
    table = {0: t}
    got = _residual_on(table, 0, bucket, "error_dict")
    assert got.is_contiguous() and table[0] is got and torch.equal(got, t)


# DDP's reverse parameter order: a bias / BN vector before each conv, so cuts land on RAW
# segments; with r = 2 a 3x3 conv's V (m * r = 36) leaves the next V offset 4 mod 8
GROUP_SHAPE_SETS = SHAPE_SETS + [
    [[64], [64, 64, 3, 3], [64], [64], [64, 64, 3, 3], [64], [128, 64, 3, 3], [128], [128, 128, 3, 3]] * 3,
    [[10], [10, 511], [512], [512], [512, 512, 3, 3], [512], [512, 256, 1, 1], [256], [256, 256, 3, 3]] * 2,
    [[80, 80, 3, 3], [80]] * 6 + [[80, 80, 3, 3]],
]


def plan_group_accepts(segs, a, b):
    """arctopk_plan_group's (plan.hip) alignment rule for the run [a, b), restated: the run's
    first segment's bucket / sketch / packed offsets multiples of 8, its slot-map offset of 4,
    and the V offset of the run's first SKETCH segment a multiple of 8."""
    s = segs[a]
    if s.offset % 8 or s.sketch_off % 8 or s.packed_off % 8 or s.row_off % 4:
        return False
    v = next((t.v_off for t in segs[a:b] if t.kind == N.SEG_SKETCH), -1)
    return v <= 0 or v % 8 == 0


@pytest.mark.parametrize("shapes", GROUP_SHAPE_SETS)
@pytest.mark.parametrize("target", [1 << 12, 1 << 20, 64 << 20])
@pytest.mark.parametrize("r", [2, 4, 3])
def test_group_runs_cut_only_at_aligned_boundaries(lib, shapes, target, r):
    """The exchange groups (arctopk_plan_group): consecutive runs covering every segment once,
    each one a run the native group planner accepts (its rule restated), about `target` bytes
    each."""
    from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import group_runs
    st, segs, info = _describe(lib, shapes, r=r)
    assert st == 0
    runs = group_runs(segs, info.numel, 4, target)
    if runs is None:
        return
    assert runs[0][0] == 0 and runs[-1][1] == len(segs) and len(runs) >= 2
    for (a, b), (c, _) in zip(runs, runs[1:]):
        assert a < b == c
    for a, b in runs:
        assert plan_group_accepts(segs, a, b), (a, b)
    assert len(runs) <= -(-info.numel * 4 // target)


def test_group_runs_skip_misaligned_v_after_a_bias(lib):
    """The ADVICE r05 case: r = 2, a bias then a 3x3 conv whose V offset is 4 mod 8 -- the
    bias's own offsets are aligned, but a run starting there would bind a misaligned V."""
    from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import group_runs
    shapes = [[80, 80, 3, 3], [80]] * 6 + [[80, 80, 3, 3]]
    st, segs, info = _describe(lib, shapes, r=2)
    assert st == 0
    bad = [i for i in range(1, len(segs)) if segs[i].kind == N.SEG_RAW
           and not plan_group_accepts(segs, i, len(segs))
           and segs[i].offset % 8 == 0 and segs[i].sketch_off % 8 == 0 and segs[i].packed_off % 8 == 0]
    assert bad, "the shape set no longer exercises the misaligned-V cut"
    cut = 0
    for target in (1 << 12, 1 << 16, 1 << 18, 1 << 19):
        runs = group_runs(segs, info.numel, 4, target) or []
        assert not any(a in bad for a, _ in runs)
        cut += len(runs)
    assert cut, "no run at all: the test checks nothing"


def test_group_runs_headline_bucket():
    from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import group_runs
    st, segs, info = _describe(N.lib(), [[2048, 2048]] * 16)
    assert group_runs(segs, info.numel, 4, 64 << 20) == [(0, 4), (4, 8), (8, 12), (12, 16)]
    assert group_runs(segs, info.numel, 4, 256 << 20) is None
    st, segs, info = _describe(N.lib(), [[32000, 2048]])
    assert group_runs(segs, info.numel, 4, 64 << 20) is None  # one tensor: never cut
