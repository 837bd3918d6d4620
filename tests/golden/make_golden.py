"""Generate the golden vectors that pin the oracle (and through it the HIP path).

RUNS ONLY IN THE BUILD CONTAINER: it imports the reference hooks from
``/root/reference`` (read-only, pure Python) and drives them on CPU through a
duck-typed bucket over a real ``gloo`` process group of size 1 or 2.  The
reference never travels to the GPU box -- only the ``*.npz`` files written
next to this script do (inputs and expected outputs; no reference source).

Captured per bucket call (reference file:line the value comes from):
  G            input gradient bucket per rank
  seed         ``torch.randint(0, 1e9, generator=state.rng)`` (group_topk_hook_no_reshape.py:254,
               sparse_hook.py:231)
  V_t          projection drawn by ``torch.randn(m, r)`` per 2-D/ND tensor (:49, :79)
  AR_j         every all-reduce result in call order (sketches :33/:58/:88, values :280,
               EF21 init :242; sparse: :218, :273)
  topk_t       (input, k, returned indices) of every ``torch.topk`` (:38/:63/:93; sparse :26)
  perm_t       ``torch.randperm`` outputs (sparse_hook.py:20)
  out          bucket returned by the hook's future
  E, gE        ``state.error_dict[0]`` / ``state.global_error_dict[0]`` after the call
  bits         ``state.comm_bits_this_round`` after the call (utils.py:38)

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import json
import os
import socket
import sys
import tempfile
from contextlib import contextmanager

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE = "/root/reference"
sys.path.insert(0, REPO)

from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel  # noqa: E402

# --------------------------------------------------------------------------
# cases
# --------------------------------------------------------------------------
MIX = [[10], [40, 16], [4, 3, 3, 3], [16, 8, 3, 3], [16, 8, 1, 1], [96, 40], [7]]
SPARSE_MIX = [[10], [40, 16], [4, 3, 3, 3], [96, 40]]
TIES = [[256, 32], [64]]

CASES = []
for ef, iters in (("noef", 2), ("ef14", 3), ("ef21", 3)):
    CASES.append(dict(name=f"arc_mix_{ef}_ws1", hook="arc", shapes=MIX, ratio=0.2, r=4,
                      ef=ef, ws=1, iters=iters, start=0, seed=1234))
for ef in ("ef14", "ef21"):
    CASES.append(dict(name=f"arc_mix_{ef}_ws2", hook="arc", shapes=MIX, ratio=0.2, r=4,
                      ef=ef, ws=2, iters=2, start=0, seed=1234))
CASES += [
    dict(name="arc_mix_ratio008_r2_ws1", hook="arc", shapes=MIX, ratio=0.08, r=2, ef="ef14",
         ws=1, iters=2, start=0, seed=7),
    dict(name="arc_warmup_ef21_ws2", hook="arc", shapes=MIX, ratio=0.2, r=4, ef="ef21",
         ws=2, iters=3, start=1, seed=3),
    dict(name="arc_ties_ef14_ws1", hook="arc", shapes=TIES, ratio=0.2, r=4, ef="ef14",
         ws=1, iters=2, start=0, seed=11, ties=True),
    dict(name="arc_ties_noef_ws1", hook="arc", shapes=TIES, ratio=0.25, r=4, ef="noef",
         ws=1, iters=1, start=0, seed=11, ties=True),
]
# a mix in DDP's reverse order (a bias / norm vector before each weight) whose offsets allow the
# exchange's cuts below a bucket (group_runs: 6 groups of <= 8 KiB): the two-rank grouped
# exchange replays these (tests/test_gpu_multirank.py)
GMIX = [[16], [16, 64], [64], [64], [64, 32, 3, 3], [32], [32, 32, 1, 1], [96, 40], [40], [40, 16, 3, 3], [8]]
CASES += [
    dict(name="arc_gmix_ef14_ws2", hook="arc", shapes=GMIX, ratio=0.2, r=4, ef="ef14", ws=2, iters=3,
         start=0, seed=4321),
    dict(name="arc_gmix_ef21_ws2", hook="arc", shapes=GMIX, ratio=0.2, r=4, ef="ef21", ws=2, iters=3,
         start=0, seed=4321),
    dict(name="arc_gmix_noef_bf16_ws2", hook="arc", shapes=GMIX, ratio=0.2, r=4, ef="noef", ws=2, iters=2,
         start=0, seed=4321, dtype="bf16"),
]
# bf16 buckets (the Llama driver's default dtype, c4/run_llama_pretraining.py:55): V, the
# sketch, norms and values all in bf16 as the reference keeps them in the bucket dtype
for ef, ws, iters in (("ef14", 1, 3), ("ef21", 1, 3), ("noef", 2, 2)):
    CASES.append(dict(name=f"arc_mix_{ef}_bf16_ws{ws}", hook="arc", shapes=MIX, ratio=0.2, r=4,
                      ef=ef, ws=ws, iters=iters, start=0, seed=1234, dtype="bf16"))
for ef in ("noef", "ef14", "ef21"):
    CASES.append(dict(name=f"topk_mix_{ef}_ws1", hook="sparse", random=False, shapes=SPARSE_MIX,
                      ratio=0.2, ef=ef, ws=1, iters=2, start=0, seed=5))
CASES += [
    dict(name="topk_mix_ef14_ws2", hook="sparse", random=False, shapes=SPARSE_MIX, ratio=0.2,
         ef="ef14", ws=2, iters=2, start=0, seed=5),
    dict(name="topk_mix_ef21_ws2", hook="sparse", random=False, shapes=SPARSE_MIX, ratio=0.2,
         ef="ef21", ws=2, iters=2, start=0, seed=5),
    dict(name="randk_mix_ef14_ws1", hook="sparse", random=True, shapes=SPARSE_MIX, ratio=0.2,
         ef="ef14", ws=1, iters=2, start=0, seed=9),
    dict(name="randk_mix_noef_ws2", hook="sparse", random=True, shapes=SPARSE_MIX, ratio=0.2,
         ef="noef", ws=2, iters=2, start=0, seed=9),
    dict(name="topk_c4_gradual_ef14_ws1", hook="sparse_c4", random=False, shapes=SPARSE_MIX,
         ratio=0.2, ef="ef14", ws=1, iters=4, start=1, seed=5),
    dict(name="randk_c4_gradual_ef21_ws1", hook="sparse_c4", random=True, shapes=SPARSE_MIX,
         ratio=0.1, ef="ef21", ws=1, iters=4, start=1, seed=21),
    # EF21 residual scaling (state.error_decay, set by hand: sparse_hook.py:145 fixes 1.0;
    # applied at :265 and :296)
    dict(name="topk_mix_ef21_decay09_ws1", hook="sparse", random=False, shapes=SPARSE_MIX,
         ratio=0.2, ef="ef21", ws=1, iters=3, start=0, seed=5, error_decay=0.9),
    dict(name="topk_mix_ef21_decay07_ws2", hook="sparse", random=False, shapes=SPARSE_MIX,
         ratio=0.2, ef="ef21", ws=2, iters=3, start=0, seed=5, error_decay=0.7),
    dict(name="topk_c4_gradual_ef21_decay09_ws1", hook="sparse_c4", random=False, shapes=SPARSE_MIX,
         ratio=0.2, ef="ef21", ws=1, iters=3, start=1, seed=5, error_decay=0.9),
    # EF21 with large-batch initialisation (state.large_batch_init, set by hand: both
    # constructors fix False; sparse_hook.py:172-175 -> :307-416).  Its iteration-0 branch calls
    # default_hooks._allreduce_fut without the required hook_state and raises TypeError, and the
    # registered copy (sparse_hook_c4.py:353-457) also fails at its first compressed call
    # (large_batch_errors.json), so these runs use sparse_hook and start at iteration 1 (iter0):
    # two accumulating dense iterations, then the averaged residuals and compressed calls.
    dict(name="topk_largebatch_ef21_ws1", hook="sparse", random=False, shapes=SPARSE_MIX,
         ratio=0.2, ef="ef21", ws=1, iters=4, start=3, seed=5, large_batch=True, iter0=1),
    dict(name="topk_largebatch_ef21_decay07_ws2", hook="sparse", random=False, shapes=SPARSE_MIX,
         ratio=0.2, ef="ef21", ws=2, iters=4, start=3, seed=5, large_batch=True, iter0=1,
         error_decay=0.7),
    dict(name="randk_largebatch_ef21_ws2", hook="sparse", random=True, shapes=SPARSE_MIX,
         ratio=0.2, ef="ef21", ws=2, iters=4, start=3, seed=9, large_batch=True, iter0=1),
]


def make_grad(case, it, rank):
    """Deterministic synthetic gradient bucket for (iteration, rank)."""
    g = torch.Generator().manual_seed(1000 + 100 * it + rank)
    x = torch.randn(bucket_numel(case["shapes"]), generator=g)
    if case.get("ties"):
        # embedding-like: most rows exactly zero (common in real embedding grads), and a
        # 1-D tensor with zeros -> exact ties at the k-th norm.
        n0 = case["shapes"][0][0] * case["shapes"][0][1]
        rows = x[:n0].view(case["shapes"][0])
        keep = torch.zeros(case["shapes"][0][0], dtype=torch.bool)
        keep[torch.randperm(case["shapes"][0][0], generator=g)[: case["shapes"][0][0] // 8]] = True
        rows[~keep] = 0.0
        tail = x[n0:]
        tail[torch.rand(tail.numel(), generator=g) < 0.6] = 0.0
    if case.get("dtype") == "bf16":
        x = x.to(torch.bfloat16)
    return x


def _np(t):
    """numpy has no bf16: bf16 tensors are stored as their int16 bit patterns (meta dtype)."""
    t = t.detach().cpu()
    return t.view(torch.int16).numpy() if t.dtype == torch.bfloat16 else t.numpy()


# --------------------------------------------------------------------------
# capture of reference internals
# --------------------------------------------------------------------------
@contextmanager
def capture(rec):
    orig = dict(manual_seed=torch.manual_seed, randn=torch.randn, topk=torch.topk,
                randperm=torch.randperm, all_reduce=dist.all_reduce)

    def manual_seed(s):
        rec.setdefault("seed", []).append(int(s))
        return orig["manual_seed"](s)

    def randn(*a, **k):
        out = orig["randn"](*a, **k)
        rec.setdefault("V", []).append(out.detach().clone())
        return out

    def topk(inp, k=None, *a, **kw):
        res = orig["topk"](inp, k, *a, **kw)
        rec.setdefault("topk", []).append((inp.detach().clone(), int(k), res[1].detach().clone()))
        return res

    def randperm(*a, **k):
        out = orig["randperm"](*a, **k)
        rec.setdefault("perm", []).append(out.detach().clone())
        return out

    def all_reduce(t, *a, **k):
        res = orig["all_reduce"](t, *a, **k)
        if k.get("async_op"):
            res.wait()
        rec.setdefault("AR", []).append(t.detach().clone())
        return res

    torch.manual_seed, torch.randn, torch.topk, torch.randperm = manual_seed, randn, topk, randperm
    dist.all_reduce = all_reduce
    try:
        yield rec
    finally:
        torch.manual_seed = orig["manual_seed"]
        torch.randn, torch.topk, torch.randperm = orig["randn"], orig["topk"], orig["randperm"]
        dist.all_reduce = orig["all_reduce"]


def make_state(case):
    st, hook = _make_state(case)
    if "error_decay" in case:
        st.error_decay = case["error_decay"]
    if case.get("large_batch"):
        st.large_batch_init = True
    st.iter = case.get("iter0", 0)
    return st, hook


def _make_state(case):
    if case["hook"] == "arc":
        from comm_hooks.group_topk_hook_no_reshape import GroupTopKState, group_topk_hook
        st = GroupTopKState(process_group=None, r=case["r"], compress_ratio=case["ratio"],
                            start_compress_iter=case["start"], use_error_feedback=case["ef"],
                            seed=case["seed"])
        return st, group_topk_hook
    if case["hook"] == "sparse":
        from comm_hooks.sparse_hook import SparseState, sparse_hook_sync
        st = SparseState(process_group=None, compress_ratio=case["ratio"],
                         start_compress_iter=case["start"], sparse_type="tensor",
                         random=case["random"], use_error_feedback=case["ef"],
                         random_seed=case["seed"])
        return st, sparse_hook_sync
    from comm_hooks.sparse_hook_c4 import SparseState, sparse_hook_sync
    st = SparseState(process_group=None, compress_ratio=case["ratio"],
                     start_compress_iter=case["start"], sparse_type="tensor",
                     random=case["random"], use_error_feedback=case["ef"],
                     random_seed=case["seed"])
    return st, sparse_hook_sync


def run_rank(rank, ws, case, port, outdir):
    sys.path.insert(0, REFERENCE)
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    torch.set_num_threads(max(1, 8 // ws))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=ws)
    state, hook = make_state(case)
    arrays = {}
    for it in range(case["iters"]):
        G = make_grad(case, it, rank)
        bucket = SyntheticBucket(G.clone(), case["shapes"], index=0, is_last=True)
        rec = {}
        with capture(rec):
            fut = hook(state, bucket)
            out = fut.wait()
        p = f"it{it}_"
        arrays[p + "G"] = _np(G)
        arrays[p + "out"] = _np(out.clone())
        if 0 in getattr(state, "error_dict", {}):
            arrays[p + "E"] = _np(state.error_dict[0].clone())
        if 0 in getattr(state, "global_error_dict", {}):
            arrays[p + "gE"] = _np(state.global_error_dict[0].clone())
        arrays[p + "bits"] = np.array(int(state.comm_bits_this_round), dtype=np.int64)
        arrays[p + "iter_after"] = np.array(int(state.iter), dtype=np.int64)
        if "seed" in rec:
            arrays[p + "seed"] = np.array(rec["seed"], dtype=np.int64)
        for j, v in enumerate(rec.get("V", [])):
            arrays[p + f"V{j}"] = _np(v)
        for j, a in enumerate(rec.get("AR", [])):
            arrays[p + f"AR{j}"] = _np(a)
        for j, (inp, k, idx) in enumerate(rec.get("topk", [])):
            arrays[p + f"topk{j}_in"] = _np(inp)
            arrays[p + f"topk{j}_k"] = np.array(k, dtype=np.int64)
            arrays[p + f"topk{j}_idx"] = idx.numpy()
        for j, perm in enumerate(rec.get("perm", [])):
            arrays[p + f"perm{j}"] = perm.numpy()
        if hasattr(state, "get_current_compress_ratio"):
            arrays[p + "ratio_now"] = np.array(state.get_current_compress_ratio(), dtype=np.float64)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **arrays)
    dist.barrier()
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def make_error_case():
    """ND tensor whose numel is not divisible by m = 2*t^2 -> reference raises."""
    sys.path.insert(0, REFERENCE)
    from comm_hooks.group_topk_hook_no_reshape import group_topk_project_and_select
    t = torch.randn(3, 5, 2)
    try:
        group_topk_project_and_select(t, 4, 0.2, None)
    except RuntimeError as e:  # raised by reshape before any collective
        return type(e).__name__
    return "no-error"


def large_batch_errors(rank, port, outdir):
    """How the large-batch EF21 hooks fail (sparse_hook.py:336-338, sparse_hook_c4.py:384-386 at
    iteration 0; sparse_hook_c4.py:421 at the first compressed call): exception, message, and
    the iteration counter afterwards."""
    sys.path.insert(0, REFERENCE)
    sys.dont_write_bytecode = True
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    out = {}
    for tag, hook_name, iter0 in (("sparse_iter0", "sparse", 0), ("sparse_c4_iter0", "sparse_c4", 0),
                                  ("sparse_c4_compressed", "sparse_c4", 3)):
        case = dict(hook=hook_name, random=False, ratio=0.2, start=3, ef="ef21", seed=5, large_batch=True,
                    iter0=iter0)
        state, hook = make_state(case)
        if iter0 >= 3:  # residuals as the accumulating iterations leave them
            state.error_dict[0] = torch.zeros(bucket_numel(SPARSE_MIX))
            state.global_error_dict[0] = torch.zeros(bucket_numel(SPARSE_MIX))
        bucket = SyntheticBucket(torch.randn(bucket_numel(SPARSE_MIX)), SPARSE_MIX, index=0, is_last=True)
        try:
            hook(state, bucket)
            res = dict(raises="no-error")
        except Exception as e:  # noqa: BLE001 -- recorded as the reference's behaviour
            res = dict(raises=type(e).__name__, message=str(e))
        res["iter_after"] = int(state.iter)
        out[tag] = res
    with open(os.path.join(outdir, "err.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


def main():
    meta_common = dict(torch=torch.__version__, cpu_capability=torch.backends.cpu.get_cpu_capability(),
                       reference="Aris-ma/AllreduceTopK @ /root/reference (read-only)")
    only = set(sys.argv[1:])
    for case in CASES:
        if only and case["name"] not in only:
            continue
        with tempfile.TemporaryDirectory() as td:
            port = free_port()
            mp.spawn(run_rank, args=(case["ws"], case, port, td), nprocs=case["ws"], join=True)
            merged = {}
            for rk in range(case["ws"]):
                with np.load(os.path.join(td, f"rank{rk}.npz")) as z:
                    for k in z.files:
                        merged[f"r{rk}_{k}"] = z[k]
        meta = dict(meta_common, **case)
        merged["meta"] = np.array(json.dumps(meta))
        np.savez_compressed(os.path.join(HERE, case["name"] + ".npz"), **merged)
        print("wrote", case["name"], sum(v.nbytes for v in merged.values()), "bytes raw")
    err = make_error_case()
    with open(os.path.join(HERE, "nd_indivisible_error.json"), "w") as f:
        json.dump(dict(meta_common, shape=[3, 5, 2], r=4, ratio=0.2, raises=err), f, indent=1)
    with tempfile.TemporaryDirectory() as td:
        port = free_port()
        mp.spawn(large_batch_errors, args=(port, td), nprocs=1, join=True)
        with open(os.path.join(td, "err.json")) as f:
            res = json.load(f)
    with open(os.path.join(HERE, "large_batch_errors.json"), "w") as f:
        json.dump(dict(meta_common, cases=res), f, indent=1)


if __name__ == "__main__":
    main()
