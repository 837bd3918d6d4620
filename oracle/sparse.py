"""ORACLE (test infrastructure only) -- CPU restatement of the TopK / RandK baselines.

Restates comm_hooks/sparse_hook.py (fixed ratio) and comm_hooks/sparse_hook_c4.py
(gradual ratio 0.8 -> target, the copy the reference registry actually uses,
comm_hooks/utils.py:94) with ``sparse_type='tensor'`` -- the only working type
(row/column return 2-tuples where 3 are unpacked, sparse_hook.py:54, :75, :96).

  sparsify   TopK: topk(|x|, k, sorted=False) -> int32 idx; RandK: randperm(numel)[:k]
             after the shared reseed (sparse_hook.py:16-34, :230-235)
  pack       values/indices per tensor; EF14 zero / EF21 keep-only (:92-110)
  decode     RandK: all-reduce, /ws, scatter (=) (:270-278)
             TopK : all-gather, scatter-add in rank order, /ws (:279-292)
  EF         pre-apply (:202-226) and residual persistence (:257-267), EF21 gE (:295-297)
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch


def numel_of(shape) -> int:
    n = 1
    for d in shape:
        n *= int(d)
    return n


def cal_k(numel: int, ratio: float) -> int:  # sparse_hook.py:77-78
    return max(1, int(numel * ratio))


def gradual_ratio(base: float, it: int, start: int, warmup_iters: int = 100,
                  started: bool = True, gradual: bool = True) -> float:
    """sparse_hook_c4.py:175-189 (note warmup span = start + warmup_iters, :151)."""
    if not gradual or not started:
        return base
    span = start + warmup_iters
    prog = it - start
    if prog < span:
        cur = 0.8 - (0.8 - base) * (prog / span)
        return max(cur, base)
    return base


def topk_indices(x: torch.Tensor, k: int) -> torch.Tensor:
    _, idx = torch.topk(x.abs(), k, sorted=False)
    return idx.to(torch.int32)


def randk_indices(numel: int, k: int, g: torch.Generator) -> torch.Tensor:
    return torch.randperm(numel, generator=g)[:k].to(torch.int32)


_M32 = 0xFFFFFFFF


def _rk_mix(h):  # numpy uint64 arrays holding 32-bit values
    import numpy as np
    h = h ^ (h >> np.uint64(16))
    h = (h * np.uint64(0x7FEB352D)) & np.uint64(_M32)
    h = h ^ (h >> np.uint64(15))
    h = (h * np.uint64(0x846CA68B)) & np.uint64(_M32)
    return h ^ (h >> np.uint64(16))


def randk_hash_seed(seed: int, t: int) -> int:
    """The tensor key seed of the device RandK draw (sparse_kernels.hip rk_tensor_seed):
    splitmix64(seed + golden * (t + 1)), low 32 bits."""
    m = (1 << 64) - 1
    z = (seed + 0x9E3779B97F4A7C15 * (t + 1)) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return (z ^ (z >> 31)) & _M32


def randk_hash_indices(numel: int, k: int, seed: int, t: int) -> torch.Tensor:
    """The device RandK index rule (index_source="hash", the performance mode -- not the
    reference's torch.randperm draw, sparse_hook.py:20): the indices of the k largest keys
    rk(s, j) = mix(mix(j ^ s) + 0x9E3779B9 * (s | 1)) over j < numel, ascending.  mix is a
    bijection on 32 bits, so the keys are distinct and the subset is a uniform k-subset."""
    import numpy as np
    s = np.uint64(randk_hash_seed(seed, t))
    j = np.arange(numel, dtype=np.uint64)
    inner = _rk_mix(j ^ s)
    key = _rk_mix((inner + np.uint64((0x9E3779B9 * (int(s) | 1)) & _M32)) & np.uint64(_M32))
    top = np.argpartition(-key.astype(np.int64), k - 1)[:k] if k < numel else np.arange(numel)
    return torch.from_numpy(np.sort(top).astype(np.int32))


def encode(G, E, ef):
    X = G.clone()
    if E is not None:
        if ef == "ef14":
            X.add_(E, alpha=1.0)
        elif ef == "ef21":
            X.add_(E, alpha=-1.0)
    return X


def pack(X: torch.Tensor, shapes, ratio: float, ef: str, random: bool, seed: Optional[int],
         indices_override=None):
    """Returns (values, indices int32, k_list, bits_sum); mutates X per EF mode.

    ``indices_override`` (one index tensor per tensor) replaces the index draw.
    """
    g = torch.Generator().manual_seed(int(seed)) if (random and indices_override is None) else None
    vals, idxs, ks, bits = [], [], [], 0
    off = 0
    for s in shapes:
        n = numel_of(s)
        v = X[off:off + n]
        k = cal_k(n, ratio)
        if indices_override is not None:
            idx = torch.as_tensor(indices_override[len(ks)]).to(torch.int32)
        else:
            idx = randk_indices(n, k, g) if random else topk_indices(v, k)
        val = v[idx.long()].clone()
        vals.append(val)
        idxs.append(idx)
        ks.append(k)
        bits += val.numel() * torch.finfo(X.dtype).bits + (0 if random else idx.numel() * 32)
        if ef == "ef14":
            v[idx.long()] = 0
        elif ef == "ef21":
            v.zero_()
            v[idx.long()] = val
        off += n
    return torch.cat(vals), torch.cat(idxs), ks, bits


def decode_randk(vsum: torch.Tensor, idx: torch.Tensor, shapes, ks, ws: int, numel: int):
    vals = vsum.clone()
    vals.div_(ws)
    out = torch.zeros(numel, dtype=vsum.dtype)
    off = koff = 0
    for s, k in zip(shapes, ks):
        n = numel_of(s)
        out[off:off + n][idx[koff:koff + k].long()] = vals[koff:koff + k]
        off += n
        koff += k
    return out


def decode_topk(all_vals: List[torch.Tensor], all_idx: List[torch.Tensor], shapes, ks, ws: int,
                numel: int):
    out = torch.zeros(numel, dtype=all_vals[0].dtype)
    for vals, idx in zip(all_vals, all_idx):  # rank order
        off = koff = 0
        for s, k in zip(shapes, ks):
            n = numel_of(s)
            view = out[off:off + n]
            view[idx[koff:koff + k].long()] += vals[koff:koff + k]
            off += n
            koff += k
    out.div_(ws)
    return out


def simulate_step(Gs, Es, gE, shapes, ratio: float, ef: str, random: bool, seed: Optional[int],
                  indices_override=None, error_decay: float = 1.0, residual_decay: Optional[float] = None):
    """One steady-state compressed call on len(Gs) ranks in one process.

    ``indices_override``: per rank, a list of per-tensor index tensors (RandK draws
    made elsewhere, e.g. by the device generator).  ``error_decay``: EF21's residual scaling
    (``E.add_(C, alpha=error_decay)``, ``gE.add_(out, alpha=error_decay)``, sparse_hook.py:265,
    :296; sparse_hook_c4.py:311, :342).  ``residual_decay`` overrides the local residual's
    factor (the large-batch hook adds C with alpha 1.0 but scales gE: sparse_hook.py:386, :410).
    """
    e_decay = error_decay if residual_decay is None else residual_decay
    ws = len(Gs)
    Xs, packs = [], []
    for q, (G, E) in enumerate(zip(Gs, Es)):
        X = encode(G, E, ef)
        ov = indices_override[q] if indices_override is not None else None
        packs.append(pack(X, shapes, ratio, ef, random, seed, ov))
        Xs.append(X)
    ks = packs[0][2]
    numel = Gs[0].numel()
    if random:
        vsum = packs[0][0].clone()
        for q in range(1, ws):
            vsum = vsum + packs[q][0]
        out = decode_randk(vsum, packs[0][1], shapes, ks, ws, numel)
    else:
        out = decode_topk([p[0] for p in packs], [p[1] for p in packs], shapes, ks, ws, numel)
    E_new = []
    for X, E in zip(Xs, Es):
        if ef == "ef14":
            E_new.append(X.clone())
        elif ef == "ef21":  # X holds C(D): zero except the selection (:265)
            E_new.append(E.clone().add_(X, alpha=e_decay))
        else:
            E_new.append(None)
    gE_new = None
    if ef == "ef21":  # (:296-297)
        gE_new = gE.clone().add_(out, alpha=error_decay)
        out = gE_new.clone()
    return dict(X=Xs, values=[p[0] for p in packs], indices=[p[1] for p in packs], ks=ks,
                bits=packs[0][3], out=out, E_new=E_new, gE_new=gE_new)


@dataclass
class LargeBatchState:
    """The EF21 large-batch-initialisation hook's state (sparse_hook.py:307-416, reached when
    ``state.large_batch_init`` is set by hand), for ``ws`` ranks simulated in one process."""
    ws: int
    shapes: list
    ratio: float
    random: bool
    start: int
    seed: int = 0
    error_decay: float = 1.0
    iter: int = 0
    Es: Optional[List[torch.Tensor]] = None
    gE: Optional[torch.Tensor] = None
    rng: torch.Generator = field(default=None)

    def __post_init__(self):
        if self.rng is None:
            self.rng = torch.Generator().manual_seed(int(self.seed))


def large_batch_call(st: LargeBatchState, Gs: List[torch.Tensor]) -> dict:
    """One call of sparse_hook_sync_large_batch_ef21 on every rank (one bucket, iter advancing
    as for the last bucket).  Returns dict(out, E, gE, seed, indices) after the call.

      iter < 1            : TypeError (the reference calls default_hooks._allreduce_fut without
                            its required hook_state, :336-338), after iter += 1
      1 <= iter < start   : E += G; out = all_reduce(G) / ws; gE += out            (:339-353)
      iter == start       : E /= start - 1; gE /= start - 1                         (:354-356)
      iter >= start       : D = G - E; C = sparsify(D) (compress_ratio, not the gradual one);
                            E += C; out = mean of C over ranks (RandK: all_reduce / ws;
                            TopK: rank-ordered scatter-add / ws); gE += error_decay * out;
                            out = gE                                                 (:358-410)
    The hook counts no communication bits."""
    ws = st.ws
    if st.iter < 1:
        st.iter += 1
        raise TypeError("_allreduce_fut() missing 1 required positional argument: 'hook_state'")
    if st.iter < st.start:
        if st.Es is None:
            st.Es = [torch.zeros_like(G) for G in Gs]
            st.gE = torch.zeros_like(Gs[0])
        for E, G in zip(st.Es, Gs):
            E.add_(G, alpha=1.0)
        acc = Gs[0].clone()
        for q in range(1, ws):
            acc = acc + Gs[q]
        acc.div_(ws)
        st.gE.add_(acc, alpha=1.0)
        st.iter += 1
        return dict(out=acc, E=[E.clone() for E in st.Es], gE=st.gE.clone(), seed=None, indices=None)
    if st.iter == st.start:
        for E in st.Es:
            E.div_(st.start - 1)
        st.gE.div_(st.start - 1)
    seed = int(torch.randint(0, 1_000_000_000, (1,), generator=st.rng).item()) if st.random else None
    res = simulate_step(Gs, st.Es, st.gE, st.shapes, st.ratio, "ef21", st.random, seed,
                        error_decay=st.error_decay, residual_decay=1.0)
    st.Es, st.gE = res["E_new"], res["gE_new"]
    st.iter += 1
    return dict(out=res["out"], E=[E.clone() for E in st.Es], gE=st.gE.clone(), seed=seed,
                indices=res["indices"])
