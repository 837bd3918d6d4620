"""ORACLE (test infrastructure only) -- CPU restatement of ARC-TopK.

Restates comm_hooks/group_topk_hook_no_reshape.py of the reference as four
phases, the same cut the HIP path uses, so each kernel can be checked on its
own:

  encode  EF pre-apply + per-tensor rank-r sketch      (ref :224-250, :28, :49-53, :79-83)
  select  mean of all-reduced sketch, row energy, top-k (ref :33-38, :58-63, :88-93)
  pack    gather selected rows, EF residual update      (ref :64-71, :94-102, :111-129, :270-275)
  decode  mean of all-reduced values, scatter, EF21 gE  (ref :280-290, :131-141)

plus ``oracle_group_topk_hook`` which chains them behind a real
``torch.distributed`` group, and ``simulate`` which runs ``ws`` ranks in one
process (sums in rank order; bitwise equal to gloo for ws <= 2).

Float arithmetic follows the reference op for op (torch CPU ``mm``,
``P /= ws``, ``sum(P**2, dim=1)``, ``torch.topk(sorted=False)``, ``div_``),
so at ws=1 outputs are bit-identical to the reference (pinned by
tests/test_oracle_golden.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

RAW, SKETCH = 0, 1


@dataclass
class Segment:
    """One gradient view of the bucket, seen as an (n rows x m cols) matrix."""
    kind: int      # RAW (1-D tensor: every element is a 'row', sketch = the values) or SKETCH
    offset: int    # element offset inside the flat bucket
    numel: int
    n: int         # rows
    m: int         # columns (1 for RAW)
    k_rows: int    # selected rows
    shape: tuple

    @property
    def k(self) -> int:  # selected elements (reference cal_k)
        return self.k_rows * self.m


def geometry(shape: Sequence[int]):
    """(kind, n, m) of a gradient tensor -- ref :19 / :44-46 / :73-76."""
    shape = tuple(int(s) for s in shape)
    d = 1
    for s in shape:
        d *= s
    if len(shape) == 1:
        return RAW, d, 1
    if len(shape) == 2:
        return SKETCH, shape[0], shape[1]
    t = shape[-1]
    m = 2 * t * t
    n = d // m
    if n * m != d:  # tensor.reshape(n, m) raises in the reference (:76)
        raise RuntimeError(f"shape '[{n}, {m}]' is invalid for input of size {d}")
    return SKETCH, n, m


def cal_k(shape, ratio: float) -> int:
    """Reference cal_k (:173-187): float64 product, truncation by int()."""
    kind, n, m = geometry(shape)
    return max(1, int(n * ratio)) * m


def segments(shapes, ratio: float) -> List[Segment]:
    out, off = [], 0
    for s in shapes:
        kind, n, m = geometry(s)
        out.append(Segment(kind, off, n * m, n, m, max(1, int(n * ratio)), tuple(s)))
        off += n * m
    return out


def draw_projections(seed: int, segs: List[Segment], r: int, dtype=torch.float32, device=None):
    """V per SKETCH tensor, in bucket order, as the reference draws them after its global
    reseed (``torch.manual_seed(seed)``, :255): ``torch.randn(m, r, device=tensor.device,
    dtype)`` per 2-D/ND tensor in order (:49, :79).

    device None: the reference run on CPU -- a private CPU generator seeded the same way
    yields the same stream.  device "cuda:i": the reference run on that GPU -- the same
    global reseed and per-tensor torch.randn on the device (the device's Philox stream),
    returned on the CPU for the oracle's arithmetic.
    """
    if device is None:
        g = torch.Generator().manual_seed(int(seed))
        return [torch.randn(s.m, r, generator=g, dtype=dtype) if s.kind == SKETCH else None
                for s in segs]
    torch.manual_seed(int(seed))
    return [torch.randn(s.m, r, device=device, dtype=dtype).cpu() if s.kind == SKETCH else None
            for s in segs]


def encode(G: torch.Tensor, E: Optional[torch.Tensor], ef: str, segs, Vs):
    """EF pre-apply then local sketches.  Returns (X, [P_local per segment]).

    X is the bucket after EF pre-apply (ef14: G+E, ef21: G-E, noef/first call: G).
    """
    X = G.clone()
    if E is not None:
        if ef == "ef14":
            X.add_(E, alpha=1.0)
        elif ef == "ef21":
            X.add_(E, alpha=-1.0)
    Ps = []
    for s, V in zip(segs, Vs):
        v = X[s.offset:s.offset + s.numel]
        Ps.append(v.clone() if s.kind == RAW else v.view(s.n, s.m) @ V)
    return X, Ps


def row_energy(P: torch.Tensor, kind: int) -> torch.Tensor:
    return P ** 2 if kind == RAW else torch.sum(P ** 2, dim=1)


def select(P_sum: List[torch.Tensor], ws: int, segs):
    """Mean sketch, row energy, top-k rows (torch.topk, sorted=False) per segment."""
    norms, rows = [], []
    for P, s in zip(P_sum, segs):
        P = P.clone()
        P /= ws
        nrm = row_energy(P, s.kind)
        _, idx = torch.topk(nrm, k=s.k_rows, largest=True, sorted=False)
        norms.append(nrm)
        rows.append(idx)
    return norms, rows


def pack(X: torch.Tensor, rows, segs, ef: str):
    """Gather selected rows (packed, in ``rows`` order); EF14 zero / EF21 keep-only.

    Mutates X like the reference mutates the bucket (:122-128); returns packed values.
    """
    vals = []
    for s, idx in zip(segs, rows):
        v2 = X[s.offset:s.offset + s.numel].view(s.n, s.m)
        sel = v2[idx].flatten().clone()
        vals.append(sel)
        if ef == "ef14":
            v2[idx] = 0
        elif ef == "ef21":
            v2.zero_()
            v2[idx] = sel.view(-1, s.m)
    return torch.cat(vals) if vals else X.new_empty(0)


def decode(values_sum: torch.Tensor, ws: int, rows, segs, numel: int, dtype):
    """Mean of the all-reduced packed values scattered into a zero bucket (:281-285)."""
    vals = values_sum.clone()
    vals.div_(ws)
    out = torch.zeros(numel, dtype=dtype)
    off = 0
    for s, idx in zip(segs, rows):
        out[s.offset:s.offset + s.numel].view(s.n, s.m)[idx] = vals[off:off + s.k].view(-1, s.m)
        off += s.k
    return out


def bits_per_call(segs, r: int, dtype_bits: int) -> int:
    """bits_sum of one bucket call: sketch P bits + selected value bits (:32, :57, :70, :119)."""
    total = 0
    for s in segs:
        p_elems = s.numel if s.kind == RAW else s.n * r
        total += (p_elems + s.k) * dtype_bits
    return total


# ---------------------------------------------------------------------------
# whole-call restatements
# ---------------------------------------------------------------------------
@dataclass
class OracleState:
    r: int = 4
    compress_ratio: float = 0.08
    start_compress_iter: int = 2
    use_error_feedback: str = "noef"
    seed: int = 0
    iter: int = 0
    comm_bits_this_round: int = 0
    error_dict: Dict[int, torch.Tensor] = field(default_factory=dict)
    global_error_dict: Dict[int, torch.Tensor] = field(default_factory=dict)
    rng: torch.Generator = None

    def __post_init__(self):
        self.rng = torch.Generator().manual_seed(self.seed)

    def next_seed(self) -> int:  # ref :254
        return int(torch.randint(0, 1_000_000_000, (1,), generator=self.rng).item())


def _dtype_bits(dtype) -> int:
    return torch.finfo(dtype).bits


def oracle_group_topk_hook(state: OracleState, bucket, group=None) -> torch.Tensor:
    """The full reference hook restated over a real process group, in the reference's
    in-place op order (group_topk_hook_no_reshape.py:190-297): EF pre-apply into the bucket,
    per-tensor sketches, select, gather + EF14 zero / EF21 keep-only in the bucket, residual
    persistence, packed all-reduce, bucket.zero_() + scatter, EF21 gE.  (bench.py's CPU
    baseline times this; the one sketch all-reduce per bucket sums the same elements as the
    reference's one per tensor.)  Returns the bucket."""
    group = group if group is not None else dist.group.WORLD
    ws = dist.get_world_size(group)
    buf = bucket.buffer()
    shapes = [tuple(t.shape) for t in bucket.gradients()]
    if state.iter < state.start_compress_iter:  # default_hooks._allreduce_fut (ref :213-215)
        buf.div_(ws)
        state.comm_bits_this_round += 2 * (ws - 1) * buf.numel() * _dtype_bits(buf.dtype)
        dist.all_reduce(buf, group=group)
        if bucket.is_last():
            state.iter += 1
        return buf
    b = bucket.index()
    ef = state.use_error_feedback
    if ef == "ef14":  # (:224-230)
        if b in state.error_dict:
            buf.add_(state.error_dict[b], alpha=1.0)
        else:
            state.error_dict[b] = torch.zeros_like(buf)
    elif ef == "ef21":  # (:231-250)
        if b in state.error_dict:
            buf.add_(state.error_dict[b], alpha=-1.0)
        else:
            state.error_dict[b] = buf.clone()
            state.comm_bits_this_round += buf.numel() * _dtype_bits(buf.dtype)
            dist.all_reduce(buf, group=group)
            buf.div_(ws)
            state.global_error_dict[b] = buf.clone()
            if bucket.is_last():
                state.iter += 1
            return buf
    seed = state.next_seed()  # (:254-255)
    torch.manual_seed(seed)
    segs = segments(shapes, state.compress_ratio)
    Vs = draw_projections(seed, segs, state.r, buf.dtype)
    Ps = [buf[s.offset:s.offset + s.numel].clone() if s.kind == RAW
          else buf[s.offset:s.offset + s.numel].view(s.n, s.m) @ V for s, V in zip(segs, Vs)]
    flat = torch.cat([p.flatten() for p in Ps])
    dist.all_reduce(flat, group=group)
    P_sum, off = [], 0
    for p in Ps:
        P_sum.append(flat[off:off + p.numel()].view_as(p))
        off += p.numel()
    _, rows = select(P_sum, ws, segs)
    vals = pack(buf, rows, segs, ef)  # gathers; EF14 zeroes / EF21 keeps only the selection, in place
    if ef == "ef14":  # (:270-275)
        state.error_dict[b].copy_(buf)
    elif ef == "ef21":
        state.error_dict[b].add_(buf)
    state.comm_bits_this_round += 2 * (ws - 1) * bits_per_call(segs, state.r, _dtype_bits(buf.dtype))
    dist.all_reduce(vals, group=group)  # (:280-285)
    vals.div_(ws)
    buf.zero_()
    off = 0
    for s_, idx in zip(segs, rows):
        buf[s_.offset:s_.offset + s_.numel].view(s_.n, s_.m)[idx] = vals[off:off + s_.k].view(-1, s_.m)
        off += s_.k
    if ef == "ef21":  # (:288-290)
        state.global_error_dict[b].add_(buf)
        buf.copy_(state.global_error_dict[b])
    if bucket.is_last():
        state.iter += 1
    return buf


def simulate_step(Gs: List[torch.Tensor], Es: List[Optional[torch.Tensor]], gE: Optional[torch.Tensor],
                  shapes, ratio: float, r: int, ef: str, seed: int, rows_override=None,
                  proj_device=None):
    """One steady-state compressed call on ``len(Gs)`` ranks in one process.

    Collectives are sums in rank order.  Returns a dict of intermediates and
    per-rank results: V, P_local, P_sum, norms, rows, X (post-pack bucket
    contents), values, out, E_new, gE_new.  ``rows_override`` (list of row index
    tensors per segment) replaces the top-k choice -- used to compare a device
    run's outputs bit for bit given the rows that run selected.  ``proj_device``: draw V
    as the reference does on that GPU (see draw_projections).
    """
    ws = len(Gs)
    segs = segments(shapes, ratio)
    Vs = draw_projections(seed, segs, r, Gs[0].dtype, device=proj_device)
    Xs, Pls = [], []
    for G, E in zip(Gs, Es):
        X, Ps = encode(G, E, ef, segs, Vs)
        Xs.append(X)
        Pls.append(Ps)
    P_sum = []
    for j in range(len(segs)):
        acc = Pls[0][j].clone()
        for q in range(1, ws):
            acc = acc + Pls[q][j]
        P_sum.append(acc)
    norms, rows = select(P_sum, ws, segs)
    if rows_override is not None:
        rows = [torch.as_tensor(x, dtype=torch.int64) for x in rows_override]
    vals = [pack(X, rows, segs, ef) for X in Xs]
    vsum = vals[0].clone()
    for q in range(1, ws):
        vsum = vsum + vals[q]
    numel = Gs[0].numel()
    out = decode(vsum, ws, rows, segs, numel, Gs[0].dtype)
    E_new = []
    for X, E in zip(Xs, Es):
        if ef == "ef14":
            E_new.append(X.clone())
        elif ef == "ef21":
            E_new.append(E + X)
        else:
            E_new.append(None)
    gE_new = None
    if ef == "ef21":
        gE_new = gE + out
        out = gE_new.clone()
    return dict(segs=segs, V=Vs, P_local=Pls, P_sum=P_sum, norms=norms, rows=rows, X=Xs,
                values=vals, values_sum=vsum, out=out, E_new=E_new, gE_new=gE_new)
