"""PyTorch operator layer over libarctopk's C ABI (``torch.ops.arctopk.*``).

The hook itself calls the C entry points directly (one foreign call per step, see
DESIGN.md section 7).  These registrations expose the same codec phases to the PyTorch
dispatcher, so a caller can use them inside code that torch.compile traces or that is
captured in a CUDA/HIP graph: each op declares which tensors it mutates and has a fake
(meta) implementation, and it enqueues on the current stream of the tensors' device.

A plan is passed as its integer handle (``BucketPlan.handle.value``); buffers are the
plan's own (``BucketPlan.sketch`` / ``rowlist`` / ``slotmap`` / ``packed`` / ``V_ring[0]``)
or any tensors of the sizes ``BucketPlan.info`` gives.

    import allreducetopk_amd.ops  # registers torch.ops.arctopk.*
    torch.ops.arctopk.draw_projections(h, seed, V)
    torch.ops.arctopk.encode(h, grad, err, ef, True, V, sketch)
    dist.all_reduce(sketch)
    torch.ops.arctopk.select(h, sketch, ws, rowlist, slotmap)
    torch.ops.arctopk.pack(h, grad, err, ef, rowlist, slotmap, packed)
    dist.all_reduce(packed)
    torch.ops.arctopk.decode(h, packed, slotmap, ws, ef, gerr, grad)

Each op replaces the same reference code as the C entry point it calls (include/arctopk.h).
"""
from __future__ import annotations

from typing import Optional

import torch

from allreducetopk_amd import _native as N


def _stream(t: torch.Tensor) -> int:
    return torch._C._cuda_getCurrentRawStream(t.device.index or 0)


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


@torch.library.custom_op("arctopk::draw_projections", mutates_args=("V",))
def draw_projections(plan: int, seed: int, V: torch.Tensor) -> None:
    """V := the reference's torch.randn(m, r, device=...) draws after manual_seed(seed)."""
    N.check(N.lib().arctopk_draw_projections(plan, seed, V.data_ptr(), _stream(V)),
            "arctopk_draw_projections")


@torch.library.custom_op("arctopk::encode", mutates_args=("err", "sketch"))
def encode(plan: int, grad: torch.Tensor, err: Optional[torch.Tensor], ef: int, err_in: bool,
           V: torch.Tensor, sketch: torch.Tensor) -> None:
    """EF pre-apply + rank-r sketch of every tensor of the bucket (K1)."""
    N.check(N.lib().arctopk_encode(plan, grad.data_ptr(), _ptr(err), ef, int(err_in), V.data_ptr(),
                                   sketch.data_ptr(), _stream(grad)), "arctopk_encode")


@torch.library.custom_op("arctopk::select", mutates_args=("rowlist", "slotmap"))
def select(plan: int, sketch: torch.Tensor, world_size: int, rowlist: torch.Tensor,
           slotmap: torch.Tensor) -> None:
    """Mean sketch -> row energies -> exact top-k rows per tensor (K2)."""
    N.check(N.lib().arctopk_select(plan, sketch.data_ptr(), world_size, rowlist.data_ptr(),
                                   slotmap.data_ptr(), _stream(sketch)), "arctopk_select")


@torch.library.custom_op("arctopk::pack", mutates_args=("err", "packed"))
def pack(plan: int, grad: torch.Tensor, err: Optional[torch.Tensor], ef: int, rowlist: torch.Tensor,
         slotmap: torch.Tensor, packed: torch.Tensor) -> None:
    """Selected rows -> packed values; EF14 / EF21 residual updates (K3)."""
    N.check(N.lib().arctopk_pack(plan, grad.data_ptr(), _ptr(err), ef, rowlist.data_ptr(),
                                 slotmap.data_ptr(), packed.data_ptr(), _stream(grad)), "arctopk_pack")


@torch.library.custom_op("arctopk::decode", mutates_args=("gerr", "out"))
def decode(plan: int, packed: torch.Tensor, slotmap: torch.Tensor, world_size: int, ef: int,
           gerr: Optional[torch.Tensor], out: torch.Tensor) -> None:
    """Bucket := mean of the selected rows (+ EF21 global residual) (K4)."""
    N.check(N.lib().arctopk_decode(plan, packed.data_ptr(), slotmap.data_ptr(), world_size, ef,
                                   _ptr(gerr), out.data_ptr(), _stream(out)), "arctopk_decode")


# fake implementations: the ops only mutate their declared outputs
@draw_projections.register_fake
def _(plan, seed, V):
    return None


@encode.register_fake
def _(plan, grad, err, ef, err_in, V, sketch):
    return None


@select.register_fake
def _(plan, sketch, world_size, rowlist, slotmap):
    return None


@pack.register_fake
def _(plan, grad, err, ef, rowlist, slotmap, packed):
    return None


@decode.register_fake
def _(plan, packed, slotmap, world_size, ef, gerr, out):
    return None
