"""Helpers for device-vs-oracle parity checks (test infrastructure)."""
from __future__ import annotations

import os
import socket
import tempfile

import torch
import torch.distributed as dist


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rendezvous() -> str:
    """A file:// rendezvous for a new process group: no TCP port to race for (a port from
    free_port() can be taken by another process before the store listens on it)."""
    fd, path = tempfile.mkstemp(prefix="arctopk_rdzv_")
    os.close(fd)
    os.unlink(path)  # (the FileStore creates it)
    return "file://" + path


def ensure_group(backend: str) -> None:
    """A world_size-1 process group (the hooks call torch.distributed collectives)."""
    if dist.is_initialized():
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group(backend, init_method=rendezvous(), rank=0, world_size=1)


def check_rows_tie_aware(rows, energy_ref: torch.Tensor, k: int, band: float = 0.0):
    """Selected rows vs the oracle's energies.

    ``rows`` must hold every row whose energy exceeds the k-th energy by more than
    ``band`` (relative) and nothing below it by more than ``band``; with band = 0
    this is the exact tie rule.  Returns the number of rows that differ from the
    oracle's strict-above-threshold set padded by the lowest tied rows.
    """
    rows = torch.as_tensor(rows, dtype=torch.int64).cpu()
    e = energy_ref.double().cpu()
    assert rows.numel() == k, f"{rows.numel()} rows selected, expected {k}"
    assert torch.unique(rows).numel() == k, "duplicate rows selected"
    kth = torch.topk(e, k).values.min().item()
    tol = band * abs(kth)
    must = torch.nonzero(e > kth + tol).flatten()
    allowed = e >= kth - tol
    sel = torch.zeros(e.numel(), dtype=torch.bool)
    sel[rows] = True
    missing = must[~sel[must]]
    assert missing.numel() == 0, f"rows above the threshold not selected: {missing[:10].tolist()}"
    bad = rows[~allowed[rows]]
    assert bad.numel() == 0, f"rows below the threshold selected: {bad[:10].tolist()}"
    # exact-rule expectation: strict-above plus lowest-index ties
    strict = torch.nonzero(e > kth).flatten()
    ties = torch.nonzero(e == kth).flatten()
    expect = torch.cat([strict, ties[: k - strict.numel()]])
    es = torch.zeros(e.numel(), dtype=torch.bool)
    es[expect] = True
    return int((sel != es).sum().item()) // 2


def assert_bitwise(a: torch.Tensor, b: torch.Tensor, what: str):
    a = a.detach().cpu()
    b = b.detach().cpu()
    assert a.shape == b.shape, f"{what}: shape {tuple(a.shape)} vs {tuple(b.shape)}"
    if not torch.equal(a, b):
        d = (a.double() - b.double()).abs()
        i = int(torch.argmax(d))
        raise AssertionError(f"{what}: {int((a != b).sum())} elements differ, max |diff| "
                             f"{d.max().item():.3e} at {i} ({a.flatten()[i].item()} vs "
                             f"{b.flatten()[i].item()})")


def assert_close_rel(a: torch.Tensor, b: torch.Tensor, rtol: float, what: str):
    """Elementwise |a-b| <= rtol*|b| + rtol*max|b| (absolute floor for cancelling sums)."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    floor = rtol * b.abs().max().clamp_min(1e-30)
    err = (a - b).abs() - (rtol * b.abs() + floor)
    assert (err <= 0).all(), f"{what}: worst excess {err.max().item():.3e} (rtol {rtol})"


def device_randk_hash(numels, ks, seed: int, device):
    """The device RandK draw (arctopk_randk_select, indices only) as per-tensor int32 CPU
    tensors, ascending."""
    from allreducetopk_amd import _native as N
    kof = [sum(ks[:i]) for i in range(len(ks))]
    nb = int(N.lib().arctopk_sparse_workspace_bytes(len(numels), N.i64_array(numels)))
    assert nb > 0
    ws = torch.empty(nb, dtype=torch.uint8, device=device)
    buf = torch.empty(sum(ks), dtype=torch.int32, device=device)
    N.check(N.lib().arctopk_randk_select(None, len(ks), None, N.i64_array(numels), N.i64_array(ks),
                                         N.i64_array(kof), int(seed), buf.data_ptr(), None,
                                         ws.data_ptr(), N.DTYPE_CODE[torch.float32], 0,
                                         torch.cuda.current_stream(device).cuda_stream),
            "arctopk_randk_select")
    flat = buf.cpu()
    return [flat[o:o + k] for o, k in zip(kof, ks)]
