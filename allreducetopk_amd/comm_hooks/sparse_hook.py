"""TopK / RandK DDP comm hooks on MI355X -- drop-in for the reference's
comm_hooks/sparse_hook.py (``SparseState`` :127-160, ``cal_k`` :77-78,
``sparse_hook_sync`` :163-304).

Per bucket call (all on the caller's stream, no host synchronisation):

    ef_apply        (EF14: x += E, E = x | EF21: x -= E), one fused pass
    TopK : topk_select  exact element top-k of |x| per tensor (radix select),
                        ascending int32 indices + gathered values
    RandK: indices      torch.randperm(numel, device)[:k] after the shared reseed
                        (index_source="torch": the reference's own draw on a GPU), the
                        same draw on the CPU generator (index_source="host": the reference
                        run on CPU, as the golden vectors were made), then gather; or
                        (index_source="hash", perf mode) the k largest keyed-hash keys per
                        tensor -- a uniform k-subset -- through the TopK radix select:
                        ascending indices, gather (and EF14's E[idx] = 0) in its last pass
    residual        EF14: E[idx] = 0 | EF21: E[idx] += values
    RandK: all_reduce(values)              -> decode: zero + scatter(values / ws)
                                              (hash: one pass over whole chunks)
    TopK : all_gather(values), all_gather(indices)
                                           -> decode: zero + rank-ordered scatter-add, / ws
    EF21: gE += out; out = gE (fused into decode)

Only ``sparse_type="tensor"`` works in the reference (row/column unpack 2 values
where 3 are expected, :54, :75, :96); the same types raise here.
Ties at the k-th |x| resolve lowest-index first.
"""

import logging
from typing import Dict, List

import torch
import torch.distributed as dist

from allreducetopk_amd import _native as N
from allreducetopk_amd.comm_hooks import default_hooks
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import _residual_on
from allreducetopk_amd.comm_hooks.utils import (HookState, _get_allgather_out_list, dtype_bits,
                                                tensor_bits)

logger = logging.getLogger(__name__)

__all__ = ["SparseState", "sparse_hook_sync", "cal_k"]


def cal_k(tensor, compress_ratio):
    """k of a tensor (ref sparse_hook.py:77-78)."""
    return max(1, int(tensor.numel() * compress_ratio))


class SparseState(HookState):
    """State of the TopK/RandK hook (reference sparse_hook.py:127-160)."""

    def __init__(self, process_group: dist.ProcessGroup, compress_ratio: float = 0.01,
                 start_compress_iter: int = 2, sparse_type: str = "row", random: bool = False,
                 use_error_feedback: str = "noef", random_seed: int = 0,
                 index_source: str = "torch"):
        super().__init__(process_group)
        self.total_bit_before_compression = 0
        self.total_bit_after_compression = 0
        self.compress_ratio = compress_ratio
        self.iter = 0
        self.start_compress_iter = start_compress_iter
        self.error_decay = 1.0
        self.large_batch_init = False
        self.sparse_type = sparse_type
        self.compressor_name = f"{sparse_type}-wise sparsification"
        self.random = random
        self.rng = torch.Generator()
        self.rng.manual_seed(random_seed)
        self.use_error_feedback = use_error_feedback
        self.error_dict: Dict[int, torch.Tensor] = {}
        self.global_error_dict: Dict[int, torch.Tensor] = {}
        self.random_seed = random_seed
        if index_source not in ("torch", "host", "hash"):
            raise ValueError("index_source must be 'torch', 'host' or 'hash'")
        self.index_source = index_source
        self._workspace = None
        self._ws_bytes: Dict[tuple, int] = {}
        self._fold_in = None  # RandK "hash" under EF14: the select applies E (1) or the first-call copy (2)

    # ratio of this call; the c4 variant overrides (gradual compression)
    def _call_ratio(self) -> float:
        return self.compress_ratio

    def _on_compression_start(self):
        pass


def _workspace(state, device, numels) -> torch.Tensor:
    """Select workspace for this bucket's tensor sizes (grown, never shrunk)."""
    key = tuple(numels)
    nbytes = state._ws_bytes.get(key)
    if nbytes is None:
        nbytes = int(N.lib().arctopk_sparse_workspace_bytes(len(numels), N.i64_array(numels)))
        if nbytes < 0:
            N.check(-nbytes, "arctopk_sparse_workspace_bytes")
        state._ws_bytes[key] = nbytes
    ws = state._workspace
    if ws is None or ws.device != device or ws.numel() < nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        state._workspace = ws
    return ws


def _sparse_hook_impl(state: SparseState, bucket, c4: bool = False) -> "torch.futures.Future[torch.Tensor]":
    if state.use_error_feedback == "ef21" and state.large_batch_init:
        # (sparse_hook.py:172-175, sparse_hook_c4.py:201-204)
        if state.iter < state.start_compress_iter:
            logger.info("Using large batch initialization in EF21!!")
        return _large_batch_ef21(state, bucket, c4)
    state.maybe_accumulate_momentum_on_bucket(bucket)
    group = state.process_group if state.process_group is not None else dist.group.WORLD
    world_size = group.size()
    input_tensor = bucket.buffer()

    if state.iter < state.start_compress_iter:  # (:190-193)
        state.maybe_increase_iter(bucket)
        return default_hooks._allreduce_fut(group, input_tensor, state)

    state._on_compression_start()
    _check_compressible(state, input_tensor)
    L = N.lib()
    device = input_tensor.device
    dtype = input_tensor.dtype
    b = bucket.index()
    total = input_tensor.shape[0]
    stream = torch.cuda.current_stream(device).cuda_stream
    ef = N.EF_CODE[state.use_error_feedback]
    dt = N.DTYPE_CODE[dtype]
    # EF21 residual scaling: E += error_decay * C(D), gE += error_decay * out (:265, :296)
    decay = float(state.error_decay)

    if ef == N.EF14:
        err_in = b in state.error_dict
        if not err_in:
            logger.info("A zero tensor of length %s that represents local error is created.", total)
            state.error_dict[b] = torch.zeros(total, device=device, dtype=dtype)
        err = _residual_on(state.error_dict, b, input_tensor, "error_dict")
        # E := G + E (:205, :258); selection and gathers then read the pre-compression bucket
        # from E, and the decode writes the bucket once.  RandK's device draw folds E itself in
        # its write pass (arctopk_randk_select_ef14: its keys never read the data)
        # (and fp32 TopK folds it in its first pass: arctopk_topk_select_ef14)
        if not _select_folds(state, dtype):
            N.check(L.arctopk_ef14_fold(input_tensor.data_ptr(), err.data_ptr(), total, int(err_in),
                                        dt, stream), "arctopk_ef14_fold")
        state._fold_in = int(err_in)
    elif ef == N.EF21:
        if b in state.error_dict:
            err = _residual_on(state.error_dict, b, input_tensor, "error_dict")
            _residual_on(state.global_error_dict, b, input_tensor, "global_error_dict")
            N.check(L.arctopk_ef_apply(input_tensor.data_ptr(), err.data_ptr(),
                                       total, N.EF21, 1, dt, stream), "arctopk_ef_apply")
        else:  # (:213-226)
            logger.info("A tensor of length %s that represents local/global error is created.", total)
            state.error_dict[b] = torch.clone(input_tensor).detach()
            dist.all_reduce(input_tensor, group=group, async_op=False)
            input_tensor.div_(world_size)
            state.global_error_dict[b] = torch.clone(input_tensor).detach()
            state.maybe_increase_iter(bucket)
            fut = torch.futures.Future()
            fut.set_result(input_tensor)
            return fut

    if ef != N.EF14 or not _select_folds(state, dtype):
        state._fold_in = None  # (set above only when the select folds E itself)
    seed = None
    if state.random:  # shared reseed so every rank draws the same indices (:230-235)
        seed = torch.randint(0, 1_000_000_000, (1,), generator=state.rng).item()
        torch.manual_seed(seed)
    _compress_exchange(state, bucket, group, world_size, ef, state._call_ratio(), seed,
                       e_decay=decay, g_decay=decay, count_bits=True)
    state.maybe_increase_iter(bucket)
    fut = torch.futures.Future()
    fut.set_result(input_tensor)
    return fut


def _select_folds(state: SparseState, dtype) -> bool:
    """EF14's E := G + E is applied by the select itself (RandK's device draw: in its write pass;
    fp32 TopK: in its first histogram pass), not by a fold pass of its own."""
    if state.random:
        return state.index_source == "hash"
    return dtype == torch.float32


def _check_compressible(state: SparseState, input_tensor: torch.Tensor) -> None:
    if state.sparse_type != "tensor":  # the reference crashes for row/column (:96)
        raise ValueError(f"not enough values to unpack (sparse_type={state.sparse_type!r}: only "
                         "'tensor' is functional in the reference)")
    if not input_tensor.is_cuda or input_tensor.dtype not in N.DTYPE_CODE:
        raise RuntimeError("sparse HIP codec needs a float32 or bfloat16 bucket on a GPU")


def _compress_exchange(state: SparseState, bucket, group, world_size: int, ef: int, ratio: float,
                       seed, e_decay: float, g_decay: float, count_bits: bool, on_values=None) -> None:
    """The compressed call after the EF pre-apply, on the caller's stream: select (TopK) or draw
    (RandK) the indices, gather the values, persist the residual (EF14: E[idx] = 0; EF21:
    E[idx] += e_decay * values), exchange (RandK: all-reduce; TopK: all-gather of values and
    indices) and decode into the bucket (EF21: gE += g_decay * out, out = gE).
    Reference: sparse_hook.py:237-297 (and :363-410 for the large-batch hook)."""
    L = N.lib()
    input_tensor = bucket.buffer()
    tensors = bucket.gradients()
    device = input_tensor.device
    dtype = input_tensor.dtype
    b = bucket.index()
    total = input_tensor.shape[0]
    stream = torch.cuda.current_stream(device).cuda_stream
    dt = N.DTYPE_CODE[dtype]
    numels = [t.numel() for t in tensors]
    ks = [max(1, int(n * ratio)) for n in numels]
    offsets: List[int] = []
    off = 0
    for t in tensors:
        if (t.data_ptr() - input_tensor.data_ptr()) // input_tensor.element_size() != off:
            raise RuntimeError("bucket gradient views must tile the buffer in order")
        offsets.append(off)
        off += t.numel()
    k_off: List[int] = []
    acc = 0
    for k in ks:
        k_off.append(acc)
        acc += k
    sum_k = acc
    nt = len(tensors)
    fold14 = ef == N.EF14  # the pre-compression bucket lives in E (arctopk_ef14_fold)
    a_off, a_n, a_k, a_ko = (N.i64_array(offsets), N.i64_array(numels), N.i64_array(ks),
                             N.i64_array(k_off))
    values = torch.empty(sum_k, dtype=dtype, device=device)
    indices = torch.empty(sum_k, dtype=torch.int32, device=device)
    x = input_tensor.data_ptr()
    xsrc = state.error_dict[b].data_ptr() if fold14 else x
    if state.random:
        if state.index_source == "torch":  # the reference's own draw (:20), per tensor in order
            for t, k, ko in zip(tensors, ks, k_off):
                indices[ko:ko + k].copy_(torch.randperm(t.numel(), device=device)[:k])
        elif state.index_source == "host":
            # parity mode: the reference run on CPU (sparse_hook_c4.py:20 with CPU tensors, after
            # the reseed at :269-274) draws from the CPU generator; the same draws, in tensor
            # order (so the generator is left where the reference leaves it), copied to the GPU
            host = torch.empty(sum_k, dtype=torch.int32)
            for t, k, ko in zip(tensors, ks, k_off):
                host[ko:ko + k].copy_(torch.randperm(t.numel())[:k])
            indices.copy_(host)
        elif fold14 and state._fold_in is not None:
            # "hash" under EF14: the draw, with the fold E := G + E (:205), the gather and
            # `E[indices] = 0` (:104) all in the select's last pass
            ws_buf = _workspace(state, device, numels)
            N.check(L.arctopk_randk_select_ef14(x, state.error_dict[b].data_ptr(), state._fold_in, nt, a_off,
                                                a_n, a_k, a_ko, int(seed), indices.data_ptr(), values.data_ptr(),
                                                ws_buf.data_ptr(), dt, stream), "arctopk_randk_select_ef14")
        else:  # "hash": the k largest keyed-hash keys per tensor, ascending, gathered in the select;
            # EF14's `E[indices] = 0` (:104) happens in its last pass, as for TopK
            ws_buf = _workspace(state, device, numels)
            N.check(L.arctopk_randk_select(xsrc, nt, a_off, a_n, a_k, a_ko, int(seed), indices.data_ptr(),
                                           values.data_ptr(), ws_buf.data_ptr(), dt, int(fold14), stream),
                    "arctopk_randk_select")
        if state.index_source != "hash":
            N.check(L.arctopk_sparse_gather(xsrc, nt, a_off, a_k, a_ko, indices.data_ptr(),
                                            values.data_ptr(), dt, stream), "arctopk_sparse_gather")
        bits_sum = sum_k * dtype_bits(dtype)
    else:
        ws_buf = _workspace(state, device, numels)
        rc = N.EINVAL
        if fold14 and state._fold_in is not None:  # E := G + E (:205) in the select's first pass
            rc = L.arctopk_topk_select_ef14(x, xsrc, state._fold_in, nt, a_off, a_n, a_k, a_ko,
                                            indices.data_ptr(), values.data_ptr(), ws_buf.data_ptr(), dt, stream)
            if rc == N.EINVAL:  # (a tensor not 16-B aligned / of numel % 4 != 0): fold, then select
                N.check(L.arctopk_ef14_fold(x, xsrc, total, state._fold_in, dt, stream), "arctopk_ef14_fold")
            else:
                N.check(rc, "arctopk_topk_select_ef14")
        if rc == N.EINVAL:
            # EF14: the residual's `E[indices] = 0` (:104) happens in the select's last pass
            N.check(L.arctopk_topk_select(xsrc, nt, a_off, a_n, a_k, a_ko, indices.data_ptr(),
                                          values.data_ptr(), ws_buf.data_ptr(), dt, int(fold14), stream),
                    "arctopk_topk_select")
        bits_sum = sum_k * (dtype_bits(dtype) + 32)

    # the call's selection, for inspection and tests (int32 indices per tensor, concatenated
    # in bucket order at the k offsets; TopK: ascending within a tensor)
    state.last_indices, state.last_k = indices, ks
    if on_values is not None:
        on_values(values)
    fused_residual = fold14 and (not state.random or state.index_source == "hash")
    if ef != N.EF_NONE and not fused_residual:  # residual persistence (:257-267)
        N.check(L.arctopk_sparse_residual(state.error_dict[b].data_ptr(), nt, a_off, a_k, a_ko,
                                          indices.data_ptr(), values.data_ptr(), ef, e_decay, dt, stream),
                "arctopk_sparse_residual")
    gerr = state.global_error_dict[b].data_ptr() if ef == N.EF21 else None

    if state.random:
        if count_bits:
            state.comm_bits_this_round += 2 * (world_size - 1) * bits_sum
        if world_size > 1:
            dist.all_reduce(values, group=group, async_op=False)
        ascending = 2 if state.index_source == "hash" else 0  # one pass of whole chunks
        N.check(L.arctopk_sparse_decode(x, total, nt, a_off, a_k, a_ko, sum_k, indices.data_ptr(),
                                        values.data_ptr(), 1, world_size, ascending, gerr, g_decay, dt,
                                        stream),
                "arctopk_sparse_decode")
    else:
        if count_bits:
            state.comm_bits_this_round += (world_size - 1) * world_size * bits_sum
        if world_size > 1:
            all_vals = torch.empty(world_size * sum_k, dtype=dtype, device=device)
            all_idx = torch.empty(world_size * sum_k, dtype=torch.int32, device=device)
            _all_gather_flat(all_vals, values, group, world_size)
            _all_gather_flat(all_idx, indices, group, world_size)
        else:  # gathering from one rank is the identity
            all_vals, all_idx = values, indices
        N.check(L.arctopk_sparse_decode(x, total, nt, a_off, a_k, a_ko, sum_k, all_idx.data_ptr(),
                                        all_vals.data_ptr(), world_size, world_size, 1, gerr,
                                        g_decay, dt, stream), "arctopk_sparse_decode")


def _large_batch_ef21(state: SparseState, bucket, c4: bool) -> "torch.futures.Future[torch.Tensor]":
    """EF21 with large-batch initialisation (reference sparse_hook.py:307-416; the registered
    copy sparse_hook_c4.py:353-457), reached when ``state.large_batch_init`` is set by hand:

    - iteration 0: the reference calls ``default_hooks._allreduce_fut`` without its required
      ``hook_state`` argument, so it raises TypeError (after advancing ``iter``); so does this;
    - 1 <= iter < start_compress_iter: E += G; the bucket is all-reduced and averaged; gE += it;
    - iter == start_compress_iter: E and gE are divided by start_compress_iter - 1;
    - compressed calls: D = G - E, C(D) at ``compress_ratio`` (never the gradual ratio),
      E += C(D) (alpha 1), the exchange, gE += error_decay * out, out = gE.  No communication
      bits are counted (the reference counts none in this hook).  The registered copy then
      fails in the reference (its ``cal_k(state, tensor)`` is called as ``cal_k(tensor,
      ratio)``: AttributeError, sparse_hook_c4.py:421); with ``c4`` so does this, at the same
      point (after the residual division, the pre-apply and the reseed)."""
    assert state.use_error_feedback == "ef21", "This hook is only for EF21"
    assert state.large_batch_init, "This hook is only for large batch initialization"
    state.maybe_accumulate_momentum_on_bucket(bucket)
    group = state.process_group if state.process_group is not None else dist.group.WORLD
    world_size = group.size()
    input_tensor = bucket.buffer()
    b = bucket.index()
    total = input_tensor.shape[0]
    if state.iter < 1:
        state.maybe_increase_iter(bucket)
        raise TypeError("_allreduce_fut() missing 1 required positional argument: 'hook_state'")
    if state.iter < state.start_compress_iter:
        if b not in state.error_dict:
            logger.info("A tensor of length %s that represents local/global error is created.", total)
            state.error_dict[b] = torch.zeros(total, device=input_tensor.device, dtype=input_tensor.dtype)
            state.global_error_dict[b] = torch.zeros(total, device=input_tensor.device, dtype=input_tensor.dtype)
        state.error_dict[b].add_(input_tensor, alpha=1.0)
        dist.all_reduce(input_tensor, group=group, async_op=False)
        input_tensor.div_(world_size)
        state.global_error_dict[b].add_(input_tensor, alpha=1.0)
        state.maybe_increase_iter(bucket)
        fut = torch.futures.Future()
        fut.set_result(input_tensor)
        return fut
    if state.iter == state.start_compress_iter:
        state.error_dict[b].div_(state.start_compress_iter - 1)
        state.global_error_dict[b].div_(state.start_compress_iter - 1)
    _check_compressible(state, input_tensor)
    err = _residual_on(state.error_dict, b, input_tensor, "error_dict")
    _residual_on(state.global_error_dict, b, input_tensor, "global_error_dict")
    L = N.lib()
    stream = torch.cuda.current_stream(input_tensor.device).cuda_stream
    N.check(L.arctopk_ef_apply(input_tensor.data_ptr(), err.data_ptr(), total, N.EF21, 1,
                               N.DTYPE_CODE[input_tensor.dtype], stream), "arctopk_ef_apply")
    seed = None
    if state.random:
        seed = torch.randint(0, 1_000_000_000, (1,), generator=state.rng).item()
        torch.manual_seed(seed)
    if c4:
        raise AttributeError("'Tensor' object has no attribute 'get_current_compress_ratio'")
    log_diff = bucket.is_last() and dist.get_rank() == 0 and logger.isEnabledFor(logging.INFO)
    sq = [None]
    if log_diff:  # |D - C(D)| = sqrt(|D|^2 - |values|^2): only computed when the log is on
        dn = input_tensor.float().pow(2).sum()
        sq[0] = lambda v: float((dn - v.float().pow(2).sum()).clamp_min(0).sqrt())
    vals_seen = []
    _compress_exchange(state, bucket, group, world_size, N.EF21, state.compress_ratio, seed,
                       e_decay=1.0, g_decay=float(state.error_decay), count_bits=False,
                       on_values=vals_seen.append if log_diff else None)
    if log_diff:
        logger.info(f"Rank[{dist.get_rank()}] Iter[{state.iter}], Diff error{sq[0](vals_seen[0])}")
    state.maybe_increase_iter(bucket)
    fut = torch.futures.Future()
    fut.set_result(input_tensor)
    return fut


def _all_gather_flat(out: torch.Tensor, inp: torch.Tensor, group, world_size: int) -> None:
    try:
        dist.all_gather_into_tensor(out, inp, group=group, async_op=False)
    except (RuntimeError, NotImplementedError, AttributeError):  # backends without the flat form
        parts = _get_allgather_out_list(inp, world_size)
        dist.all_gather(parts, inp, group=group, async_op=False)
        torch.cat(parts, out=out)


def sparse_hook_sync(state: SparseState, bucket: dist.GradBucket
                     ) -> torch.futures.Future[torch.Tensor]:
    return _sparse_hook_impl(state, bucket)


# bits helpers kept for drivers that import them from here
__all__ += ["tensor_bits", "dtype_bits"]
