"""Hook state base, bit accounting, compressor registry and CLI flags.

Mirrors the reference's plugin surface (comm_hooks/utils.py) name for name:
``HookState`` (:21-88), ``register_comm_hook_for_ddp_model`` (:91-140),
``add_comm_hook_args`` (:142-193), ``dtype_bits`` / ``tensor_bits`` (:196-210),
``_get_allgather_out_list`` (:9-18).  Drivers written against the reference
switch by changing the import root from ``comm_hooks`` to
``allreducetopk_amd.comm_hooks``.
"""
from __future__ import annotations

import logging

import torch
import torch.distributed as dist

logger = logging.getLogger(__name__)


def _get_allgather_out_list(all_gather_in_list, world_size):
    """One zero tensor shaped like the input per rank (ref utils.py:9-18)."""
    return [torch.zeros_like(all_gather_in_list, device=all_gather_in_list.device,
                             dtype=all_gather_in_list.dtype) for _ in range(world_size)]


class HookState:
    """Per-model hook state: iteration counter, comm accounting, momentum fields.

    Same attributes and semantics as the reference (utils.py:21-88):
    ``iter`` advances once per backward (when the last bucket, bucket 0 in DDP's
    order, is processed); ``comm_bits_this_round`` is cumulative and never reset.
    """

    def __init__(self, process_group: dist.ProcessGroup):
        self.process_group = process_group
        self.start_compress_iter = 0
        self.iter = 0
        self.total_bit_before_compression = 0
        self.total_bit_after_compression = 0
        self.compressor_name = "none compressor"
        self.compress_momentum = False
        self.param_state = None
        self.param_to_name = None
        self.beta1 = None
        self.adam_freeze_key = False
        self.comm_bits_this_round = 0

    def init_momentum_field(self, param_state, beta1):
        self.param_state = param_state
        self.beta1 = beta1
        self.compress_momentum = True

    def maybe_accumulate_momentum_on_bucket(self, bucket):
        if not self.compress_momentum:
            return
        if self.iter >= self.start_compress_iter and not self.adam_freeze_key:
            self.adam_freeze_key = True
            logger.info("Freeze the second momentum of Adam optimizer after %s(included) steps",
                        self.iter)
        if self.adam_freeze_key:
            self.accumulate_momentum_on_bucket(bucket)

    def accumulate_momentum_on_bucket(self, bucket):
        """grad <- (1 - beta1) * grad + beta1 * exp_avg, in place (ref utils.py:54-65)."""
        if not self.compress_momentum:
            raise RuntimeError("Momentum compression is not enabled!")
        if self.param_state is None:
            raise RuntimeError("Parameter state is not initialized!")
        parameters, gradients = bucket.parameters(), bucket.gradients()
        assert len(parameters) == len(gradients), \
            "The number of parameters and gradients should be the same."
        for p, grad in zip(parameters, gradients):
            st = self.param_state[p]
            grad.mul_(1 - self.beta1).add_(st["exp_avg"], alpha=self.beta1)

    def maybe_increase_iter(self, bucket):
        """Advance ``iter`` when the last bucket of a backward is processed (ref :67-75)."""
        if bucket.is_last():
            self.iter += 1
            if self.iter == self.start_compress_iter:
                logger.info("Start to apply %s hook after %s iterations.", self.compressor_name,
                            self.start_compress_iter)

    # -- checkpointing (not in the reference, which loses E / gE / rng on resume) --------
    _CKPT_SCALARS = ("iter", "comm_bits_this_round", "total_bit_before_compression",
                     "total_bit_after_compression", "adam_freeze_key")

    def state_dict(self) -> dict:
        """Everything a resumed run needs to continue bit-identically.

        Scalars, the seed generator's state (``rng``, when the state has one) and the
        per-bucket residuals ``error_dict`` / ``global_error_dict`` (EF14 / EF21), as
        references to the live tensors -- ``torch.save`` copies them.  Loadable with
        ``torch.load(..., weights_only=True)``.
        """
        out = {k: getattr(self, k) for k in self._CKPT_SCALARS}
        rng = self._checkpoint_rng() if hasattr(self, "_checkpoint_rng") else getattr(self, "rng", None)
        if rng is not None:
            out["rng_state"] = rng.get_state()
        for name in ("error_dict", "global_error_dict"):
            d = getattr(self, name, None)
            if d is not None:
                out[name] = {int(b): t for b, t in d.items()}
        return out

    def load_state_dict(self, sd: dict, device=None) -> None:
        """Restore :meth:`state_dict`; residuals are copied to ``device`` when given."""
        for k in self._CKPT_SCALARS:
            if k in sd:
                setattr(self, k, sd[k])
        if "rng_state" in sd:
            rng = self._checkpoint_rng() if hasattr(self, "_checkpoint_rng") else getattr(self, "rng", None)
            if rng is None:
                raise KeyError("checkpoint holds an rng state but this hook state has no rng")
            rng.set_state(sd["rng_state"])
        for name in ("error_dict", "global_error_dict"):
            if name in sd:
                setattr(self, name, {int(b): (t.to(device) if device is not None else t).clone()
                                     for b, t in sd[name].items()})
        self._after_load()

    def _after_load(self) -> None:
        """Hook for subclasses holding derived state (look-ahead seeds etc.)."""

    def compression_bits_stats(self):
        rate = (self.total_bit_before_compression / self.total_bit_after_compression
                if self.total_bit_after_compression > 0 else 0)
        return rate, self.total_bit_before_compression, self.total_bit_after_compression


def register_comm_hook_for_ddp_model(model, process_group, args, optimizer=None):
    """Build the hook state selected by ``args.compressor`` and register it on ``model``.

    Same dispatch as the reference (utils.py:91-140): ``topk_sync``/``randk_sync`` ->
    the gradual-ratio sparse hook (sparse_hook_c4), ``group_topk_no_reshape`` -> ARC-TopK,
    ``none`` -> dense all-reduce hook, ``noop`` -> no communication; anything else
    raises ``ValueError``.
    """
    hook_state = None
    if args.compressor in ("topk_sync", "randk_sync"):
        from allreducetopk_amd.comm_hooks.sparse_hook_c4 import SparseState, sparse_hook_sync
        hook_state = SparseState(
            process_group=process_group, compress_ratio=args.compress_ratio,
            sparse_type=args.sparse_type, use_error_feedback=args.use_error_feedback,
            random="randk" in args.compressor, start_compress_iter=args.start_compress_iter,
            random_seed=args.seed)
        model.register_comm_hook(hook_state, sparse_hook_sync)
    elif args.compressor == "group_topk_no_reshape":
        from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import (GroupTopKState,
                                                                              group_topk_hook)
        hook_state = GroupTopKState(
            process_group=process_group, r=args.r, use_error_feedback=args.use_error_feedback,
            seed=args.seed, start_compress_iter=args.start_compress_iter,
            compress_ratio=args.compress_ratio)
        if dist.is_available() and dist.is_initialized():
            group = process_group if process_group is not None else dist.group.WORLD
            if group.size() > 1 or hook_state.force_exchange:
                # the exchange's communicators, now, on every rank (collective)
                dev = next((p.device for p in model.parameters() if p.is_cuda), None)
                hook_state.init_exchange_comms(dev)
        hook_state._ddp_registered = True  # DDP waits on the Futures at finalize: decodes may defer
        model.register_comm_hook(hook_state, group_topk_hook)
    elif args.compressor == "noop":
        from torch.distributed.algorithms.ddp_comm_hooks.debugging_hooks import noop_hook
        model.register_comm_hook(None, noop_hook)
    elif args.compressor == "none":
        from allreducetopk_amd.comm_hooks.default_hooks import my_allreduce_hook
        hook_state = HookState(process_group)
        hook_state.start_compress_iter = args.start_compress_iter
        model.register_comm_hook(hook_state, my_allreduce_hook)
    else:
        raise ValueError(f"Compressor {args.compressor} not supported.")
    if hasattr(hook_state, "param_to_name"):
        hook_state.param_to_name = {param: name for name, param in model.named_parameters()}
    return hook_state


def add_comm_hook_args(parser):
    """The reference's compressor flags, same names, types, defaults (utils.py:142-193)."""
    parser.add_argument("--compressor", type=str, default="none",
                        help="Set the compressor to use.")
    parser.add_argument("--start_compress_iter", type=int, default=10,
                        help="Set the iteration to start compression.")
    parser.add_argument("--use_error_feedback", type=str, default="noef",
                        choices=["noef", "ef14", "ef21"], help="Set the error feedback to use.")
    parser.add_argument("--sparse_type", type=str, default="tensor",
                        choices=["row", "column", "tensor"],
                        help="Set the type of top-k sparsification to use.")
    parser.add_argument("--compress_ratio", type=float, default=0.08,
                        help="Set the ratio of the top-k elements to keep.")
    parser.add_argument("--r", type=int, default=4, help="num of cols after projection.")
    parser.add_argument("--check_grad", action="store_true", default=False,
                        help="Whether to check the identity of the gradients.")


def dtype_bits(tensor) -> int:
    """Bits per element (ref utils.py:196-207)."""
    dtype = tensor.dtype if isinstance(tensor, torch.Tensor) else tensor
    if dtype.is_floating_point:
        return torch.finfo(dtype).bits
    if dtype.is_complex:
        return torch.finfo(dtype).bits * 2
    if dtype == torch.bool:
        return 1
    if "int" in str(dtype):
        return torch.iinfo(dtype).bits
    raise ValueError(f"Unsupported dtype: {dtype}")


def tensor_bits(tensor) -> int:
    return tensor.numel() * dtype_bits(tensor)
