"""TopK / RandK hooks with gradual compression -- drop-in for the reference's
comm_hooks/sparse_hook_c4.py, the copy its registry actually registers for
``topk_sync`` / ``randk_sync`` (comm_hooks/utils.py:94).

Differences from ``sparse_hook`` (reference sparse_hook_c4.py:140-151, :175-189,
:224-237, :287): ``gradual_compression`` (default True) ramps the ratio from 0.8
down to ``compress_ratio`` over ``start_compress_iter + warmup_iters`` iterations
after compression starts, and ``cal_k`` takes ``(state, tensor)``.
"""

import logging

import torch
import torch.distributed as dist

from allreducetopk_amd.comm_hooks import sparse_hook as _base

logger = logging.getLogger(__name__)

__all__ = ["SparseState", "sparse_hook_sync", "cal_k"]


class SparseState(_base.SparseState):
    def __init__(self, process_group: dist.ProcessGroup, compress_ratio: float = 0.01,
                 start_compress_iter: int = 2, sparse_type: str = "row", random: bool = False,
                 use_error_feedback: str = "noef", random_seed: int = 0,
                 gradual_compression=True, warmup_iters=100, index_source: str = "torch"):
        super().__init__(process_group, compress_ratio=compress_ratio,
                         start_compress_iter=start_compress_iter, sparse_type=sparse_type,
                         random=random, use_error_feedback=use_error_feedback,
                         random_seed=random_seed, index_source=index_source)
        self.base_compress_ratio = compress_ratio
        self.gradual_compression = gradual_compression
        # note: the ramp spans start_compress_iter + warmup_iters iterations (ref :151)
        self.warmup_iters = start_compress_iter + warmup_iters
        self.compression_started = False

    def get_current_compress_ratio(self):
        """0.8 -> base ratio, linear in iterations since compression started (ref :175-189)."""
        if not self.gradual_compression or not self.compression_started:
            return self.base_compress_ratio
        progress = self.iter - self.start_compress_iter
        if progress < self.warmup_iters:
            start_ratio = 0.8
            cur = start_ratio - (start_ratio - self.base_compress_ratio) * (progress / self.warmup_iters)
            return max(cur, self.base_compress_ratio)
        return self.base_compress_ratio

    def _call_ratio(self) -> float:
        return self.get_current_compress_ratio()

    def _on_compression_start(self):
        if not self.compression_started:
            self.compression_started = True
            logger.info("Starting compression at iteration %s with gradual compression enabled: %s",
                        self.iter, self.gradual_compression)


def cal_k(state, tensor):
    return max(1, int(tensor.numel() * state.get_current_compress_ratio()))


def sparse_hook_sync(state: SparseState, bucket: dist.GradBucket
                     ) -> torch.futures.Future[torch.Tensor]:
    return _base._sparse_hook_impl(state, bucket, c4=True)
