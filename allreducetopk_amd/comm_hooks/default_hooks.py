"""Dense all-reduce hooks (warm-up path of the compressors; compressor ``none``).

Mirrors comm_hooks/default_hooks.py of the reference: divide by world size
first, then an async SUM all-reduce (RCCL on ROCm) whose future yields the
bucket (:15-35).
"""

import torch
import torch.distributed as dist

from allreducetopk_amd.comm_hooks.utils import HookState, tensor_bits

__all__ = ["allreduce_hook", "my_allreduce_hook"]


def _allreduce_fut(process_group: dist.ProcessGroup, tensor: torch.Tensor,
                   hook_state=None) -> torch.futures.Future[torch.Tensor]:
    """Average ``tensor`` across the group; returns a Future of it (ref :15-35)."""
    group = process_group if process_group is not None else dist.group.WORLD
    world_size = group.size()
    tensor.div_(world_size)  # divide first (fp16 overflow guard), as the reference
    if hook_state is not None:
        hook_state.comm_bits_this_round += 2 * (world_size - 1) * tensor_bits(tensor)
    return dist.all_reduce(tensor, group=group, async_op=True).get_future().then(
        lambda fut: fut.value()[0])


def my_allreduce_hook(state: HookState, bucket: dist.GradBucket
                      ) -> torch.futures.Future[torch.Tensor]:
    state.maybe_accumulate_momentum_on_bucket(bucket)
    state.maybe_increase_iter(bucket)
    return _allreduce_fut(state.process_group, bucket.buffer(), state)


def allreduce_hook(process_group: dist.ProcessGroup, bucket: dist.GradBucket
                   ) -> torch.futures.Future[torch.Tensor]:
    return _allreduce_fut(process_group, bucket.buffer())
