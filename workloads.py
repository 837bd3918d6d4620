"""Bucket shape sets of the BASELINE configs (bench.py workloads; tests/ parity cases).

SURVEY.md section 8(d): the headline bucket (16 x [2048, 2048] fp32, the Llama-1B projection
shape) and the real DDP buckets of configs[1]-[4] (parameter shapes from the reference's
model definitions: cifar10/resnet.py, c4/configs/llama_1b.json, roberta-base).
"""
from __future__ import annotations

from allreducetopk_amd.bucket import bucket_numel

HEADLINE = [[2048, 2048]] * 16
# secondary buckets: real DDP bucket shapes of the BASELINE configs
WORKLOADS = {
    "headline": ("bucket_16x2048x2048_fp32_256MiB", HEADLINE),
    "llama_embed": ("bucket_llama1b_embed_32000x2048_fp32_250MiB", [[32000, 2048]]),
    "roberta_embed": ("bucket_roberta_embed_50265x768_fp32_147MiB", [[50265, 768]]),
    "resnet18_conv": ("bucket_28x512x512x3x3_fp32_252MiB", [[512, 512, 3, 3]] * 28),
    "resnet50_mixed": ("bucket_resnet50_stage4_mixed_fp32",
                       [[2048], [2048], [2048, 512, 1, 1], [512], [512], [512, 512, 3, 3], [512],
                        [512], [512, 2048, 1, 1]] * 3 + [[2048, 1024, 1, 1]]),
    "llama_layer_mixed": ("bucket_llama1b_layer_mixed_1d_fp32",
                          [[2048], [5632, 2048], [2048, 5632], [5632, 2048], [2048]]
                          + [[2048, 2048]] * 4 + [[2048]]),
}


def resnet18_cifar_shapes():
    """Parameter shapes of the CIFAR ResNet-18 of configs[1] in definition order (the
    reference's cifar10/resnet.py: 3x3 stem, BasicBlock [2, 2, 2, 2], 1x1 shortcuts,
    BatchNorm weight + bias, Linear(512, 10)); 62 tensors, 11.17 M parameters."""
    shapes = [[64, 3, 3, 3], [64], [64]]
    cin = 64
    for planes, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
        for b in range(2):
            s_ = stride if b == 0 else 1
            shapes += [[planes, cin, 3, 3], [planes], [planes], [planes, planes, 3, 3], [planes], [planes]]
            if s_ != 1 or cin != planes:
                shapes += [[planes, cin, 1, 1], [planes], [planes]]
            cin = planes
    return shapes + [[10, 512], [10]]


def resnet50_cifar_shapes(num_classes=100):
    """Parameter shapes of the CIFAR-100 ResNet-50 of configs[3] in definition order (the
    reference's cifar10/resnet.py:40-112 Bottleneck [3, 4, 6, 3]: 1x1 -> 3x3 -> 1x1 (x4), each
    conv followed by BatchNorm weight + bias, a 1x1 conv + BN shortcut on each layer's first
    block; run_cifar100_resnet50.py:155 ResNet50(num_classes=100)); 161 tensors, 23.71 M
    parameters."""
    shapes = [[64, 3, 3, 3], [64], [64]]
    cin = 64
    for planes, nblocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(nblocks):
            s_ = stride if b == 0 else 1
            shapes += [[planes, cin, 1, 1], [planes], [planes], [planes, planes, 3, 3], [planes], [planes],
                       [4 * planes, planes, 1, 1], [4 * planes], [4 * planes]]
            if s_ != 1 or cin != 4 * planes:
                shapes += [[4 * planes, cin, 1, 1], [4 * planes], [4 * planes]]
            cin = 4 * planes
    return shapes + [[num_classes, 2048], [num_classes]]


def ddp_buckets(shapes, first_cap=1 << 20, cap=25 << 20, elem_bytes=4):
    """DDP's bucketing as the Reducer sees it: parameters in reverse definition order (the
    order gradients become ready), a first bucket of <= 1 MiB, then <= 25 MiB buckets
    (DistributedDataParallel defaults; a tensor larger than the cap gets its own bucket)."""
    out, cur, size = [], [], 0
    for s_ in reversed(shapes):
        nbytes = elem_bytes * bucket_numel([s_])
        limit = first_cap if not out else cap
        if cur and size + nbytes > limit:
            out.append(cur)
            cur, size = [], 0
        cur.append(s_)
        size += nbytes
    if cur:
        out.append(cur)
    return out


# whole models as their DDP buckets (bench.py --workload; one step = one backward's buckets)
DDP_MODELS = {
    "resnet18_ddp": ("resnet18_cifar_ddp_buckets_fp32_44.7MB", resnet18_cifar_shapes),      # configs[1]
    "resnet50_ddp": ("resnet50_cifar100_ddp_buckets_fp32_94.8MB", resnet50_cifar_shapes),   # configs[3]
}
