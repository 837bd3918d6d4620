"""Encode-kernel time for small buckets (diagnostic): arctopk_encode alone, back to back.

    python scripts/encode_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.bucket import bucket_numel  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402

SETS = {
    "r18_b0": [[10], [10, 512], [512], [512]],
    "fc_only": [[10, 512]],
    "bn_only": [[512], [512]],
    "conv3x3": [[512, 512, 3, 3]],
    "conv1x1": [[512, 256, 1, 1]],
}


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    for name, shapes in SETS.items():
        shapes = [tuple(x) for x in shapes]
        plan = BucketPlan(shapes, 4, 0.2, torch.float32, dev)
        n = bucket_numel(shapes)
        G = torch.randn(n, device=dev)
        E = torch.randn(n, device=dev)
        V = plan.V_ring[0]
        V.normal_()
        for ef, ein in ((N.EF_NONE, 1), (N.EF14, 1)):
            f = lambda: plan.encode(G, E, ef, bool(ein), V, s)  # noqa: E731
            for _ in range(5):
                f()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(50):
                f()
            b.record()
            torch.cuda.synchronize()
            t_solo = a.elapsed_time(b) / 50 * 1e3
            # after a kernel that leaves 32 MiB of dirty lines (plain stores), timed alone
            dirty = torch.empty(8 << 20, device=dev)
            tot = 0.0
            for i in range(20):
                dirty.fill_(float(i))
                a.record()
                f()
                b.record()
                torch.cuda.synchronize()
                tot += a.elapsed_time(b)
            print(f"{name:8s} n={n:9d} ef={ef}: encode {t_solo:7.2f} us back to back, "
                  f"{tot / 20 * 1e3:7.2f} us after a 32 MiB fill")


if __name__ == "__main__":
    main()
