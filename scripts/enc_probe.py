"""Encode-kernel time per sub-bucket (GPU box): which tensor classes of a workload are
slow.  Prints device us and effective GB/s (EF14: 12 B/element + sketch)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.bucket import bucket_numel  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402

dev = "cuda:0"
s = torch.cuda.current_stream().cuda_stream
CASES = {
    "headline 16x[2048,2048]": [[2048, 2048]] * 16,
    "1x[2048,2048]": [[2048, 2048]],
    "4x[2048,2048]": [[2048, 2048]] * 4,
    "[5632,2048]": [[5632, 2048]],
    "2x[5632,2048]": [[5632, 2048]] * 2,
    "[2048,5632] (split V)": [[2048, 5632]],
    "llama layer": [[2048], [5632, 2048], [2048, 5632], [5632, 2048], [2048]] + [[2048, 2048]] * 4 + [[2048]],
    "llama layer no 1-D": [[5632, 2048], [2048, 5632], [5632, 2048]] + [[2048, 2048]] * 4,
    "[2048]+15x[2048,2048]": [[2048]] + [[2048, 2048]] * 15,
    "[32000,2048]": [[32000, 2048]],
}
only = os.environ.get("CASES")
res = {}
for name, shapes in CASES.items():
    if only and not any(o in name for o in only.split(",")):
        continue
    plan = BucketPlan([tuple(x) for x in shapes], 4, 0.2, torch.float32, dev)
    n = plan.info.numel
    G = torch.randn(n, device=dev)
    E = torch.randn(n, device=dev)
    V = torch.randn(max(1, plan.info.v_len), device=dev)
    plan.encode(G, E, N.EF14, True, V, s)
    torch.cuda.synchronize()
    ts = []
    for _ in range(15):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        plan.encode(G, E, N.EF14, True, V, s)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    us = statistics.median(ts)
    print(f"{os.environ.get('TAG', ''):10s} {name:28s} numel {n / 1e6:7.2f}M  {us:8.1f} us  {12 * n / us / 1e3:8.1f} GB/s", flush=True)
    del G, E, V, plan
    torch.cuda.empty_cache()
