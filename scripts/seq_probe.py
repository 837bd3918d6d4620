"""Bare kernel sequences on one stream (no hook, no events) for a kernel trace: is the idle
time before encode intrinsic to the launch sequence?  GPU box only; run under rocprofv3."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402

dev = "cuda:0"
plan = BucketPlan([(2048, 2048)] * 16, 4, 0.2, torch.float32, dev)
n = plan.info.numel
G = torch.randn(n, device=dev)
E = torch.randn(n, device=dev) * 0.1
V = torch.randn(plan.info.v_len, device=dev)
sid = torch.cuda.current_stream().cuda_stream
mode = os.environ.get("SEQ", "full")
from allreducetopk_amd import _native as N  # noqa: E402
dev_ev = N.DeviceEvent()
t_ev = torch.cuda.Event()
cs = torch.cuda.Stream()
host = torch.randn(plan.info.v_len).pin_memory()
Vs = [torch.empty_like(V) for _ in range(4)]
torch.cuda.synchronize()
for it in range(60):
    plan.encode(G, E, 1, True, V, sid)
    if mode == "rec_dev":
        dev_ev.record(sid)
    elif mode == "rec_torch":
        t_ev.record()
    elif mode == "h2d_side":  # the hook's projection copy pattern, without its waits
        N.check(N.lib().arctopk_memcpy_h2d_async(Vs[it % 4].data_ptr(), host.data_ptr(),
                                                 host.numel() * 4, cs.cuda_stream), "h2d")
        t_ev.record(cs)
        t_ev.query()
    if mode != "enc":
        plan.select(1, sid)
        plan.pack(G, E, 1, sid)
        plan.decode(1, 1, None, G, sid)
torch.cuda.synchronize()
print("done", mode)
