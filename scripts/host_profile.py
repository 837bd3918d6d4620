"""Host-side cost of one ARC-TopK hook call (cProfile + loop timings). GPU box only."""
import cProfile
import os
import pstats
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import GroupTopKState, group_topk_hook  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29511")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from workloads import WORKLOADS, ddp_buckets, resnet18_cifar_shapes  # noqa: E402
wl = os.environ.get("WORKLOAD", "headline")
layouts = ddp_buckets(resnet18_cifar_shapes()) if wl == "resnet18_ddp" else [WORKLOADS[wl][1]]
bks = [SyntheticBucket(torch.randn(bucket_numel(sh), device="cuda:0"), sh, index=i,
                       is_last=(i == len(layouts) - 1)) for i, sh in enumerate(layouts)]
st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback="ef14", seed=1)


def call_all():
    for b in bks:
        group_topk_hook(st, b)


for _ in range(5):
    call_all()
torch.cuda.synchronize()


def loop(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        call_all()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6


print("no events: host enqueue %.1f us/step, wall %.1f us/step" % loop(50))
for depth, workers in ((8, 1), (0, 1), (8, 8)):
    st._proj.close()
    st._proj.depth, st._proj._workers = depth, workers
    st._proj.reset()
    loop(5)
    print("proj depth %d workers %d: host enqueue %.1f us/step, wall %.1f us/step" % ((depth, workers) + loop(50)))
# bare launch cost: the encode entry point alone, back to back
plan = st._plan_for(bks[0])
sid = torch.cuda.current_stream().cuda_stream
err = st.error_dict[0]
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(200):
    plan.encode(bks[0].buffer(), err, 1, True, plan.V_ring[0], sid)
t1 = time.perf_counter()
torch.cuda.synchronize()
print("bare encode launch %.1f us host, %.1f us wall" % ((t1 - t) / 200 * 1e6, (time.perf_counter() - t) / 200 * 1e6))
t = time.perf_counter()
for _ in range(200):
    plan.select(1, sid)
t1 = time.perf_counter()
torch.cuda.synchronize()
print("bare select launch %.1f us host, %.1f us wall" % ((t1 - t) / 200 * 1e6, (time.perf_counter() - t) / 200 * 1e6))
st.phase_events = []
print("events   : host enqueue %.1f us/step, wall %.1f us/step" % loop(50))
st.phase_events = None
print("proj hits/misses", st._proj.hits, st._proj.misses)
# components
t = time.perf_counter()
for _ in range(200):
    torch.manual_seed(123)
print("torch.manual_seed %.1f us" % ((time.perf_counter() - t) / 200 * 1e6))
x = torch.empty(1, device="cuda:0")
t = time.perf_counter()
for _ in range(200):
    dist.all_reduce(x)
torch.cuda.synchronize()
print("dist.all_reduce(1 elem) %.1f us" % ((time.perf_counter() - t) / 200 * 1e6))
pr = cProfile.Profile()
pr.enable()
loop(50)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
dist.destroy_process_group()
