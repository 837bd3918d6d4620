"""Host-ahead and projection pre-staging diagnostics for the 4-bucket headline step. GPU box only."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel  # noqa: E402
from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as H  # noqa: E402
from bench import WORKLOADS  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29512")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
sh = WORKLOADS["headline"][1]
bks = [SyntheticBucket(torch.randn(bucket_numel(sh), device="cuda:0"), sh, index=i, is_last=(i == 3))
       for i in range(4)]
st = H.GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback="ef14", seed=1)


def loop(n):
    torch.cuda.synchronize()
    h0, p0 = st.prestage_hits, st._proj.hits
    t0 = time.perf_counter()
    for _ in range(n):
        for b in bks:
            H.group_topk_hook(st, b)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"  host enqueue {(t1 - t0) / n / 4 * 1e6:.1f} us/call, wall {(t2 - t0) / n / 4 * 1e6:.1f} us/call, "
          f"prestaged {st.prestage_hits - h0}/{4 * n}, v_waits {sum(p[1].v_waits for p in st._plans.values())}, draw hits {st._proj.hits - p0} misses {st._proj.misses}",
          flush=True)


for _ in range(3):
    loop(5)
if os.environ.get("ONLY_ON"):
    loop(40)
    sys.exit(0)
print("prestaging on:")
loop(40)
orig = H._prestage_next
H._prestage_next = lambda *a: None
loop(5)
print("prestaging off:")
loop(40)
H._prestage_next = orig
