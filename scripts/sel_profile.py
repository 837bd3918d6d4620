"""Select / pack / decode launches on the ResNet-shaped bucket and the TopK select, for a
rocprofv3 --kernel-trace --stats breakdown per kernel (GPU box only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402

dev = "cuda:0"
REPS = int(os.environ.get("REPS", "10"))
s = torch.cuda.current_stream().cuda_stream
shapes = [(512, 512, 3, 3)] * 28
plan = BucketPlan(shapes, 4, 0.2, torch.float32, dev)
n = plan.info.numel
G = torch.randn(n, device=dev)
E = torch.randn(n, device=dev)
V = torch.randn(plan.info.v_len, device=dev)
out = torch.empty(n, device=dev)
plan.encode(G, E, N.EF14, True, V, s)
for _ in range(REPS):
    plan.select(1, s)
    plan.pack(G, E, N.EF14, s)
    plan.decode(1, N.EF_NONE, None, out, s)
L = N.lib()
tshapes = [(2048, 2048)] * 16
numel_t = [int(torch.Size(sh).numel()) for sh in tshapes]
ks = [max(1, int(x * 0.2)) for x in numel_t]
offs = [sum(numel_t[:i]) for i in range(len(ks))]
kof = [sum(ks[:i]) for i in range(len(ks))]
X = torch.randn(sum(numel_t), device=dev)
idx = torch.empty(sum(ks), dtype=torch.int32, device=dev)
val = torch.empty(sum(ks), device=dev)
wsb = torch.empty(int(L.arctopk_sparse_workspace_bytes(len(ks), N.i64_array(numel_t))), dtype=torch.uint8, device=dev)
for _ in range(REPS):
    N.check(L.arctopk_topk_select(X.data_ptr(), len(ks), N.i64_array(offs), N.i64_array(numel_t),
                                  N.i64_array(ks), N.i64_array(kof), idx.data_ptr(), val.data_ptr(),
                                  wsb.data_ptr(), 0, 0, s), "topk_select")
torch.cuda.synchronize()
print("done")
