"""Debug probe (measurement only): structured inputs through the bf16 wave-per-row encode."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402

dev = torch.device("cuda", 0)
n, m = 4, 64


def run(G, V, dt=torch.bfloat16):
    p = BucketPlan([(n, m)], 4, 0.25, dt, dev)
    p.encode(G.to(dt).to(dev), None, N.EF_NONE, True, V.to(dt).to(dev), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return p.sketch[:n * 4].view(n, 4).float().cpu()


ones = torch.ones(n * m)
print("G=1, V=1 (expect 64):\n", run(ones, torch.ones(m * 4)))
Gr = torch.arange(1, n + 1, dtype=torch.float32).repeat_interleave(m)
print("G=row+1, V=1 (expect 64*(r+1)):\n", run(Gr, torch.ones(m * 4)))
V = torch.zeros(m, 4)
for j in range(4):
    V[j, j] = 1.0
Gc = (torch.arange(m, dtype=torch.float32) + 1).repeat(n)
print("G=col+1, V[c][j]=[c==j] (expect cols 1..4):\n", run(Gc, V.flatten()))
V2 = torch.zeros(m, 4)
V2[:, 0] = 1.0
print("G=col+1, V[:,0]=1 (expect 2080, 0, 0, 0):\n", run(Gc, V2.flatten()))
print("fp32 same:\n", run(Gc, V2.flatten(), torch.float32))
