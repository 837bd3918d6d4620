"""Per-kernel device time and achieved HBM GB/s on the headline bucket (GPU box only).

Interleaves every variant in one process (guide rule 24) and reports the median of
REPS launches per variant, next to memcpy-class torch ops moving comparable bytes.
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
shapes = [tuple(s) for s in ([[2048, 2048]] * 16)]
if os.environ.get("SHAPES") == "resnet18":
    shapes = [(512, 512, 3, 3)] * 28
dev = "cuda:0"
plan = BucketPlan(shapes, 4, 0.2, torch.float32, dev)
n = plan.info.numel
K = plan.info.values_len
G = torch.randn(n, device=dev)
E = torch.randn(n, device=dev) * 0.1
gE = torch.randn(n, device=dev)
out = torch.empty(n, device=dev)
V = torch.randn(plan.info.v_len, device=dev)
a = torch.empty(n, device=dev)
b = torch.empty(n, device=dev)
s = torch.cuda.current_stream().cuda_stream
sk = plan.info.sketch_len * 4

plan.encode(G, E, N.EF14, True, V, s)
plan.select(1, s)
torch.cuda.synchronize()

variants = {
    "torch copy_ (R4N W4N)": (lambda: a.copy_(G), 8 * n),
    "torch add out= (R8N W4N)": (lambda: torch.add(G, E, out=a), 12 * n),
    "torch sum (R4N)": (lambda: G.sum(), 4 * n),
    "torch fill_ zero (W4N)": (lambda: a.zero_(), 4 * n),
    "encode noef": (lambda: plan.encode(G, None, N.EF_NONE, True, V, s), 4 * n + sk),
    "encode ef14": (lambda: plan.encode(G, a, N.EF14, True, V, s), 12 * n + sk),
    "encode ef21": (lambda: plan.encode(G, E, N.EF21, True, V, s), 8 * n + sk),
    "select": (lambda: plan.select(1, s), 2 * sk),
    "pack noef": (lambda: plan.pack(G, None, N.EF_NONE, s), 8 * K),
    "pack ef14": (lambda: plan.pack(G, b, N.EF14, s), 12 * K),
    "pack ef21": (lambda: plan.pack(G, b, N.EF21, s), 16 * K),
    "decode noef/ef14": (lambda: plan.decode(1, N.EF_NONE, None, out, s), 4 * K + 4 * n),
    "decode ef21": (lambda: plan.decode(1, N.EF21, gE, out, s), 8 * K + 8 * n),
    "decode(out=G)+encode ef14 pair": (lambda: (plan.decode(1, N.EF_NONE, None, G, s),
                                                plan.encode(G, a, N.EF14, True, V, s)),
                                       4 * K + 4 * n + 12 * n + sk),
}
L = N.lib()
nt = len(shapes)
numel_t = [int(torch.Size(sh).numel()) for sh in shapes]
ks = [max(1, int(x * 0.2)) for x in numel_t]
offs = [sum(numel_t[:i]) for i in range(nt)]
kof = [sum(ks[:i]) for i in range(nt)]
A_off, A_n, A_k, A_ko = N.i64_array(offs), N.i64_array(numel_t), N.i64_array(ks), N.i64_array(kof)
sk_idx = torch.empty(sum(ks), dtype=torch.int32, device=dev)
sk_val = torch.empty(sum(ks), device=dev)
wsb = torch.empty(int(L.arctopk_sparse_workspace_bytes(len(ks), N.i64_array(numel_t))), dtype=torch.uint8, device=dev)
KS = sum(ks)
variants["sparse ef_apply ef14"] = (lambda: L.arctopk_ef_apply(a.data_ptr(), b.data_ptr(), n, N.EF14, 1, 0, s), 12 * n)
variants["topk_select (16 tensors)"] = (lambda: L.arctopk_topk_select(G.data_ptr(), nt, A_off, A_n, A_k, A_ko, sk_idx.data_ptr(), sk_val.data_ptr(), wsb.data_ptr(), 0, 0, s), 4 * 5 * n + 8 * KS)
variants["randk_indices hash"] = (lambda: L.arctopk_randk_indices(nt, A_n, A_k, A_ko, 7, sk_idx.data_ptr(), s), 4 * KS)
variants["sparse_gather"] = (lambda: L.arctopk_sparse_gather(G.data_ptr(), nt, A_off, A_k, A_ko, sk_idx.data_ptr(), sk_val.data_ptr(), 0, s), 12 * KS)
variants["sparse_residual ef14"] = (lambda: L.arctopk_sparse_residual(b.data_ptr(), nt, A_off, A_k, A_ko, sk_idx.data_ptr(), sk_val.data_ptr(), N.EF14, 0, s), 8 * KS)
variants["sparse_decode randk"] = (lambda: L.arctopk_sparse_decode(out.data_ptr(), n, nt, A_off, A_k, A_ko, KS, sk_idx.data_ptr(), sk_val.data_ptr(), 1, 1, 0, None, 0, s), 4 * n + 12 * KS)
variants["sparse_decode topk ws1"] = (lambda: L.arctopk_sparse_decode(out.data_ptr(), n, nt, A_off, A_k, A_ko, KS, sk_idx.data_ptr(), sk_val.data_ptr(), 1, 1, 1, None, 0, s), 12 * n + 12 * KS)
times = {k: [] for k in variants}
for k, (fn, _) in variants.items():  # warm
    fn()
torch.cuda.synchronize()
for rep in range(REPS):
    for k, (fn, _) in variants.items():
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        times[k].append(e0.elapsed_time(e1) * 1e3)
print(f"shapes={shapes[0]}x{len(shapes)} numel={n} packed={K} reps={REPS}")
for k, (fn, nbytes) in variants.items():
    med = statistics.median(times[k])
    print(f"{k:28s} {med:9.2f} us  min {min(times[k]):9.2f}  {nbytes / med / 1e3:8.1f} GB/s")
