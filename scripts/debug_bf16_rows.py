"""Debug probe (measurement only): device encode sketch of bf16 / fp32 wave-per-row tensors vs
an fp32-accumulate, round-once reference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402

dev = torch.device("cuda", 0)
for dt in (torch.bfloat16, torch.float32):
    for shapes in ([[16, 64]], [[8], [16, 64]], [[64, 128]], [[256, 2048]], [[16], [256, 2048]], [[100, 64]],
                   [[2048, 2048]] * 2):
        g = torch.Generator().manual_seed(3)
        numel = sum(a * b if len(s) == 2 else s[0] for s in shapes for a, b in [tuple(s) if len(s) == 2 else (s[0], 1)])
        G = torch.randn(numel, generator=g).to(dt)
        p = BucketPlan([tuple(s) for s in shapes], 4, 0.2, dt, dev)
        V = torch.randn(max(1, p.info.v_len), generator=g).to(dt)
        p.encode(G.to(dev), None, N.EF_NONE, True, V.to(dev), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        sk = p.sketch.cpu()
        out = []
        for s in p.segments:
            if s.kind == N.SEG_RAW:
                continue
            x = G[s.offset:s.offset + s.n * s.m].view(s.n, s.m).float()
            v = V[s.v_off:s.v_off + s.m * 4].view(s.m, 4).float()
            ref = (x @ v).to(dt)
            d = sk[s.sketch_off:s.sketch_off + s.n * 4].view(s.n, 4)
            bad = int((d.float() - ref.float()).abs().gt(ref.float().abs() * 2 ** -6 + 1e-3).sum())
            out.append((s.n, s.m, bad))
        print(str(dt), shapes if len(shapes) < 3 else f"{len(shapes)}x{shapes[0]}", "(n, m, far-off entries):", out,
              flush=True)
