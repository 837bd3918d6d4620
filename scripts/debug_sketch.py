"""Debug probe (measurement only): the device encode's sketch per segment vs torch CPU `mm` on
the same V, for a golden fixture's first bucket (rank 0)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402
from golden_io import Golden  # noqa: E402
from oracle import arctopk as A  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "arc_gmix_noef_bf16_ws2"
g = Golden(name)
m = g.meta
shapes = [tuple(s) for s in m["shapes"]]
dt = torch.bfloat16 if m.get("dtype") == "bf16" else torch.float32
G = g.t(0, 0, "G")
seed = int(g.np(0, 0, "seed")[0])
segs = A.segments(shapes, m["ratio"])
Vs = A.draw_projections(seed, segs, m["r"], dt)
X, Ps = A.encode(G, None, "noef", segs, Vs)
dev = torch.device("cuda", 0)
p = BucketPlan(shapes, m["r"], m["ratio"], dt, dev)
V = torch.cat([v.flatten() for v, s in zip(Vs, segs) if s.kind != A.RAW]).to(dev)
Gd = G.to(dev)
p.encode(Gd, None, N.EF_NONE, True, V, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
sk = p.sketch.cpu()
for j, (s, P, seg) in enumerate(zip(segs, Ps, p.segments)):
    d = sk[int(seg.sketch_off):int(seg.sketch_off) + P.numel()].view_as(P)
    diff = (d.double() - P.double()).abs()
    rel = (diff / P.double().abs().clamp_min(1e-30)).max().item()
    neq = int((d != P).sum())
    print(f"seg {j} shape {shapes[j]} n {s.n} m {s.m} kind {s.kind} off {s.offset} differs {neq}/{P.numel()} max rel {rel:.3e}")
    if neq:
        idx = torch.nonzero((d != P).flatten()).flatten()[:6]
        print("   dev", d.flatten()[idx].tolist(), "ref", P.flatten()[idx].tolist(), d.dtype, P.dtype)
        if s.kind != A.RAW:  # fp32 accumulation, one rounding (what the device forms)
            x = X[s.offset:s.offset + s.numel].view(s.n, s.m).float()
            f = (x @ Vs[j].float()).to(dt)
            print("   fp32-acc-once differs from dev in", int((f != d).sum()), "from CPU mm in", int((f != P).sum()))
# the native CPU-stream draw (projections="host") vs torch's own
sizes = [s.m * m["r"] for s in segs if s.kind != A.RAW]
host = torch.empty(sum(sizes), dtype=dt)
arr = (N.c_int64 * len(sizes))(*sizes)
N.check(N.lib().arctopk_draw_normal(seed, N.DTYPE_CODE[dt], len(sizes), arr, host.data_ptr()), "draw")
ref = torch.cat([v.flatten() for v in Vs if v is not None])
off = 0
for s_, n_ in zip([s for s in segs if s.kind != A.RAW], sizes):
    a, b = host[off:off + n_], ref[off:off + n_]
    print(f"V m {s_.m}: native draw differs in {int((a != b).sum())}/{n_}")
    off += n_
