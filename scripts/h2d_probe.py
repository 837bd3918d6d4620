"""Host cost of the projection H2D: torch copy_ vs libarctopk's hipMemcpyAsync (GPU box)."""
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from allreducetopk_amd import _native as N  # noqa: E402

n = 131072
h = torch.randn(n).pin_memory()
h2 = torch.empty(n, pin_memory=True)
d = torch.empty(n, device="cuda")
s = torch.cuda.Stream()
print("pinned", h.is_pinned(), h2.is_pinned())
for name, src in (("pin_memory()", h), ("empty(pin_memory)", h2)):
    for how in ("torch", "native"):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(100):
            if how == "torch":
                with torch.cuda.stream(s):
                    d.copy_(src, non_blocking=True)
            else:
                N.check(N.lib().arctopk_memcpy_h2d_async(d.data_ptr(), src.data_ptr(), n * 4, s.cuda_stream), "h2d")
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"{name:18s} {how:7s} host {(t1 - t) / 100 * 1e6:7.1f} us  wall {(time.perf_counter() - t) / 100 * 1e6:7.1f} us")
