"""Read back the multi-block select's per-item state after a TopK select (GPU box):
candidate mode flag, candidate count and threshold, to check the mode each item took."""
import os
import struct
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd import _native as N  # noqa: E402

KMB, KBINS = 48, 4096
ST_OFF = KMB * KBINS * 4            # MWorkspace::st
NC_OFF = ST_OFF + KMB * 64          # MWorkspace::ncand (128-B counters)
dev = "cuda:0"
L = N.lib()
s = torch.cuda.current_stream().cuda_stream
for label, numel_t, gen in [("topk 16x4M randn", [4 << 20] * 16, lambda n: torch.randn(n, device=dev)),
                            ("chi2_4-like energies 28x131072", [131072] * 28,
                             lambda n: (torch.randn(n, 4, device=dev) ** 2).sum(1))]:
    ks = [max(1, int(x * 0.2)) for x in numel_t]
    offs = [sum(numel_t[:i]) for i in range(len(ks))]
    kof = [sum(ks[:i]) for i in range(len(ks))]
    X = gen(sum(numel_t))
    idx = torch.empty(sum(ks), dtype=torch.int32, device=dev)
    val = torch.empty(sum(ks), device=dev)
    nb = int(L.arctopk_sparse_workspace_bytes(len(ks), N.i64_array(numel_t)))
    wsb = torch.zeros(nb, dtype=torch.uint8, device=dev)
    N.check(L.arctopk_topk_select(X.data_ptr(), len(ks), N.i64_array(offs), N.i64_array(numel_t),
                                  N.i64_array(ks), N.i64_array(kof), idx.data_ptr(), val.data_ptr(),
                                  wsb.data_ptr(), 0, 0, s), "topk_select")
    torch.cuda.synchronize()
    w = wsb.cpu().numpy().tobytes()
    print("==", label, "workspace", nb)
    for t in range(min(len(ks), 4)):
        prefix, mask, bit, cand, kk, p1, m1 = struct.unpack_from("<IIiiqII", w, ST_OFF + 64 * t)
        ncand = struct.unpack_from("<I", w, NC_OFF + 128 * t)[0]
        print(f"item {t}: cand={cand} ncand={ncand} ({ncand / numel_t[t]:.4f} of n) bit={bit} kk={kk} "
              f"T={prefix:#010x}")
