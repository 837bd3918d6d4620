"""Keys + compact passes alone (library built with ARCTOPK_DIAG_STOP=2) under a first-digit window
set by hand: the device histogram and per-range compact counts vs the host's."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import sel_window_dbg as D  # noqa: E402
from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402
from oracle import arctopk as A  # noqa: E402

setf = N.lib().arctopk_diag_set_mws
setf.restype = ctypes.c_int32
setf.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]


def main():
    shapes = [(2048, 1024, 1, 1), (40000, 8)]
    segs = A.segments(shapes, 0.2)
    plan = BucketPlan(shapes, 4, 0.2, torch.float32, D.DEV)
    stream = torch.cuda.current_stream().cuda_stream
    gen = torch.Generator().manual_seed(11)
    for call, (sh, bases) in enumerate([(19, (0, 0)), (14, (64254, 64258)), (14, (64254, 64258)), (19, (0, 0))]):
        wsh = np.array([sh, sh], dtype=np.uint32) if sh != 19 else np.zeros(2, dtype=np.uint32)
        wb = np.array(bases, dtype=np.uint32)
        N.check(setf(plan.handle, D.OFF_WSH, wsh.ctypes.data, 8), "set")
        N.check(setf(plan.handle, D.OFF_WBASE, wb.ctypes.data, 8), "set")
        # the histogram is cleared by the refine, which this library does not run
        z = np.zeros(2 * D.BINS, dtype=np.uint32)
        N.check(setf(plan.handle, D.OFF_HIST, z.ctypes.data, z.nbytes), "set")
        Ps = [torch.randn(s.n * 4, generator=gen).reshape(-1, 4) for s in segs]
        ref = torch.cat([p.flatten() for p in Ps])
        plan.sketch[:ref.numel()].copy_(ref.to(D.DEV))
        plan.select(1, stream)
        torch.cuda.synchronize()
        buf = D.dump(plan)
        norms, _ = A.select(Ps, 1, segs)
        for t, (s, nrm) in enumerate(zip(plan.segments, norms)):
            keys = nrm.numpy().astype(np.float32).view(np.uint32).astype(np.int64)
            base = bases[t]
            h = keys >> sh
            d_all = np.where(h < base, 0, np.minimum(h - base, 4095))
            hist = np.bincount(d_all, minlength=4096)
            slots = D.u32(buf, D.OFF_HIST + t * D.BINS * 4, D.BINS)
            bins = np.arange(4096)
            dev_hist = slots[((bins & 127) << 5) | (bins >> 7)]
            k = int(s.k_rows)
            cum, b = 0, 4095
            for b in range(4095, -1, -1):
                if cum + hist[b] >= k:
                    break
                cum += hist[b]
            nr = (s.n + 4095) // 4096
            gt_dev = D.u32(buf, D.OFF_GT + t * D.RANGES * 4, nr).astype(np.int64)
            cand_dev = D.u32(buf, D.OFF_CAND + t * D.RANGES * 4, nr).astype(np.int64)
            rng_idx = np.arange(s.n) // 4096
            gt_host = np.bincount(rng_idx[d_all > b], minlength=nr)
            cand_host = np.bincount(rng_idx[d_all == b], minlength=nr)
            st = buf[D.OFF_ST + 64 * t: D.OFF_ST + 64 * (t + 1)]
            prefix, mask = st[0:8].view(np.uint32)
            kk = int(st[16:24].view(np.int64)[0])
            print(f"call {call} item {t} sh {sh} base {base}: hist differs at {(dev_hist != hist).sum()} bins "
                  f"(sum dev {dev_hist.sum()} host {hist.sum()}); host bin {b} kk {k - cum}; dev state prefix "
                  f"{int(prefix):#x} mask {int(mask):#x} kk {kk}; gt ranges differing {(gt_dev != gt_host).sum()}, "
                  f"cand ranges differing {(cand_dev != cand_host).sum()}", flush=True)


if __name__ == "__main__":
    main()
