"""Diagnose the multi-block ARC select's first-digit window on one GPU: after each select call,
dump the plan's select workspace (arctopk_diag_mws) and compare the device's item state and
per-range counts with the same quantities computed on the host from the oracle's energies.

    python scripts/sel_window_dbg.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402
from oracle import arctopk as A  # noqa: E402

DEV = "cuda:0"
MB, BINS, MWIN, RANGES = 48, 4096, 4096, 1024
OFF_HIST = 0
OFF_WSH = OFF_HIST + MB * BINS * 4
OFF_WBASE = OFF_WSH + MWIN * 4
OFF_ST = OFF_WBASE + MWIN * 4
OFF_NCAND = OFF_ST + MB * 64
OFF_DONE = OFF_NCAND + MB * 128
OFF_POR = OFF_DONE + MB * 128
OFF_PAND = OFF_POR + MB * 512 * 4
OFF_GT = OFF_PAND + MB * 512 * 4
OFF_EQ = OFF_GT + MB * RANGES * 4
OFF_TAKE = OFF_EQ + MB * RANGES * 4
OFF_SELB = OFF_TAKE + MB * RANGES * 4
OFF_CAND = OFF_SELB + MB * RANGES * 4
OFF_COR = OFF_CAND + MB * RANGES * 4
OFF_CAND_AND = OFF_COR + MB * RANGES * 4
TOTAL = OFF_CAND_AND + MB * RANGES * 4

L = N.lib()
dump_fn = L.arctopk_diag_mws
dump_fn.restype = ctypes.c_int32
dump_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]


keys_fn = L.arctopk_diag_keys
keys_fn.restype = ctypes.c_int32
keys_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]


def dev_keys(plan):
    k = np.zeros(int(plan.info.rows_total), dtype=np.uint32)
    N.check(keys_fn(plan.handle, k.ctypes.data, k.size), "diag_keys")
    return k


def dump(plan):
    buf = np.zeros(TOTAL, dtype=np.uint8)
    N.check(dump_fn(plan.handle, buf.ctypes.data, TOTAL), "diag_mws")
    return buf


def u32(buf, off, n):
    return buf[off:off + 4 * n].view(np.uint32)


def main():
    shapes = [(2048, 1024, 1, 1), (40000, 8)]
    segs = A.segments(shapes, 0.2)
    plan = BucketPlan(shapes, 4, 0.2, torch.float32, DEV)
    stream = torch.cuda.current_stream().cuda_stream
    gen = torch.Generator().manual_seed(11)
    win_prev = dump(plan)
    for call in range(3):
        Ps = [torch.randn(s.n * 4, generator=gen).reshape(-1, 4) for s in segs]
        ref = torch.cat([p.flatten() for p in Ps])
        plan.sketch[:ref.numel()].copy_(ref.to(DEV))
        plan.select(1, stream)
        torch.cuda.synchronize()
        buf = dump(plan)
        dk = dev_keys(plan)
        norms, _ = A.select(Ps, 1, segs)
        for t, (s, nrm) in enumerate(zip(plan.segments, norms)):
            keys = nrm.numpy().astype(np.float32).view(np.uint32).astype(np.int64)
            sh = int(u32(win_prev, OFF_WSH, MWIN)[t]) or 19
            base = int(u32(win_prev, OFF_WBASE, MWIN)[t]) if u32(win_prev, OFF_WSH, MWIN)[t] else 0
            h = keys >> sh
            d_all = np.where(h < base, 0, np.minimum(h - base, 4095))
            hist = np.bincount(d_all, minlength=4096)
            k = int(s.k_rows)
            cum, b = 0, 4095
            for b in range(4095, -1, -1):
                if cum + hist[b] >= k:
                    break
                cum += hist[b]
            st = buf[OFF_ST + 64 * t: OFF_ST + 64 * (t + 1)]
            prefix, mask = st[0:8].view(np.uint32)
            bit = int(st[8:12].view(np.int32)[0])
            kk = int(st[16:24].view(np.int64)[0])
            nr = (s.n + 4095) // 4096
            gt_dev = u32(buf, OFF_GT + t * RANGES * 4, nr).astype(np.int64)
            cand_dev = u32(buf, OFF_CAND + t * RANGES * 4, nr).astype(np.int64)
            take = u32(buf, OFF_TAKE + t * RANGES * 4, nr).astype(np.int64)
            selb = u32(buf, OFF_SELB + t * RANGES * 4, nr).astype(np.int64)
            rng_idx = np.arange(s.n) // 4096
            gt_host = np.bincount(rng_idx[d_all > b], minlength=nr)
            cand_host = np.bincount(rng_idx[d_all == b], minlength=nr)
            T = int(np.sort(keys)[::-1][k - 1])
            print(f"call {call} item {t}: window sh={sh} base={base}; host bin {b} above {cum} cand {hist[b]} "
                  f"T {T:#x} | dev prefix {int(prefix):#x} mask {int(mask):#x} bit {bit} kk {kk} "
                  f"(host kk {k - cum}); cnt_gt sum dev {gt_dev.sum()} host {gt_host.sum()} "
                  f"(ranges differing {(gt_dev != gt_host).sum()}); cand sum dev {cand_dev.sum()} host "
                  f"{cand_host.sum()} (differing {(cand_dev != cand_host).sum()}); take sum {take.sum()} "
                  f"sel_before last {selb[-1]}", flush=True)
            kd = dk[s.row_off:s.row_off + s.n].astype(np.int64)
            bad = np.nonzero(gt_dev != gt_host)[0]
            print(f"   device keys differ from host keys at {(kd != keys).sum()} rows; first ranges "
                  f"differing (r, dev gt, host gt, dev cand, host cand): "
                  f"{[(int(r_), int(gt_dev[r_]), int(gt_host[r_]), int(cand_dev[r_]), int(cand_host[r_])) for r_ in bad[:6]]}")
            # which bin would make each differing range's device counts?
            for r_ in bad[:3]:
                kr = keys[r_ * 4096:(r_ + 1) * 4096]
                hr = kr >> sh
                dd = np.where(hr < base, 0, np.minimum(hr - base, 4095))
                sols = [bb for bb in range(max(0, b - 64), min(4096, b + 64))
                        if (dd > bb).sum() == gt_dev[r_] and (dd == bb).sum() == cand_dev[r_]]
                alt = []
                for sh2, base2 in ((19, 0), (14, base - 1), (14, base + 1)):
                    h2 = kr >> sh2
                    d2 = np.where(h2 < base2, 0, np.minimum(h2 - base2, 4095))
                    alt += [(sh2, base2, bb) for bb in range(4096) if (d2 > bb).sum() == gt_dev[r_] and (d2 == bb).sum() == cand_dev[r_]]
                print(f"      range {int(r_)}: bins matching the device counts {sols[:5]}, other windows {alt[:5]}")
            sm = plan.slotmap[s.row_off:s.row_off + s.n].cpu()
            print(f"   slots set {int((sm >= 0).sum())} of {k}; new window sh="
                  f"{int(u32(buf, OFF_WSH, MWIN)[t])} base={int(u32(buf, OFF_WBASE, MWIN)[t])}", flush=True)
        win_prev = buf


if __name__ == "__main__":
    main()
