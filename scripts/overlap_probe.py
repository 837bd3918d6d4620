"""Probe (measurement only): does the latency-bound select chain of bucket b hide behind the
next bucket's encode when it runs on a side stream?  Phase entry points (encode -> select ->
pack -> decode, EF14, world size 1) over one backward's DDP buckets, K steps:

  serial : every phase on the caller's stream (the step path's order)
  side   : encodes on the caller's stream; each bucket's select / pack / decode on a
           high-priority side stream after an event on its encode
  side2  : as side, buckets alternating between two side streams

    python scripts/overlap_probe.py --workload resnet50_ddp --steps 50
Prints one JSON line per mode (us per step, GB/s of bucket)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.bucket import bucket_numel  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import BucketPlan  # noqa: E402
from workloads import DDP_MODELS, WORKLOADS, ddp_buckets  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="resnet50_ddp")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--buckets", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.workload in DDP_MODELS:
        layouts = ddp_buckets(DDP_MODELS[a.workload][1]())
    else:
        layouts = [WORKLOADS[a.workload][1]] * a.buckets
    L = N.lib()
    g = torch.Generator(device=dev).manual_seed(1000)
    plans, G, E = [], [], []
    for sh in layouts:
        p = BucketPlan([tuple(s) for s in sh], 4, 0.2, torch.float32, dev)
        N.check(L.arctopk_draw_projections(p.handle, 1234, p.V_ring[0].data_ptr(), 0), "draw")
        plans.append(p)
        G.append(torch.randn(bucket_numel(sh), device=dev, generator=g))
        E.append(torch.zeros(bucket_numel(sh), device=dev))
    nbytes = sum(4 * bucket_numel(sh) for sh in layouts)
    st = torch.cuda.current_stream(dev)
    sides = [torch.cuda.Stream(device=dev, priority=-1) for _ in range(2)]
    evs = [N.DeviceEvent() for _ in plans]
    join = [N.DeviceEvent() for _ in sides]

    def step(mode):
        ns = {"serial": 0, "side": 1, "side2": 2}[mode]
        for b, p in enumerate(plans):
            p.encode(G[b], E[b], N.EF14, True, p.V_ring[0], st.cuda_stream)
            if ns == 0:
                s = st.cuda_stream
            else:
                s = sides[b % ns].cuda_stream
                evs[b].record(st.cuda_stream)
                evs[b].wait(s)
            p.select(1, s)
            p.pack(G[b], E[b], N.EF14, s)
            p.decode(1, N.EF14, None, G[b], s)
        if ns:
            for i in range(ns):
                join[i].record(sides[i].cuda_stream)
                join[i].wait(st.cuda_stream)

    for mode in ("serial", "side", "side2", "serial", "side", "side2"):
        for _ in range(3):
            step(mode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step(mode)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(json.dumps({"workload": a.workload, "mode": mode, "us_per_step": round(dt * 1e6, 1),
                          "GBps": round(nbytes / dt / 1e9, 1), "buckets": len(plans)}), flush=True)


if __name__ == "__main__":
    main()
