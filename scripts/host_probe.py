"""Host side of the hook on small buckets: is the step host-bound?

For one workload (default: configs[1]'s ResNet-18 DDP buckets) and one hook path (the ws = 1
step, or --force-exchange), time K steps three ways:
  wall     K steps then one synchronize (what bench.py's value is made of)
  enqueue  the host time of the same K steps, measured before the synchronize (when it is
           close to `wall`, the host, not the GPU, sets the pace)
  per call the host time of each hook call (median over calls of a bucket index)
and print one JSON line.  Run on the GPU box:  python scripts/host_probe.py [--force-exchange]
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="resnet18_ddp")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--force-exchange", action="store_true")
    args = ap.parse_args()
    import bench
    from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel
    from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import GroupTopKState, group_topk_hook
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    if args.workload in bench.DDP_MODELS:
        layouts = bench.ddp_buckets(bench.DDP_MODELS[args.workload][1]())
    else:
        layouts = [bench.WORKLOADS[args.workload][1]] * 4
    g = torch.Generator(device=dev).manual_seed(1000)
    buckets = [SyntheticBucket(torch.randn(bucket_numel(sh), device=dev, generator=g), sh, index=i,
                               is_last=(i == len(layouts) - 1)) for i, sh in enumerate(layouts)]
    st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback="ef14", seed=1)
    st.force_exchange = args.force_exchange
    st.defer_decode = True
    if args.force_exchange:
        st.init_exchange_comms(dev)
    per_call = [[] for _ in buckets]

    def step(record):
        futs = []
        for i, bk in enumerate(buckets):
            t = time.perf_counter()
            futs.append(group_topk_hook(st, bk))
            if record:
                per_call[i].append(time.perf_counter() - t)
        t = time.perf_counter()
        for f in futs:
            f.wait()
        if record:
            per_call[-1][-1] += time.perf_counter() - t  # the finalize counts with the last call

    for _ in range(10):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    out = {"workload": args.workload, "path": "exchange (forced)" if args.force_exchange else "step",
           "steps": args.steps, "wall_us_per_step": round(t_wall / args.steps * 1e6, 1),
           "enqueue_us_per_step": round(t_enq / args.steps * 1e6, 1),
           "host_us_per_call_median": [round(statistics.median(c) * 1e6, 1) for c in per_call],
           "bucket_mib": [round(bucket_numel(sh) * 4 / 2**20, 2) for sh in layouts]}
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
