"""ORACLE (test infrastructure only) -- the CPU baseline leg of bench.py.

Times the oracle's full restatement of the reference hook (``oracle_group_topk_hook``:
comm_hooks/group_topk_hook_no_reshape.py:190-297 op for op, torch CPU ops, collectives over
a real gloo group on 127.0.0.1) on the bench's bucket, at world size 1 or 2, as SURVEY.md
section 8(d) defines the CPU path: ``threads = host CPU share // ws`` per rank.  Run as a
child process of bench.py with no GPU visible (it never initialises a device):

    python -m oracle.cpu_bench --ws 2 --threads 8 --seconds 8 --ef ef14 --workload headline

Prints one JSON line: median seconds per hook call (max over ranks), calls timed, threads.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def _rank(rank: int, args, port: int, out_q) -> None:
    import torch
    import torch.distributed as dist

    from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel
    from workloads import DDP_MODELS, WORKLOADS
    from oracle import arctopk as A

    torch.set_num_threads(args.threads)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=args.ws)
    if args.workload in DDP_MODELS:  # configs[1] / configs[3]: the first of the model's DDP buckets
        from workloads import ddp_buckets
        shapes = ddp_buckets(DDP_MODELS[args.workload][1]())[0]
    else:
        shapes = WORKLOADS[args.workload][1]
    n = bucket_numel(shapes)
    g = torch.Generator().manual_seed(1000 + rank)
    G = torch.randn(n, generator=g)
    st = A.OracleState(r=4, compress_ratio=0.2, start_compress_iter=0,
                       use_error_feedback=args.ef, seed=1234)
    buf = torch.empty(n)
    times = []
    t_end = time.perf_counter() + args.seconds
    calls = 0
    while True:
        buf.copy_(G)  # the bucket evolves in place in the hook: restart from G (untimed)
        dist.barrier()
        t0 = time.perf_counter()
        A.oracle_group_topk_hook(st, SyntheticBucket(buf, shapes))
        dt = time.perf_counter() - t0
        calls += 1
        # the first calls create E (EF14) or run the dense init (EF21): steady state only
        if calls > 2:
            times.append(dt)
        flag = torch.tensor([1 if (time.perf_counter() < t_end or len(times) < 2) else 0])
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)  # every rank stops at the same call
        if int(flag.item()) == 0:
            break
    t = torch.tensor(times, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # a call ends when its slowest rank ends
    if rank == 0:
        out_q.put({"median_s": statistics.median(t.tolist()), "calls": len(times)})
    dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", type=int, default=1)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--ef", default="ef14")
    ap.add_argument("--workload", default="headline")
    args = ap.parse_args()
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, args, port, q)) for r in range(args.ws)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
    res.update({"ws": args.ws, "threads_per_rank": args.threads})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
