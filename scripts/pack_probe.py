"""Per-segment-kind timing of the pack and decode kernels on one workload's bucket (diagnostic).

    python scripts/pack_probe.py resnet50_mixed [ef14]

Runs one hook call to populate the select outputs, then times arctopk_pack_segments /
arctopk_decode_segments over each segment kind (1-D, m <= 2, 3 <= m < 256, m >= 256) with
HIP events, and the whole-bucket launches for comparison.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd import _native as N  # noqa: E402
from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel  # noqa: E402
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import GroupTopKState, group_topk_hook  # noqa: E402
from workloads import WORKLOADS  # noqa: E402


def timed(fn, reps=50):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def timed_cold(fn, reps=20):
    """Each call after a 512 MiB memset (evicts the MALL / L2), timed alone."""
    big = torch.empty(128 << 20, dtype=torch.float32, device="cuda")
    tot = 0.0
    for _ in range(reps):
        big.fill_(1.0)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        tot += s.elapsed_time(e)
    return tot / reps * 1e3


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "resnet50_mixed"
    efn = sys.argv[2] if len(sys.argv) > 2 else "ef14"
    shapes = [tuple(s) for s in WORKLOADS[wl][1]]
    dev = torch.device("cuda:0")
    import socket
    import torch.distributed as dist
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    n = bucket_numel(shapes)
    G = torch.randn(n, device=dev)
    st = GroupTopKState(None, r=4, compress_ratio=0.2, start_compress_iter=0, use_error_feedback=efn, seed=1)
    for _ in range(3):
        group_topk_hook(st, SyntheticBucket(G.clone(), shapes, index=0, is_last=True)).wait()
    torch.cuda.synchronize()
    plan = st._plans[0][1]
    E = st.error_dict.get(0)
    gE = st.global_error_dict.get(0)
    ef = N.EF_CODE[efn]
    sid = torch.cuda.current_stream().cuda_stream
    out = G.clone()
    kinds = {}
    for i, s in enumerate(plan.segments):
        k = "1d" if s.kind == N.SEG_RAW else ("m<=2" if s.m <= 2 else ("m<256" if s.m < 256 else "m>=256"))
        kinds.setdefault(k, []).append(i)
    print(f"{wl} {efn}: numel {n}, segments {len(plan.segments)}")
    tp = timed(lambda: plan.pack(G, E, ef, sid))
    td = timed(lambda: plan.decode(1, ef, gE, out, sid))
    print(f"  whole bucket: pack {tp:7.2f} us  decode {td:7.2f} us  (back to back)")
    print(f"  whole bucket, cold: pack {timed_cold(lambda: plan.pack(G, E, ef, sid)):7.2f} us  "
          f"decode {timed_cold(lambda: plan.decode(1, ef, gE, out, sid)):7.2f} us  "
          f"select {timed_cold(lambda: plan.select(1, sid)):7.2f} us")
    for k, ids in kinds.items():
        segs = [plan.segments[i] for i in ids]
        el = sum(int(s.n * s.m) for s in segs)
        sel = sum(int(s.k_rows * s.m) for s in segs)

        def pk():
            for i in ids:
                plan.pack_range(i, i + 1, G, E, ef, sid)

        def dc():
            for i in ids:
                plan.decode_range(i, i + 1, 1, ef, gE, out, sid)
        print(f"  {k:7s} segs {len(ids):3d} elements {el:10d} selected {sel:9d}: "
              f"pack {timed(pk):7.2f} us  decode {timed(dc):7.2f} us  (one launch per segment)")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
