"""Benchmark of the ARC-TopK comm-hook codec on MI355X (BASELINE.json metric).

One "step" = one backward's worth of buckets hooked in order as DDP does (default:
4 buckets of 256 MiB fp32, 16 x [2048, 2048] each, the Llama-1B projection shape;
SURVEY.md section 8d): per bucket encode -> RCCL all_reduce(sketch) -> select -> pack
-> RCCL all_reduce(packed) -> decode, steady-state EF14 (configs[1]'s mode),
compress_ratio 0.2, r 4, inputs resident in HBM.  At world size > 1 a bucket's packed
all-reduce and decode overlap the next bucket's encode.

    python bench.py [--gpus N --steps K --warmup W --ef ef14|ef21|noef --workload W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints ONE JSON line (rank 0).  ``value`` = bucket bytes processed by all ranks
/ wall time of the K timed steps (max over ranks).  ``roofline`` prices the
dominant kernel (encode) by its algorithmic HBM bytes over its HIP-event
duration; ``cpu_baseline`` times the CPU oracle (test infrastructure) on a
bounded sample of the same bucket on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from allreducetopk_amd.bucket import SyntheticBucket, bucket_numel  # noqa: E402
from workloads import DDP_MODELS, HEADLINE, WORKLOADS, ddp_buckets, resnet18_cifar_shapes  # noqa: E402,F401
from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import (GroupTopKState,  # noqa: E402
                                                                      group_topk_hook)

METRIC = "compressed grad GB/s (device-resident) per GPU at k=0.2, r=4; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured float4 copy
PHASES = ["encode", "sketch_allreduce", "select", "pack", "packed_allreduce", "decode"]


# the plan's select rules (csrc/common.h): single-block selects up to 15,360 rows, or 4,096 beside
# multi-block items; V^T slices of at most 64 KiB per encode part
SMALL_SEL_ROWS, SMALL_SEL_ROWS_MIXED, V_LDS_MAX_BYTES = 15360, 4096, 64 * 1024


def algorithmic_bytes(ef: str, shapes, ratio: float, r: int, eb: int = 4, keyed: bool = False):
    """Minimum HBM bytes per call, per phase (element size eb, fused design).

    1-D tensors are their own sketch (written by encode, read by select); 2-D/ND
    tensors add an [n, r] sketch and read an [m, r] projection.  keyed (world size 1, the step
    path): the multi-block select items' encode writes a 4-B energy key per row instead of
    their sketch rows, and the select reads those keys (keys mode); and for
    EF14 / noef the pack and the decode are one pass with no packed copy (the all-reduce is the
    identity: DESIGN.md section 4, finalize).
    """
    from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import _geometry
    n_el = bucket_numel(shapes)
    geo = [(_geometry(s_), len(s_)) for s_ in shapes]
    any_large = any(n > SMALL_SEL_ROWS for (_, n, _), _nd in geo)
    small_cap = SMALL_SEL_ROWS_MIXED if any_large else SMALL_SEL_ROWS
    k_el = sk = vbytes = rows = k_rows = 0
    for (kind, n, m), nd in geo:
        k_el += max(1, int(n * ratio)) * m
        rows += n
        k_rows += max(1, int(n * ratio))
        va = 8 if eb == 2 else 4  # (the plan's column-part rule: unsplit rows only)
        if keyed and nd > 1 and n > small_cap and m <= V_LDS_MAX_BYTES // (4 * r) // va * va:
            sk += 4 * n  # the row's energy key instead of its sketch
        else:
            sk += eb * n * (1 if m == 1 and nd == 1 else r)
        vbytes += 0 if nd == 1 else m * r * eb
    if ef == "noef" and keyed:  # world size 1: no packed copy; the unselected elements are zeroed
        enc = eb * n_el + sk + vbytes
        pack = 0
        dec = eb * (n_el - k_el)
        read = eb * n_el + vbytes + sk
    elif ef == "noef":
        enc = eb * n_el + sk + vbytes
        pack = 2 * eb * k_el
        dec = eb * (k_el + n_el)
        read = eb * n_el + vbytes + sk + eb * k_el + eb * k_el
    elif ef == "ef14" and keyed:  # world size 1: decode := the selected rows of E, which are zeroed
        enc = 3 * eb * n_el + sk + vbytes
        pack = 0
        dec = eb * (n_el + 2 * k_el)  # write out; read E rows, zero E rows
        read = 2 * eb * n_el + vbytes + sk + eb * k_el
    elif ef == "ef14":
        enc = 3 * eb * n_el + sk + vbytes          # read G, E; write E := G + E
        pack = 3 * eb * k_el  # read E rows, write packed, zero E rows
        dec = eb * (k_el + n_el)
        read = 2 * eb * n_el + vbytes + sk + eb * k_el + eb * k_el
    else:  # ef21
        enc = 2 * eb * n_el + sk + vbytes           # read G, E
        pack = 4 * eb * k_el  # read G, E rows; write packed, E rows
        dec = eb * (2 * k_el + 2 * n_el)  # packed, gE, out, gE rows
        read = 2 * eb * n_el + vbytes + sk + 2 * eb * k_el + eb * (k_el + n_el)
    # select: read the sketch once; write the slot map (int32 per row) and the row list
    # (int32 per selected row)
    sel = sk + 4 * rows + 4 * k_rows
    return dict(encode=enc, select=sel, pack=pack, decode=dec, total=enc + sel + pack + dec,
                read=read)


def sparse_algorithmic_bytes(hook: str, ef: str, n_el: int, k_el: int, ws: int, eb: int = 4):
    """Minimum HBM bytes per call of the TopK / RandK baselines (EF14 only; None otherwise).

    TopK: SURVEY.md section 8(d)'s (28 + (8 + 16 ws) rho) B per element -- the EF14 fold
    (read G, E; write E: 12), a two-pass radix select over |x| (2 x 4), compaction (4), the
    decode's zero-fill (4), the gathered values and indices (8 rho) and the rank-ordered
    scatter of every rank's values and indices (16 ws rho), with rho = k / N.
    RandK: the fold (12), the index draw and the gather (12 rho: indices written, values read
    and written), the residual zero at the indices (8 rho: indices read, E written), the decode
    (4 + 8 rho: zero-fill, values and indices read) -> 16 + 28 rho."""
    if ef != "ef14" or eb != 4:
        return None
    if hook == "topk":
        return int(28 * n_el + (8 + 16 * ws) * k_el)
    return int(16 * n_el + 28 * k_el)


def pmc_call_traffic(workload: str, ef: str, tag: str = "fx"):
    """HBM bytes per hook call of the N > 1 code path (every libarctopk kernel of a call: encode,
    key / select passes, pack, decode) from the newest profiles/<round>/pmc_<workload>_<ef>_<tag>.json
    (scripts/profile.sh with BENCH_ARGS=--force-exchange; summarize_prof.py's `per_call`)."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "*", f"pmc_{workload}_{ef}_{tag}.json")))
    if not paths:
        return None, None, None
    with open(paths[-1]) as fh:
        doc = json.load(fh)
    pc = doc.get("per_call")
    if not pc:
        return None, None, None
    from allreducetopk_amd.build import embedded_hash
    lib = doc.get("lib_hash")
    return pc["bytes"], os.path.relpath(paths[-1], REPO), (None if lib is None else lib == embedded_hash())


def pmc_traffic(workload: str, ef: str, kernel: str, n_gpus: int = 1):
    """HBM bytes per launch of `kernel` from the newest committed PMC profile of this
    workload (profiles/<round>/pmc_<workload>_<ef>.json, written by
    scripts/summarize_prof.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes of
    this same bench command; FETCH_SIZE doubled per the gfx950 correction).  At N > 1 only a
    profile taken at that N counts (pmc_<workload>_<ef>_n<N>.json): the N = 1 file is never
    reported for a multi-GPU line."""
    import glob
    suffix = "" if n_gpus == 1 else f"_n{n_gpus}"
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "*", f"pmc_{workload}_{ef}{suffix}.json")))
    if not paths:
        return None, None, None
    with open(paths[-1]) as fh:
        doc = json.load(fh)
    ent = doc["kernels"].get(kernel)
    if not ent:
        return None, None, None
    # the profile's library vs the one running now (PMC files stamped with the source hash)
    from allreducetopk_amd.build import embedded_hash
    lib = doc.get("lib_hash")
    match = None if lib is None else lib == embedded_hash()
    return ent["bytes_per_launch"], os.path.relpath(paths[-1], REPO), match


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> int:
    """Host CPU threads this job may use: the affinity mask, capped by OMP_NUM_THREADS (the
    GPU box exports 16, its share of a many-core host)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(ef: str, seconds: float, workload: str, label: str, bucket_bytes: int,
                 hook: str = "arc"):
    """SURVEY.md section 8(d)'s CPU path: the oracle's restatement of the reference hook
    (oracle/cpu_bench.py, torch CPU ops, collectives over gloo on 127.0.0.1) on the same
    bucket at world size 1 and 2, threads = host CPU share // ws per rank, run in child
    processes that see no GPU.  value = bucket GB/s per rank at ws = 1."""
    if hook != "arc":
        return None
    import subprocess
    threads = cpu_share()
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS=str(threads))
    runs = {}
    for ws in (1, 2):
        per = max(1, threads // ws)
        cmd = [sys.executable, "-m", "oracle.cpu_bench", "--ws", str(ws), "--threads", str(per),
               "--seconds", str(seconds), "--ef", ef, "--workload", workload]
        try:
            r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
            runs[ws] = json.loads(line)
        except (subprocess.SubprocessError, IndexError, ValueError) as e:
            runs[ws] = {"error": f"{type(e).__name__}: {e}"[:200]}
    if "median_s" not in runs.get(1, {}):
        return {"value": None, "unit": "GB/s", "cores": threads, "kind": "port",
                "sample": f"CPU oracle failed: {runs}"}
    gbs = {ws: round(bucket_bytes / r["median_s"] / 1e9, 3) for ws, r in runs.items() if "median_s" in r}
    return {"value": gbs[1], "unit": "GB/s", "cores": threads, "kind": "port",
            "ws2_per_rank": gbs.get(2), "ws2_cores_per_rank": max(1, threads // 2),
            "cpu_model": _cpu_model(), "host_cpus_visible": os.cpu_count(),
            "sample": f"oracle restatement of group_topk_hook ({ef}, steady state) over gloo on "
                      f"127.0.0.1 on one {label} bucket per rank: ws=1 {runs[1]['calls']} calls "
                      f"(median {runs[1]['median_s'] * 1e3:.1f} ms, {threads} threads), ws=2 "
                      + (f"{runs[2]['calls']} calls (median {runs[2]['median_s'] * 1e3:.1f} ms, "
                         f"{max(1, threads // 2)} threads per rank)" if "median_s" in runs.get(2, {})
                         else f"failed ({runs.get(2)})")
                      + f"; host CPU share {threads} of {os.cpu_count()} visible"}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, cmd, env=None, timeout=None) -> int:
    """Start `cmd` as n rank processes on this node (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT in their environment, as torch.distributed.run sets them) and
    return the first non-zero exit status, else 0.  A failing rank ends the others.  Used by
    `bench.py --gpus N` without a launcher; it runs before this process touches the GPU, and
    the ranks are children (no exec from this process)."""
    import subprocess
    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base["MASTER_PORT"] = str(_free_port())
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                 LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0")
        procs.append(subprocess.Popen(cmd, env=e))
    t_end = None if timeout is None else time.monotonic() + timeout
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:  # one rank failed: the others would wait for it forever
                    q.terminate()
        if t_end is not None and time.monotonic() > t_end:
            for q in live:
                q.kill()
            rc = rc or 124
            break
        time.sleep(0.05)
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ef", default="ef14", choices=["noef", "ef14", "ef21"])
    ap.add_argument("--workload", default="headline", choices=sorted(WORKLOADS) + sorted(DDP_MODELS),
                    help="bucket shape set (headline = the BASELINE metric's bucket)")
    ap.add_argument("--hook", default="arc", choices=["arc", "topk", "randk"],
                    help="arc = ARC-TopK (the metric's codec); topk / randk = the reference's "
                         "baselines (sparse_hook.py; RandK with the device index source)")
    ap.add_argument("--buckets", type=int, default=4,
                    help="buckets per step (a backward's worth, hooked in order as DDP does); "
                         "each is one workload bucket")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                    help="bucket dtype (f32: every BASELINE config; bf16: the Llama driver's default)")
    ap.add_argument("--ratio", type=float, default=0.2)
    ap.add_argument("--r", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-phase-events", action="store_true")
    ap.add_argument("--no-forced-exchange", action="store_true",
                    help="at N = 1, skip the extra timing of the forced-exchange path")
    ap.add_argument("--force-exchange", action="store_true",
                    help="at N = 1, run the N > 1 code path: the native exchange step with its "
                         "all-reduces on one-rank RCCL communicators and the exchange stream")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL (real runs); gloo lets N ranks share one GPU (rehearsal)")
    ap.add_argument("--host-staged", action="store_true",
                    help="D2H + H2D of the packed payload around the all-reduce (NIC model)")
    ap.add_argument("--wire-busbw", type=float, nargs="*", default=[350.0],
                    help="at N = 1: also time the exchange path beside an emulated WIRE_RANKS-rank ring "
                         "all-reduce paced to each of these bus bandwidths (GB/s; none: skip)")
    ap.add_argument("--wire-ranks", type=int, default=8)
    ap.add_argument("--wire-blocks", type=int, default=64,
                    help="workgroups of the emulated collective (its CU footprint)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print each rank's parsed launch (rank, world, master) and exit: no GPU")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N ranks here, one process
        # per GPU, before anything touches the GPU; rank 0 prints the JSON line
        rc = launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:])
        raise SystemExit(rc if rc >= 0 else 128 - rc)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:  # the launch plumbing only (tests): no GPU, no process group
        print(json.dumps({"rank": rank, "world": world, "local_rank": local, "gpus": args.gpus,
                          "steps": args.steps, "warmup": args.warmup, "backend": args.backend,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}),
              flush=True)
        return
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and world > ndev:
        raise SystemExit(f"{world} ranks but {ndev} visible GPUs (RCCL needs one GPU per rank)")
    local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    if args.backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)

    if args.workload in DDP_MODELS:  # configs[1] / configs[3]'s model, as its DDP buckets
        label, model_shapes = DDP_MODELS[args.workload]
        layouts = ddp_buckets(model_shapes())
        shapes = layouts[0]
    else:
        label, shapes = WORKLOADS[args.workload]
        layouts = [shapes] * args.buckets
    nb = len(layouts)
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    eb = 2 if args.dtype == "bf16" else 4
    bytes_per_step = sum(eb * bucket_numel(sh) for sh in layouts)
    n = bucket_numel(shapes)
    bucket_bytes = bytes_per_step // nb
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    # one step = one backward's worth of buckets, hooked in bucket order as DDP does
    buckets = [SyntheticBucket(torch.randn(bucket_numel(sh), device=dev, generator=g).to(dt), sh, index=i,
                               is_last=(i == nb - 1)) for i, sh in enumerate(layouts)]
    if args.hook == "arc":
        st = GroupTopKState(None, r=args.r, compress_ratio=args.ratio, start_compress_iter=0,
                            use_error_feedback=args.ef, seed=1234)
        st.host_staged = args.host_staged
        st.force_exchange = args.force_exchange
        st.defer_decode = True  # step() waits every Future after the last bucket, as DDP's finalize
        if world > 1 or args.force_exchange:
            st.init_exchange_comms(dev)  # collective, before any step (as the registry does)
        hook = group_topk_hook
    else:  # the reference's TopK / RandK baselines on the same buckets (sparse_hook.py)
        from allreducetopk_amd.comm_hooks.sparse_hook import SparseState, sparse_hook_sync
        st = SparseState(None, compress_ratio=args.ratio, start_compress_iter=0,
                         sparse_type="tensor", random=(args.hook == "randk"),
                         use_error_feedback=args.ef, random_seed=1234, index_source="hash")
        hook = sparse_hook_sync

    def step():
        futs = [hook(st, bk) for bk in buckets]
        for f in futs:  # DDP's finalize: the caller's stream waits for every bucket's future
            f.wait()

    # warm-up (EF14: first call creates E; EF21: first call is the dense init)
    for _ in range(max(args.warmup, 2 if args.ef == "ef21" else 1)):
        step()
    torch.cuda.synchronize()
    from allreducetopk_amd.comm_hooks import group_topk_hook_no_reshape as _G
    native_ht = None
    if _G.HOST_TIMES is not None:  # ARCTOPK_HOST_TIMING=1: steady-state calls only
        _G.HOST_TIMES.clear()
        import ctypes
        from allreducetopk_amd import _native as N
        native_ht = N.lib().arctopk_diag_host_times  # (diagnostics section of include/arctopk.h)
        _ns, _calls = (ctypes.c_int64 * 8)(), ctypes.c_int64()
        native_ht(_ns, 8, ctypes.byref(_calls))  # reset
    # the timed region: K steps, no markers
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    host_times = dict(_G.HOST_TIMES) if _G.HOST_TIMES is not None else None
    native_parts = None
    if native_ht is not None:
        native_ht(_ns, 8, ctypes.byref(_calls))
        if _calls.value:
            native_parts = {k: round(_ns[i] / _calls.value / 1e3, 2) for i, k in enumerate(
                ("entry", "encode", "sketch_allreduce", "select", "pack", "packed_allreduce", "finish", "decode"))}

    # At N = 1 the hook's own path has no collectives; the N > 1 code path (one-rank RCCL
    # communicators, packed all-reduce on the exchange stream, deferred decodes) is timed
    # beside it in the same run, so the N = 1 point of a scaling run can be read on either.
    forced = None
    if (world == 1 and args.hook == "arc" and not args.host_staged and not args.force_exchange
            and not args.no_forced_exchange and args.backend == "nccl"):
        st.force_exchange = True
        st.init_exchange_comms(dev)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        fe = time.perf_counter() - t1
        forced = {"value": round(args.steps * bytes_per_step / fe / 1e9, 2),
                  "ms_per_bucket": round(fe / args.steps / nb * 1e3, 4), "steps": args.steps,
                  "hook_path": "exchange (one-rank RCCL communicators)"}
        # the N > 1 code path's own roofline: its algorithmic bytes -- the
        # sketch all-reduced between encode and select, so no keys mode; packed values formed,
        # all-reduced and decoded: (16 + 16 rho) N + sketch + select for EF14 --
        # over the wall time per bucket (the path is device-bound at these sizes: host enqueue
        # below device time, scripts/host_probe.py), PMC bytes per call beside it
        fx_alg = [algorithmic_bytes(args.ef, sh, args.ratio, args.r, eb, keyed=False) for sh in layouts]
        fx_bytes = sum(d["total"] for d in fx_alg) / nb
        fx_s = fe / args.steps / nb
        tr, tr_src, tr_match = pmc_call_traffic(args.workload + ("_bf16" if args.dtype == "bf16" else ""), args.ef)
        forced["roofline"] = {
            "bound": "hbm", "algorithmic_bytes_per_call": int(fx_bytes),
            "bytes_formula": {"ef14": "(16 + 16 rho) N + sketch + select", "noef": "(8 + 12 rho) N + sketch + select",
                              "ef21": "(16 + 28 rho) N + sketch + select"}[args.ef],
            "wall_us_per_call": round(fx_s * 1e6, 1), "achieved": round(fx_bytes / fx_s / 1e9, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(fx_bytes / fx_s / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": tr, "traffic_source": tr_src, "traffic_lib_match": tr_match,
            "traffic_ratio": round(tr / fx_bytes, 3) if tr else None}
        st.force_exchange = False

    # The same exchange path beside an emulated N-rank wire (exchange.Comm.wire): each all-reduce
    # costs this GPU what a ring all-reduce over WIRE_RANKS GPUs would -- 2 (R-1)/R of the buffer
    # read and rewritten in HBM by WIRE_BLOCKS workgroups, paced to the bus bandwidth -- so the
    # codec's kernels run beside the collective's CU and HBM footprint.
    wire = []
    if (world == 1 and args.hook == "arc" and not args.host_staged and not args.force_exchange
            and args.backend == "nccl"):
        for bw in args.wire_busbw or []:
            st.reset_exchange_comms()
            st.emulate_wire = dict(ranks=args.wire_ranks, busbw_gbs=bw, latency_us=15.0, blocks=args.wire_blocks)
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            fe = time.perf_counter() - t1
            v = args.steps * bytes_per_step / fe / 1e9
            # the wire alone: each bucket's two ring all-reduces (sketch, packed values) at busBW
            from allreducetopk_amd.comm_hooks.group_topk_hook_no_reshape import _geometry
            R_ = args.wire_ranks
            wire_s = 0.0
            for sh in layouts:
                ab = algorithmic_bytes(args.ef, sh, args.ratio, args.r, eb)
                k_bytes = ab["pack"] // {"noef": 2, "ef14": 3}.get(args.ef, 4)  # selected elements x eb
                sk_bytes = sum(eb * _geometry(s_)[1] * (1 if len(s_) == 1 else args.r) for s_ in sh)
                for nbytes in (sk_bytes, k_bytes):
                    wire_s += 15e-6 + 2 * (R_ - 1) / R_ * nbytes / (bw * 1e9)
            ceiling = bytes_per_step / wire_s / 1e9
            wire.append({"busbw_gbs": bw, "emulated_ranks": args.wire_ranks, "blocks": args.wire_blocks,
                         "latency_us": 15.0, "per_gpu_value": round(v, 2),
                         "implied_aggregate": round(args.wire_ranks * v, 2),
                         "ms_per_bucket": round(fe / args.steps / nb * 1e3, 4),
                         "wire_ceiling_per_gpu": round(ceiling, 2),
                         "frac_of_wire_ceiling": round(v / ceiling, 4)})
        st.reset_exchange_comms()
        st.emulate_wire = None

    phase_ms = {}
    light = {}
    sample_steps = 0
    if not args.no_phase_events and args.hook == "arc":
        # a separate marker pass (not in `value`): device-scope HIP events recorded by the native
        # step itself on the streams the kernels run on.  Each marker between two kernels idles
        # the GPU a few us, so they are sparse: on every 2nd call alternately a marker after the
        # decode (the device timeline between two of them, 4 calls apart, over 4 = the hook's
        # device time per call, marker costs amortised) and the encode alone (after the V draw
        # .. after the encode); the full per-phase breakdown on every 32nd call
        st.hook_events = hs = []
        st.hook_event_every = 2
        st.phase_events = None
        pe = st.phase_event_every = 32
        sample_steps = max(args.steps, 16)
        for _ in range(sample_steps):
            step()
        torch.cuda.synchronize()
        # the per-phase breakdown from calls whose decode runs inline (with deferred decodes a
        # step's decode lands in a later call, so its markers would bracket other work)
        st.hook_events = None
        st.phase_events = pe_list = []
        st.phase_event_every = 1
        st.defer_decode = False
        for _ in range(4):
            step()
        torch.cuda.synchronize()
        st.defer_decode = True
        st.phase_events = None
        if pe_list:
            order = [p for p in ["start", "draw", "encode", "sketch_allreduce", "select", "pack", "h2d",
                                 "packed_allreduce", "decode"] if p in pe_list[0]]
            if world == 1 and not args.force_exchange:  # no collectives at world size 1
                order = [p for p in order if p not in ("sketch_allreduce", "packed_allreduce")]
            for a, b in zip(order[:-1], order[1:]):
                phase_ms[b] = statistics.median(ev[a].elapsed_time(ev[b]) for ev in pe_list)
            phase_ms["hook_device_total"] = statistics.median(
                ev["start"].elapsed_time(ev["decode"]) for ev in pe_list)
        he = [ev for ev in hs if "encode" in ev]
        hd = sorted((ev for ev in hs if "decode" in ev), key=lambda ev: ev["_call"])
        # consecutive decode markers with no full-phase sample (every 32nd call) between them
        per_call = [a_["decode"].elapsed_time(b_["decode"]) / (b_["_call"] - a_["_call"])
                    for a_, b_ in zip(hd, hd[1:])]
        if he and per_call:
            light = {"samples": len(he), "hook_samples": len(per_call),
                     "encode": statistics.median(ev["draw"].elapsed_time(ev["encode"]) for ev in he),
                     "hook": statistics.median(per_call),
                     "calls_apart": hd[1]["_call"] - hd[0]["_call"] if len(hd) > 1 else None}
    if args.hook != "arc":
        hook_path = "sparse_hook_sync"
    elif args.host_staged:
        hook_path = "phase (host-staged)"
    else:
        hook_path = "exchange" if (world > 1 or args.force_exchange) else "step"
    value = world * args.steps * bytes_per_step / elapsed / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    per_bucket = [algorithmic_bytes(args.ef, sh, args.ratio, args.r, eb, keyed=(hook_path == "step"))
                  for sh in layouts]
    alg = {k: sum(d[k] for d in per_bucket) / nb for k in per_bucket[0]}  # mean over the step's buckets
    roof = None
    if light:
        enc_s = light["encode"] / 1e3
        ach = alg["encode"] / enc_s / 1e9
        roof = {"bound": "hbm", "kernel": "k_encode (EF pre-apply + rank-r sketch)",
                "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "algorithmic_bytes_per_launch": alg["encode"],
                "avg_launch_us": round(light["encode"] * 1e3, 2),
                "event_scope": "device", "statistic": "median",
                "event_samples": light["samples"]}
        hook_s = light["hook"] / 1e3
        wall_s = elapsed / args.steps / nb
        # headline fraction: read + write algorithmic bytes of the whole hook (V draw, encode,
        # select, pack, decode) over its device time; read_frac: the bytes it reads only
        # (the north star's "HBM-read roofline"), over the same time
        roof["hook"] = {"algorithmic_bytes": alg["total"], "read_bytes": alg["read"],
                        "device_us": round(hook_s * 1e6, 1),
                        "device_time": f"device timeline between decode-end markers "
                                       f"{light['calls_apart']} calls apart, per call (median)",
                        "event_samples": light["hook_samples"],
                        "achieved": round(alg["total"] / hook_s / 1e9, 1),
                        "frac": round(alg["total"] / hook_s / 1e9 / HBM_PEAK_GBS, 4),
                        "read_frac": round(alg["read"] / hook_s / 1e9 / HBM_PEAK_GBS, 4),
                        "wall_us": round(wall_s * 1e6, 1),
                        "wall_frac": round(alg["total"] / wall_s / 1e9 / HBM_PEAK_GBS, 4),
                        "headline": "frac (read + write bytes over device time)"}
        # the north star names the HBM-read roofline; the headline fraction here
        # counts read + write bytes (every phase writes as much as it must), read_frac only reads
        roof["headline_choice"] = ("frac = encode read+write bytes over its duration; hook.frac = the whole "
                                   "codec's read+write bytes over its device time; hook.read_frac = its "
                                   "read bytes only (the north star's 'HBM-read roofline' reading)")
        roof["read_frac"] = roof["hook"]["read_frac"]
    if roof is not None:
        roof["traffic"], roof["traffic_source"], roof["traffic_lib_match"] = pmc_traffic(
            args.workload + ("_bf16" if args.dtype == "bf16" else ""), args.ef, "k_encode", world)
        if roof["traffic"] is None and world > 1:
            roof["traffic_source"] = f"none: no PMC profile taken at N = {world} (N = 1 files are not reused)"
    if args.hook != "arc":
        # the baselines' roofline: their minimum bytes per call over the wall time per bucket
        # (no markers on this path; the step is device-bound, so wall ~ device time)
        k_el = sum(max(1, int(bucket_numel([s_]) * args.ratio)) for sh in layouts for s_ in sh) / nb
        sb = sparse_algorithmic_bytes(args.hook, args.ef, bytes_per_step // nb // eb, int(k_el), world, eb)
        if sb is not None:
            wall_s = elapsed / args.steps / nb
            ach = sb / wall_s / 1e9
            roof = {"bound": "hbm", "kernel": f"whole {args.hook} hook per bucket (wall time)",
                    "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                    "algorithmic_bytes_per_call": sb, "wall_us_per_bucket": round(wall_s * 1e6, 1),
                    "formula": ("(28 + (8 + 16 ws) rho) B/elem (SURVEY 8d)" if args.hook == "topk"
                                else "(16 + 28 rho) B/elem (fused RandK minimum)")}
            # PMC bytes per call of the same command (scripts/profile.sh with BENCH_ARGS="--hook
            # <hook>", CALL_KERNELS=k_scatter_first): profiles/<round>/pmc_<workload>_<ef>_<hook>.json
            if world == 1:
                tr, tr_src, tr_match = pmc_call_traffic(args.workload + ("_bf16" if args.dtype == "bf16" else ""),
                                                        args.ef, tag=args.hook)
                roof.update({"traffic": tr, "traffic_source": tr_src, "traffic_lib_match": tr_match,
                             "traffic_ratio": round(tr / sb, 3) if tr else None})
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (N(0,1) fp32 gradients, per-rank seed)",
        "config": {"workload": f"{'arctopk' if args.hook == 'arc' else args.hook}_{args.ef}_{nb}x_{label}"
                               + ("_as_bf16" if args.dtype == "bf16" else "")
                               + ("_host_staged" if args.host_staged else ""),
                   "compress_ratio": args.ratio, "r": args.r, "use_error_feedback": args.ef,
                   "bucket_bytes": bucket_bytes, "buckets_per_step": nb,
                   "parallelism": f"dp{world}",
                   "hook_path": hook_path,
                   "collectives": ("none (world size 1: both all-reduces are identities)"
                                   if hook_path == "step" else
                                   ("RCCL" if args.backend == "nccl" else "gloo (rehearsal)")
                                   + f" all_reduce over {world} rank(s): sketch (own communicator) + "
                                     "packed values, issued by the native exchange step; packed "
                                     "all-reduce + decode on the exchange stream, overlapping the "
                                     "next bucket")},
        "per_gpu_value": round(value / world, 2),
        "forced_exchange": forced,
        "emulated_wire": wire or None,
        "ms_per_bucket": round(ms_per_step / nb, 4),
        "phase_ms": {k: round(v, 4) for k, v in phase_ms.items()},
        "phase_ms_note": "separate pass, every call marked, decodes inline (not deferred)" if phase_ms else None,
        "roofline": roof,
        "algorithmic_bytes_per_call": {k: int(v) for k, v in alg.items()},
        "cpu_baseline": None if world == 1 else {
            "value": None, "unit": "GB/s", "cores": 0, "kind": "port",
            "sample": "not timed at N > 1: the CPU baseline runs on rank 0 of the N = 1 line only "
                      "(bench contract); see that line's cpu_baseline (ws 1 and ws 2 over gloo)"},
    }
    if world > 1:
        out["value_semantics"] = (f"value = bucket bytes of all {world} ranks / wall time (whole-job "
                                  f"aggregate, bench contract); per_gpu_value = value / {world}")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.ef, args.cpu_seconds, args.workload, label,
                                           eb * bucket_numel(shapes), args.hook)
    if host_times is not None and rank == 0:  # ARCTOPK_HOST_TIMING=1: host us per hook call
        calls = max(1, args.steps * nb)
        print("host_us_per_call " + json.dumps({k: round(v / calls * 1e6, 1)
                                                for k, v in host_times.items()}), flush=True)
        if native_parts:
            print("native_step_host_us " + json.dumps(native_parts), flush=True)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
