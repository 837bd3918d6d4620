"""bench.py's own launcher (`--gpus N` without torch.distributed.run) and its bench-line
helpers, on CPU: the rank environment, argument pass-through, failure propagation, and the
baselines' algorithmic bytes."""
import json
import os
import subprocess
import sys
import time

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launch_ranks_sets_the_rank_environment(tmp_path):
    code = ("import os, sys; open(os.path.join(sys.argv[1], os.environ['RANK']), 'w').write("
            "' '.join(os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')))")
    assert bench.launch_ranks(3, [sys.executable, "-c", code, str(tmp_path)]) == 0
    seen = [open(tmp_path / str(r)).read().split() for r in range(3)]
    ports = {s[4] for s in seen}
    assert len(ports) == 1
    for r, s in enumerate(seen):
        assert s[:4] == [str(r), str(r), "3", "127.0.0.1"]


def test_launch_ranks_propagates_a_failing_rank_and_stops_the_others():
    code = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1': sys.exit(3)\n"
            "time.sleep(60)")
    t0 = time.monotonic()
    assert bench.launch_ranks(2, [sys.executable, "-c", code]) == 3
    assert time.monotonic() - t0 < 30


def test_bench_gpus_n_without_a_launcher_spawns_n_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", "--steps", "5",
                        "--warmup", "1", "--dry-run"], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    for d in lines:
        assert d["world"] == 2 and d["gpus"] == 2 and d["steps"] == 5 and d["warmup"] == 1
        assert d["backend"] == "gloo" and d["master"].startswith("127.0.0.1:")
    assert lines[0]["master"] == lines[1]["master"]


def test_bench_refuses_a_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dry-run"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_sparse_algorithmic_bytes_follow_the_survey_formula():
    n, k = 67_108_864, 13_421_760
    assert bench.sparse_algorithmic_bytes("topk", "ef14", n, k, 1) == 28 * n + 24 * k
    assert bench.sparse_algorithmic_bytes("topk", "ef14", n, k, 8) == 28 * n + (8 + 128) * k
    assert bench.sparse_algorithmic_bytes("randk", "ef14", n, k, 8) == 16 * n + 28 * k
    assert bench.sparse_algorithmic_bytes("topk", "ef21", n, k, 1) is None


def test_pmc_traffic_is_never_the_n1_file_at_n_gt_1():
    assert bench.pmc_traffic("headline", "ef14", "k_encode", 2) == (None, None, None)


def test_keys_mode_algorithmic_bytes():
    """At world size 1 the multi-block items' encode writes 4-B keys instead of their sketch rows
    (keys mode): the encode and select bytes drop by (4 r - 4) B per such row, nothing else."""
    import bench
    conv = [[512, 512, 3, 3]] * 2  # ND: m = 18, n = 131,072 rows each (multi-block items)
    a, b = bench.algorithmic_bytes("ef21", conv, 0.2, 4), bench.algorithmic_bytes("ef21", conv, 0.2, 4, keyed=True)
    rows = 2 * 131072
    assert a["encode"] - b["encode"] == (16 - 4) * rows
    assert a["select"] - b["select"] == (16 - 4) * rows
    assert a["pack"] == b["pack"] and a["decode"] == b["decode"]
    # EF14 / noef at world size 1: no packed copy -- the decode takes the selected rows from E
    # (read and zeroed) and writes the bucket: (4 + 8 rho) B per element instead of (4 + 16 rho)
    n_el, k_el = 2 * 512 * 512 * 9, 2 * int(131072 * 0.2) * 18
    c = bench.algorithmic_bytes("ef14", conv, 0.2, 4, keyed=True)
    assert c["pack"] == 0 and c["decode"] == 4 * (n_el + 2 * k_el)
    assert bench.algorithmic_bytes("noef", conv, 0.2, 4, keyed=True)["decode"] == 4 * (n_el - k_el)
    head = [[2048, 2048]] * 16  # single-block items: keys mode does not apply
    h0, h1 = bench.algorithmic_bytes("ef14", head, 0.2, 4), bench.algorithmic_bytes("ef14", head, 0.2, 4, keyed=True)
    assert h0["encode"] == h1["encode"] and h0["select"] == h1["select"]
    # a tensor beside a multi-block item joins the multi-block batch past 4,096 rows
    mixed = [[20000, 8], [5000, 8], [100, 8]]
    c, d = bench.algorithmic_bytes("ef21", mixed, 0.2, 4), bench.algorithmic_bytes("ef21", mixed, 0.2, 4, keyed=True)
    assert c["encode"] - d["encode"] == 12 * (20000 + 5000)


def test_ddp_model_workloads_match_the_reference_models():
    """configs[1] / configs[3] as DDP buckets: ResNet-18 62 tensors,
    11,173,962 parameters, 3 buckets; CIFAR-100 ResNet-50 161 tensors, 23,705,252 parameters,
    5 buckets of at most 26 MiB; every ND tensor divides into rows of 2 t^2 (cal_k's reshape)."""
    from allreducetopk_amd.bucket import bucket_numel
    from workloads import DDP_MODELS, ddp_buckets
    expect = {"resnet18_ddp": (62, 11_173_962, 3), "resnet50_ddp": (161, 23_705_252, 5)}
    for name, (label, fn) in DDP_MODELS.items():
        shapes = fn()
        layouts = ddp_buckets(shapes)
        assert (len(shapes), bucket_numel(shapes), len(layouts)) == expect[name], name
        assert sorted(map(tuple, (s for b in layouts for s in b))) == sorted(map(tuple, shapes))
        assert max(bucket_numel(b) * 4 for b in layouts) <= 26 << 20
        for s in shapes:
            if len(s) > 2:
                assert bucket_numel([s]) % (2 * s[-1] ** 2) == 0, s
