"""Summarize rocprofv3 CSVs: per-kernel launches, avg duration, and per-launch HBM bytes
from FETCH_SIZE (x2: gfx950 reports half of a wide coalesced stream, MI355X_MICROARCH.md
HBM section) and WRITE_SIZE (both counters in KiB)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(root, pattern), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


stats = rows("trace/**/*kernel_stats.csv")
print("== kernel stats (trace pass) ==")
for r in sorted(stats, key=lambda r: -float(r.get("TotalDurationNs", 0) or 0)):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:9.2f} us  "
          f"total% {float(r.get('Percentage', 0)):6.2f}")


def counter(pattern, name):
    acc = defaultdict(list)
    for r in rows(pattern):
        if r.get("Counter_Name") == name:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


fetch = counter("fetch/**/*counter_collection.csv", "FETCH_SIZE")
write = counter("write/**/*counter_collection.csv", "WRITE_SIZE")
print("== HBM traffic per launch (PMC passes; FETCH_SIZE x2 correction) ==")
for k in sorted(set(fetch) | set(write)):
    f = fetch.get(k, [])
    w = write.get(k, [])
    fa = 2 * 1024 * sum(f) / len(f) if f else float("nan")
    wa = 1024 * sum(w) / len(w) if w else float("nan")
    print(f"{k[:60]:60s} launches {len(f):5d}  read {fa/1e6:10.2f} MB  write {wa/1e6:10.2f} MB  "
          f"total {(fa + wa)/1e6:10.2f} MB")

# machine-readable per-launch traffic for bench.py's roofline.traffic
out = {}
for k in sorted(set(fetch) | set(write)):
    f = fetch.get(k, [])
    w = write.get(k, [])
    name = k.split("(")[0].split("<")[0].replace("void ", "").strip()
    if f and w:
        ent = out.setdefault(name, {"launches": 0, "read_bytes": 0.0, "write_bytes": 0.0})
        ent["launches"] += len(f)
        ent["read_bytes"] += 2 * 1024 * sum(f)
        ent["write_bytes"] += 1024 * sum(w)
for ent in out.values():
    ent["read_bytes"] = round(ent["read_bytes"] / ent["launches"])
    ent["write_bytes"] = round(ent["write_bytes"] / ent["launches"])
    ent["bytes_per_launch"] = ent["read_bytes"] + ent["write_bytes"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from allreducetopk_amd.build import embedded_hash  # noqa: E402
# per hook call: every libarctopk kernel's bytes (k_*; torch's own fills / copies / randn excluded)
# over the calls, counted as encode launches (one per call; profile runs skip the marker pass)
# (CALL_KERNELS: the kernels launched once per call, e.g. k_scatter_first for the TopK / RandK hooks)
call_kernels = os.environ.get("CALL_KERNELS", "k_encode,k_encode_short,k_encode_carry").split(",")
calls = sum(v["launches"] for k, v in out.items() if k in call_kernels)
per_call = None
if calls:
    tot = sum(v["bytes_per_launch"] * v["launches"] for k, v in out.items() if k.startswith("k_"))
    per_call = {"calls": calls, "bytes": round(tot / calls),
                "kernels": sorted(k for k in out if k.startswith("k_"))}
    print(f"== per hook call: {calls} calls, {tot / calls / 1e6:.2f} MB of libarctopk kernel traffic each ==")
with open(os.path.join(root, "pmc_per_launch.json"), "w") as fh:
    json.dump({"note": "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads) + WRITE_SIZE, "
                       "KiB -> bytes, averaged per launch; separate --pmc passes",
               "lib_hash": embedded_hash(),  # the libarctopk.so source hash these counters were taken on
               "kernels": out, "per_call": per_call}, fh, indent=1)
