"""Per-call device time by phase from rocprofv3 kernel traces of bench.py runs (one trace
directory per workload, written by scripts/trace_wl.sh).  Trace durations carry no marker
overhead, unlike bench.py's sampled event markers.

  python scripts/trace_table.py gpurun_out/trace_<tag> ...

calls = k_encode launches.  Columns: average µs per launch of each phase's kernels summed per
call; `select` counts every select launch (a deferred decode that rode in one is inside it:
`ride` says how many calls' decodes rode); `device` = all codec kernel time per call; hook
frac = the codec's algorithmic bytes per call (bench.py) / device time / 8 TB/s."""
import csv
import glob
import json
import os
import sys

PHASES = {
    "draw": ("k_draw_v",),
    "encode": ("k_encode",),
    "select": ("k_select_small", "k_arc_keys", "k_arc_compact", "k_arc_refine", "k_arc_write",
               "k_arc_write_fused", "k_select_small_dec"),
    "pack": ("k_pack",),
    "decode": ("k_decode",),
    "rccl": ("ncclDevKernel", "ncclKernel"),
}


def kname(r):
    return r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip()


def phase_of(name):
    for ph, names in PHASES.items():
        if any(name == n or name.startswith(n + "_") or (ph == "rccl" and name.startswith(n)) for n in names):
            return ph
    return None


print(f"{'workload':58s} {'path':9s} {'GB/s':>7s} {'calls':>5s} {'enc':>6s} {'sel':>6s} {'pack':>6s} "
      f"{'dec':>6s} {'rccl':>6s} {'device':>7s} {'ride':>5s} {'encTB/s':>7s} {'hook':>5s}")
for d in sys.argv[1:]:
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not tr:
        continue
    rows = list(csv.DictReader(open(tr[0])))
    b = None
    try:
        for line in open(os.path.join(d, "bench.log")):
            if line.startswith('{"metric"'):
                b = json.loads(line)
    except (OSError, ValueError):
        pass
    if b is None:
        continue
    tot = {p: 0.0 for p in PHASES}
    n = {p: 0 for p in PHASES}
    for r in rows:
        ph = phase_of(kname(r))
        if ph:
            tot[ph] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            n[ph] += 1
    calls = n["encode"]
    if not calls:
        continue
    per = {p: tot[p] / calls for p in PHASES}
    dev = sum(per.values())
    ab = b.get("algorithmic_bytes_per_call") or {}
    alg, enc_alg = ab.get("total"), ab.get("encode")
    enc_avg = tot["encode"] / calls
    ride = calls - n["decode"]
    hook = alg / (dev * 1e-6) / 8e12 if alg else float("nan")
    enc_tbs = enc_alg / (enc_avg * 1e-6) / 1e12 if enc_alg else float("nan")
    print(f"{b['config']['workload'][:58]:58s} {b['config'].get('hook_path', '?')[:9]:9s} {b['value']:7.1f} {calls:5d} "
          f"{per['encode'] + per['draw']:6.1f} {per['select']:6.1f} {per['pack']:6.1f} {per['decode']:6.1f} "
          f"{per['rccl']:6.1f} {dev:7.1f} {ride:5d} {enc_tbs:7.2f} {hook:5.3f}")
