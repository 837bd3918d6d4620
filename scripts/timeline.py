"""One step's kernel timeline from a rocprofv3 kernel trace (every stream): the step starts at the
Nth launch of the first bucket's encode (grid `--grid`) before the first emulated-wire kernel.
    python scripts/timeline.py run_kernel_trace.csv --grid 1280 --nth 6"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--grid", type=int, required=True, help="grid size X of the step's first encode")
ap.add_argument("--nth", type=int, default=5)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
stop = next((i for i, r in enumerate(rows) if "k_wire" in r["Kernel_Name"]), len(rows))
starts = [i for i, r in enumerate(rows[:stop]) if "k_encode" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == a.grid]
i0, i1 = starts[a.nth], starts[a.nth + 1]
t0 = int(rows[i0]["Start_Timestamp"])
busy_end = 0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0][-34:]
    gap = (s - busy_end) / 1e3 if s > busy_end else 0.0
    print(f"  {s / 1e3:8.1f} -> {e / 1e3:8.1f} us  ({(e - s) / 1e3:6.2f})  q{q:>2s}  idle-before {gap:5.1f}  {name:34s} grid={r['Grid_Size_X']}")
    busy_end = max(busy_end, e)
print(f"  step: {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.1f} us")
