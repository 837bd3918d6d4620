"""Summary of a rocprofv3 kernel trace of bench.py beside the emulated wire:
per-kernel statistics, the packed all-reduce kernels' durations against their pace, and a
timeline excerpt of the last step (start / end in us from the excerpt's first kernel, queue).

    python scripts/wire_trace_summary.py TRACE_DIR [paced_us]
"""
import csv
import glob
import os
import statistics as st
import sys

d = sys.argv[1]
paced = float(sys.argv[2]) if len(sys.argv) > 2 else None
print(f"# {d}")
with open(glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]) as fh:
    print("kernel statistics (rocprofv3 --stats):")
    for r in csv.DictReader(fh):
        print(f"  {r['Name'][:40]:40s} calls {int(r['Calls']):5d}  avg {float(r['AverageNs']) / 1e3:8.1f} us  "
              f"min {int(r['MinNs']) / 1e3:8.1f}  max {int(r['MaxNs']) / 1e3:8.1f}")
with open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]) as fh:
    rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"] and "elementwise" not in r["Kernel_Name"]]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
wires = [dur(r) for r in rows if "k_wire" in r["Kernel_Name"]]
big = [w for w in wires if w > 100]
small = [w for w in wires if w <= 100]
if big:
    print(f"packed all-reduce (wire) kernels: {len(big)}, median {st.median(big):.1f} us, "
          f"min {min(big):.1f}, max {max(big):.1f}" + (f" (paced {paced:.0f} us)" if paced else ""))
if small:
    print(f"sketch all-reduce (wire) kernels: {len(small)}, median {st.median(small):.1f} us")
print("timeline, last 24 kernels (us; queue):")
t0 = int(rows[-24]["Start_Timestamp"])
for r in rows[-24:]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    print(f"  {s:9.1f} {s + dur(r):9.1f} {dur(r):7.1f}  q{r['Queue_Id']}  {r['Kernel_Name'].split('(')[0][:40]}")
