"""Print a window of a rocprofv3 kernel trace (sorted by start): stream, queue, start/end (us
relative to the window's first kernel), duration, kernel.  Usage: trace_window.py CSV ENCODE_INDEX N"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if r['Kernel_Name'] == 'k_encode']
start = idx[int(sys.argv[2])]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
t0 = int(rows[start]['Start_Timestamp'])
last_end = {}
for r in rows[start:start + n]:
    s = int(r['Start_Timestamp']) - t0
    e = int(r['End_Timestamp']) - t0
    q = r['Queue_Id']
    gap = (s - last_end[q]) / 1000 if q in last_end else 0.0
    last_end[q] = e
    print(f"s{r['Stream_Id']:>3} q{q:>2} {s / 1000:9.1f} {e / 1000:9.1f} {(e - s) / 1000:7.1f} gap{gap:6.1f}  "
          f"{r['Kernel_Name'][:40]} grid={r['Grid_Size_X']}")
