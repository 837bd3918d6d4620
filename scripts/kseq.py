"""Kernel launches of one hook call (the last one in the trace) with durations and grids,
plus per-kernel averages over the whole trace."""
import collections
import csv
import os
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:14]:
    print(f"  {k:60s} n={len(v):5d} avg={sum(v) / len(v):8.2f} us")
enc = []  # the call's first kernel: the encode (ARC-TopK), else the EF fold / pre-apply (TopK / RandK)
for anchor in ("k_encode", "k_ef14_fold", "k_ef_apply", "k_ms_init"):
    enc = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    if enc:
        break
enc = enc or [0]
back = int(os.environ.get("KSEQ_BACK", "2"))  # encodes back from the end (one step: buckets + 1)
start = enc[-back] if len(enc) >= back else enc[0]
print("  -- one call:")
t0 = int(rows[start]["Start_Timestamp"])
for r in rows[start:start + 40]:
    if "k_encode" in r["Kernel_Name"] and int(r["Start_Timestamp"]) > t0 and r is not rows[start]:
        if rows.index(r) > start + 1 and "k_encode" in rows[rows.index(r) - 1]["Kernel_Name"]:
            pass
    q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
    print(f"    +{(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} us  {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.2f} us  "
          f"q{q:>3s} {r['Kernel_Name'].split('(')[0].replace('void ', '')[:50]:50s} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} lds={r['LDS_Block_Size']}")
