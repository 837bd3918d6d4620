"""Per-kernel times of one sel_profile.py run, split into the ARC (ResNet bucket) and
TopK halves of the trace, plus the launch sequence of the last select of each."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last_dec = max(i for i, r in enumerate(rows) if "k_decode" in r["Kernel_Name"])
for name, sub in [("ARC resnet", rows[:last_dec + 1]), ("TopK", rows[last_dec + 1:])]:
    agg = collections.defaultdict(list)
    for r in sub:
        n = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        agg[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("==", name)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:40s} n={len(v):4d} avg={sum(v) / len(v):8.2f} us  per-call={sum(v) / 10:8.2f}")
    seq = [(r["Kernel_Name"].split("(")[0].replace("void ", "")[:40],
            round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 2))
           for r in sub if "k_ms" in r["Kernel_Name"] or "arc_keys" in r["Kernel_Name"]]
    print("   last select:", seq[-12:])
