"""Merge kernel and memory-copy traces: the last ~2 calls' kernels and copies in time order,
plus the HIP API calls that enqueue copies / wait on events."""
import csv
import glob
import sys

d = sys.argv[1]
def rows(pat):
    f = glob.glob(f"{d}/**/{pat}", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []
ev = []
for r in rows("*kernel_trace.csv"):
    nm = r["Kernel_Name"].replace("void ", "").replace("arctopk::", "").replace("(anonymous namespace)::", "").split("(")[0]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K s" + r["Stream_Id"] + " " + nm[:40]))
for r in rows("*memory_copy_trace.csv"):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C s" + r["Stream_Id"] + " " + r.get("Direction", "")[12:]))
api = rows("*hip_api_trace.csv")
for r in api:
    if any(k in r["Function"] for k in ("Memcpy", "WaitEvent", "EventRecord", "LaunchKernel", "ExtModuleLaunch")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A " + r["Function"][:30] + " tid" + r.get("Thread_Id", "")))
ev.sort()
enc = [i for i, e in enumerate(ev) if "k_encode" in e[2]]
start = enc[-3]
t0 = ev[start][0]
for s, e, name in ev[start - 40:start + 60]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name}")
