"""Per-call gaps on the GPU timeline of a kernel trace: encode-to-encode spacing and the
idle time before each encode (after the previous kernel on the stream)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
enc = [i for i, k in enumerate(ks) if "k_encode" in k[2]]
sp = [(ks[b][0] - ks[a][0]) / 1e3 for a, b in zip(enc, enc[1:])]
idle = [(ks[i][0] - ks[i - 1][1]) / 1e3 for i in enc[1:]]
print(f"calls {len(enc)}  spacing median {statistics.median(sp):.1f} us  p90 {sorted(sp)[int(.9 * len(sp))]:.1f}"
      f"  idle-before-encode median {statistics.median(idle):.1f} p90 {sorted(idle)[int(.9 * len(idle))]:.1f} max {max(idle):.1f}")
big = sorted(range(len(idle)), key=lambda i: -idle[i])[:8]
print("largest idle gaps (us):", [round(idle[i], 1) for i in big])
# idle time before each kernel kind (GPU timeline, any stream)
kinds = {}
for i in range(1, len(ks)):
    nm = ks[i][2].replace("void ", "").replace("(anonymous namespace)::", "").split("<")[0].split("(")[0]
    kinds.setdefault(nm, []).append((ks[i][0] - ks[i - 1][1]) / 1e3)
for nm, v in sorted(kinds.items(), key=lambda kv: -sum(kv[1]))[:8]:
    v = sorted(v)
    print(f"  idle before {nm[:40]:40s} n={len(v):4d} median {v[len(v) // 2]:7.1f} p90 {v[int(.9 * len(v))]:7.1f} sum {sum(v):9.1f}")
