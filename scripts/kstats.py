"""Print a rocprofv3 kernel_stats.csv sorted by total time: name, calls, average us."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{r['Name'][:90]:90s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} us")
