"""Top kernels of a rocprofv3 kernel_stats.csv (µs): total, calls, average."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / 1e3:10.1f} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.2f}  {r['Name'][:100]}")
