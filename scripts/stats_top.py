#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 ``*_kernel_stats.csv`` (percent, calls, avg us, name)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.1f} ms")
for r in rows[:n]:
    print(f"{float(r['Percentage']):6.2f}% {int(r['Calls']):6d} {float(r['AverageNs']) / 1000:8.1f}us  {r['Name'][:100]}")
