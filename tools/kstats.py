#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv as a per-unit table: tools/kstats.py CSV [units] [top]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
units = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / units / 1e6:8.3f} ms/unit {r['Calls']:>6} calls {float(r['AverageNs']) / 1e3:9.1f} us "
          f"{float(r['Percentage']):5.1f}%  {r['Name'][:90]}")
print(f"total {tot / units / 1e6:.3f} ms/unit")
