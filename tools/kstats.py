#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv as a short table (ms)."""
import csv
import sys

for f in sys.argv[1:]:
    print(f)
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        print("%-100s %6s %9.3f %9.3f %9.3f %6.2f%%" % (
            r["Name"][:100], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["MinNs"]) / 1e6,
            float(r["MaxNs"]) / 1e6, float(r["Percentage"])))
