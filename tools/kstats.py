#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats kernel_stats.csv: python tools/kstats.py <csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f'{r["Name"][:80]:80s} {int(r["Calls"]):5d} {float(r["AverageNs"]) / 1e3:9.1f} us  tot {float(r["TotalDurationNs"]) / 1e6:8.2f} ms')
