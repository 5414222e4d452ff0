#!/usr/bin/env python3
"""Counter totals of the last dispatch of the kernels matching a substring:
python tools/pmc_sum.py <run_counter_collection.csv> [<more.csv> ...] --kernel SUBSTR"""
import csv
import sys

args = sys.argv[1:]
sub = args[args.index("--kernel") + 1]
files = [a for a in args if a.endswith(".csv")]
for f in files:
    rows = [r for r in csv.DictReader(open(f)) if sub in r["Kernel_Name"]]
    last = max(int(r["Dispatch_Id"]) for r in rows)
    agg = {}
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k, v in agg.items():
        print(f"{k:32s} {v:14.4g}")
