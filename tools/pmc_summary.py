#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs: per kernel (name prefix),
median over dispatches of each counter.  Usage: pmc_summary.py DIR... [--match S]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = None
if "--match" in sys.argv:
    match = sys.argv[sys.argv.index("--match") + 1]
    args = [a for a in args if a != match]
vals = defaultdict(lambda: defaultdict(list))
for d in args:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if match and match not in name:
                continue
            key = (name, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            per[key]["_dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for (name, _), cs in per.items():
            for c, v in cs.items():
                vals[name][c].append(v)
for name, cs in vals.items():
    print(name)
    for c in sorted(cs):
        print(f"  {c:28s} {statistics.median(cs[c]):16.0f}  (n={len(cs[c])})")
