#!/usr/bin/env python3
"""Effective shader clock per dispatch from a rocprofv3 --pmc GRBM_GUI_ACTIVE
--kernel-trace run: GRBM_GUI_ACTIVE (summed over the 8 XCDs, so / 8) over the
dispatch's duration.  With --context, each dispatch of the named kernel is
labelled by the kernel dispatched before it, skipping rs_sets_prep (and a
gap > 1 ms before it is labelled "idle").  Prints one JSON line: median clock (GHz) per (kernel,
context), with counts.

usage: clock_by_kernel.py RUN_DIR [--kernel SUBSTR ...] [--context]"""
import argparse
import csv
import glob
import json
import os
import statistics


def short(name):
    n = name
    for p in ("void ", "(anonymous namespace)::", "uplink_ec::", "enc::", "at::native::"):
        n = n.replace(p, "")
    return n.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--kernel", nargs="*", default=[])
    ap.add_argument("--context", action="store_true")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.run_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        d = int(r["Dispatch_Id"])
        rows[d] = (r["Kernel_Name"], float(r["Counter_Value"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    order = sorted(rows)
    out = {}
    prev_end, prev_name = None, "start"
    for d in order:
        name, v, t0, t1 = rows[d]
        ctx = prev_name if prev_end is None or t0 - prev_end < 1_000_000 else "idle"
        if (not a.kernel or any(k in name for k in a.kernel)) and t1 > t0:
            key = short(name) + (" after " + short(ctx) if a.context else "")
            out.setdefault(key, []).append(v / 8 / (t1 - t0))
        if "rs_sets_prep" not in name:  # (the share-set pass's own prep is not its context)
            prev_end, prev_name = t1, name
    print(json.dumps({k: {"ghz_median": round(statistics.median(x), 3), "n": len(x)} for k, x in sorted(out.items())}))


if __name__ == "__main__":
    main()
