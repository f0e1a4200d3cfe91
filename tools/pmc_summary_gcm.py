#!/usr/bin/env python3
"""Summarise a rocprofv3 counter CSV per kernel (developer tool): average of
each counter over dispatches, effective clock, VALU/LDS activity fractions."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].split("(")[0][-60:]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in agg.items():
    a = {c: sum(x) / len(x) for c, x in v.items()}
    t = sum(dur[k]) / len(dur[k]) * 1e-9
    line = f"{k}: t={t * 1e6:.0f}us"
    if "GRBM_GUI_ACTIVE" in a and t > 0:
        clk = a["GRBM_GUI_ACTIVE"] / 8 / t
        line += f" clk={clk / 1e9:.2f}GHz"
        simd_cyc = 1024 * clk * t
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if c in a:
                line += f" {c[15:]}={a[c] * 4 / simd_cyc:.2f}"
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"):
        if c in a:
            line += f" {c}={a[c]:.3g}"
    print(line)
