#!/usr/bin/env python3
"""Summarise the SQ counter passes of tools/prof_round.sh (rocprofv3 --pmc
... --kernel-trace CSVs) into per-kernel medians and the ratios DESIGN.md
quotes: wave-cycle shares (waiting, VALU active, issue-stalled), SALU:VALU,
LDS bank conflicts.
  python tools/pmc_sq_summary.py gpurun_out/r02/final/pmc_sq out.json"""
import csv
import glob
import json
import re
import statistics
import sys
from collections import defaultdict


def load(files):
    v = defaultdict(lambda: defaultdict(list))
    for f in files:
        acc, nm = defaultdict(float), {}
        for r in csv.DictReader(open(f)):
            acc[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            nm[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (dsp, c), x in acc.items():
            v[nm[dsp]][c].append(x)
    return v


def main(src, out):
    res = {"source": f"rocprofv3 SQ counter passes ({src}), median over dispatches; tools/pmc_sq_summary.py"}
    for k, c in sorted(load(glob.glob(f"{src}/**/*counter_collection.csv", recursive=True)).items()):
        m = re.search(r"(rs_\w+<[^>]*>|rs_\w+)", k)
        if not m or "targets" in k:
            continue
        med = {n: statistics.median(x) for n, x in c.items()}
        e = {"dispatches": max(len(x) for x in c.values()), "counters": med}
        if "SQ_WAVE_CYCLES" in med and "SQ_WAIT_ANY" in med:
            e["wait_share"] = round(med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"], 3)
            e["valu_active_share"] = round(med["SQ_ACTIVE_INST_VALU"] / med["SQ_WAVE_CYCLES"], 3)
            e["issue_stall_share"] = round(med["SQ_WAIT_INST_ANY"] / med["SQ_WAVE_CYCLES"], 3)
        if "SQ_INSTS_SALU" in med:
            e["salu_per_valu"] = round(med["SQ_INSTS_SALU"] / med["SQ_INSTS_VALU"], 3)
            e["lds_bank_conflicts"] = med["SQ_LDS_BANK_CONFLICT"]
        res[m.group(1)] = e
    json.dump(res, open(out, "w"), indent=1)
    for k, e in res.items():
        if isinstance(e, dict):
            print(k, {x: e[x] for x in e if x not in ("counters",)})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
