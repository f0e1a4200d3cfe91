#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps between consecutive dispatches from a
rocprofv3 --kernel-trace CSV (tools/gpu_round.sh `trace` step):
  python tools/trace_gaps.py gpurun_out/<dir>/trace/run_kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    n = re.sub(r"\(.*", "", n.replace("void ", "").replace("uplink_ec::", "").replace("(anonymous namespace)::", ""))
    return n.replace("enc::", "")[:44]


seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
stats = collections.defaultdict(list)
for n, s, e in seq:
    stats[n].append((e - s) / 1000)
print(f"{'kernel':44s} {'n':>6s} {'median us':>10s} {'mean us':>10s}")
for k, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{k:44s} {len(v):6d} {v[len(v) // 2]:10.1f} {sum(v) / len(v):10.1f}")
gaps = collections.defaultdict(list)
for i in range(1, len(seq)):
    gaps[(seq[i - 1][0], seq[i][0])].append((seq[i][1] - seq[i - 1][2]) / 1000)
print("\nidle gap between consecutive dispatches (us), pairs seen > 20 times:")
for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
    if len(v) > 20:
        v.sort()
        print(f"  {k[0]:44s} -> {k[1]:44s} n={len(v):5d} median {v[len(v) // 2]:7.1f}")
